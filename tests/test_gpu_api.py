"""The drop-in ape_lz4.h one-shot calls on a real MI355X (host buffers in and out,
pinned staging + H2D/D2H inside the library), plus the host-buffer batch API and the
device-side benchmark generator.
"""
import base64
import ctypes as C
import random

import pytest

from lz4util import I, buf, orc_compress, orc_decompress, sha

pytestmark = pytest.mark.gpu


def test_one_shot_decompress_matches_reference_kats(cuda, product, golden):
    for d in golden["decode"][::3]:
        comp = base64.b64decode(d["comp_b64"])
        r, out = product.decompress_safe(comp, d["cap"])
        assert r == d["ret"], d["name"]
        if r > 0 and not d["has_offset0"]:
            assert sha(out) == d["out_sha256"]
        pr, pout = product.decompress_safe_partial(comp, d["partial"]["target"], d["cap"])
        assert pr == d["partial"]["ret"], d["name"]


def test_one_shot_compress_roundtrip(cuda, product, oracle):
    rng = random.Random(3)
    L = product.lib()
    for i in range(40):
        src = I.make(rng.choice(["comp", "text", "rand", "zeros"]), rng.randrange(0, 65537), seed=i)
        r, comp = product.compress_default(src)
        assert 0 < r <= product.compressBound(len(src))
        er, out = orc_decompress(oracle, comp, len(src))
        assert er == len(src) and out == src
        r2, out2 = product.decompress_safe(comp, len(src))
        assert r2 == len(src) and out2 == src
        # obsolete aliases route to the same codec
        o = C.create_string_buffer(product.compressBound(len(src)) + 16)
        assert L.APE_LZ4_compress(buf(src), o, len(src)) == r
        st = C.create_string_buffer(16416)
        assert L.APE_LZ4_compress_withState(st, buf(src), o, len(src)) == r
        assert L.APE_LZ4_compress_fast_extState(st, buf(src), o, len(src), len(comp), 1) == r
        # acceleration > 1 trades ratio for speed (ref :789-808): still a valid block
        fo = C.create_string_buffer(product.compressBound(len(src)) + 16)
        fr = L.APE_LZ4_compress_fast_extState(st, buf(src), fo, len(src),
                                              product.compressBound(len(src)), 5)
        assert fr > 0 and orc_decompress(oracle, fo.raw[:fr], len(src)) == (len(src), src)
        if r > 1:
            assert L.APE_LZ4_compress_limitedOutput(buf(src), o, len(src), r - 1) == 0


def test_host_batch_api(cuda, product, oracle):
    L = product.lib()
    srcs = [I.synth_comp(65536, b) for b in range(6)] + [I.text(3000), b"", I.synth_rand(4096, 2)]
    nb = len(srcs)
    keep = [buf(s) for s in srcs]
    src_p = (C.c_void_p * nb)(*[C.addressof(k) for k in keep])
    caps = [product.compressBound(len(s)) for s in srcs]
    outs = [C.create_string_buffer(c + 16) for c in caps]
    dst_p = (C.c_void_p * nb)(*[C.addressof(o) for o in outs])
    res = (C.c_int * nb)()
    rc = L.APE_LZ4_compress_batch_host(src_p, (C.c_int * nb)(*map(len, srcs)), dst_p,
                                       (C.c_int * nb)(*caps), res, nb)
    assert rc == 0
    comps = [outs[i].raw[:res[i]] for i in range(nb)]
    for s, c in zip(srcs, comps):
        er, out = orc_decompress(oracle, c, len(s))
        assert er == len(s) and out == s
    # and back through the host-buffer decode batch
    keep2 = [buf(c) for c in comps]
    csrc = (C.c_void_p * nb)(*[C.addressof(k) for k in keep2])
    douts = [C.create_string_buffer(len(s) + 16) for s in srcs]
    ddst = (C.c_void_p * nb)(*[C.addressof(o) for o in douts])
    dres = (C.c_int * nb)()
    rc = L.APE_LZ4_decompress_safe_batch_host(csrc, (C.c_int * nb)(*map(len, comps)), ddst,
                                              (C.c_int * nb)(*map(len, srcs)), dres, nb)
    assert rc == 0
    assert list(dres) == [len(s) for s in srcs]
    assert [douts[i].raw[:len(srcs[i])] for i in range(nb)] == srcs


def test_device_generator_matches_spec(cuda, product, oracle):
    torch = cuda
    for kind, fn, n in ((1, I.synth_comp, 65536), (0, I.synth_rand, 4096), (1, I.synth_comp, 4096)):
        t = torch.zeros((5, n + 48), dtype=torch.uint8, device="cuda")
        product.synth_blocks(t, n, 1000, kind)
        torch.cuda.synchronize()
        h = t.cpu().numpy()
        for b in range(5):
            assert h[b, :n].tobytes() == fn(n, 1000 + b)


def test_concurrent_one_shot_callers(cuda, product, oracle):
    """SURVEY 8(b) threading: the shim is thread-safe per call.  8 threads issue one-shot
    compress_default / decompress_safe / decompress_safe_partial calls at once (ctypes drops
    the GIL around each call); every result must equal the single-threaded one."""
    import threading
    L = product.lib()
    srcs = [I.make(c, n, seed=n + k) for k, (c, n) in enumerate(
        [("comp", 65536), ("text", 30000), ("rand", 4096), ("zeros", 65536), ("comp", 1000),
         ("period7", 20000), ("comp", 65537), ("text", 200000)])]
    expect = []
    for s in srcs:
        r, comp = product.compress_default(s)
        assert r > 0 and orc_decompress(oracle, comp, len(s)) == (len(s), s)
        expect.append(comp)
    errors = []

    def worker(t):
        try:
            for it in range(12):
                i = (t + it) % len(srcs)
                s = srcs[i]
                o = C.create_string_buffer(product.compressBound(len(s)) + 64)
                r = L.APE_LZ4_compress_default(buf(s), o, len(s), product.compressBound(len(s)))
                if o.raw[:r] != expect[i]:
                    errors.append(("compress", t, i, r))
                d = C.create_string_buffer(len(s) + 64)
                r2 = L.APE_LZ4_decompress_safe(buf(expect[i]), d, len(expect[i]), len(s))
                if r2 != len(s) or d.raw[:len(s)] != s:
                    errors.append(("decompress", t, i, r2))
                p = C.create_string_buffer(len(s) + 64)
                r3 = L.APE_LZ4_decompress_safe_partial(buf(expect[i]), p, len(expect[i]),
                                                       len(s) // 2, len(s))
                if r3 < len(s) // 2 or p.raw[:len(s) // 2] != s[:len(s) // 2]:
                    errors.append(("partial", t, i, r3))
        except Exception as e:   # pragma: no cover
            errors.append(("exception", t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]


def test_one_shot_latency_recorded(cuda, product, oracle):
    """One-call latency of the GPU one-shot path next to the reference algorithm on one
    host core (the oracle restatement, as the checker's clock), for the routing note in
    DESIGN.md: printed, and sanity-bounded only."""
    import time
    L = product.lib()
    for n in (1024, 8192, 65536):
        s = I.make("comp", n, seed=5)
        o = C.create_string_buffer(product.compressBound(n) + 64)
        b = buf(s)
        for _ in range(3):
            L.APE_LZ4_compress_default(b, o, n, product.compressBound(n))
        t0 = time.perf_counter()
        for _ in range(20):
            r = L.APE_LZ4_compress_default(b, o, n, product.compressBound(n))
        dt = (time.perf_counter() - t0) / 20
        d = C.create_string_buffer(n + 64)
        cb = buf(o.raw[:r])
        t0 = time.perf_counter()
        for _ in range(20):
            L.APE_LZ4_decompress_safe(cb, d, r, n)
        dd = (time.perf_counter() - t0) / 20
        t0 = time.perf_counter()
        for _ in range(20):
            orc_compress(oracle, s)
        hc = (time.perf_counter() - t0) / 20
        t0 = time.perf_counter()
        for _ in range(20):
            orc_decompress(oracle, o.raw[:r], n)
        hd = (time.perf_counter() - t0) / 20
        print("one-shot n=%d: GPU compress %.1f us, decompress %.1f us | one host core "
              "(reference algorithm): compress %.1f us, decompress %.1f us" % (
                  n, dt * 1e6, dd * 1e6, hc * 1e6, hd * 1e6))
        assert dt < 0.5 and dd < 0.5
