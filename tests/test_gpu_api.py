"""The drop-in ape_lz4.h one-shot calls on a real MI355X (host buffers in and out,
pinned staging + H2D/D2H inside the library), plus the host-buffer batch API and the
device-side benchmark generator.  One-shot calls run the host codec by default (SURVEY
8(b)); the tests of the GPU one-shot path select it with the `gpu_oneshot` fixture.
"""
import base64
import ctypes as C
import random

import pytest

from lz4util import I, buf, orc_compress, orc_decompress, sha

pytestmark = pytest.mark.gpu


@pytest.fixture
def gpu_oneshot(product):
    """Every one-shot call on the GPU path for the test (threshold 0), default after."""
    with product.oneshot_on_gpu():
        yield


def test_one_shot_decompress_matches_reference_kats(cuda, product, golden, gpu_oneshot):
    for d in golden["decode"][::3]:
        comp = base64.b64decode(d["comp_b64"])
        r, out = product.decompress_safe(comp, d["cap"])
        assert r == d["ret"], d["name"]
        if r > 0 and not d["has_offset0"]:
            assert sha(out) == d["out_sha256"]
        pr, pout = product.decompress_safe_partial(comp, d["partial"]["target"], d["cap"])
        assert pr == d["partial"]["ret"], d["name"]


def test_one_shot_compress_roundtrip(cuda, product, oracle, gpu_oneshot):
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


def test_concurrent_one_shot_callers(cuda, product, oracle, gpu_oneshot):
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
    """One-call latency of the one-shot calls, by default (host codec) and on
    the GPU path (threshold 0), next to the reference algorithm on one host core (the oracle
    restatement, as the checker's clock): printed for DESIGN.md section 1; the default must
    be no slower than the host core and return the same bytes."""
    import time
    L = product.lib()

    def clock(fn, reps=20, runs=5):
        """median over `runs` of the mean of `reps` calls (one scheduler hiccup moves one run)"""
        for _ in range(3):
            fn()
        ts = []
        for _ in range(runs):
            t0 = time.perf_counter()
            for _ in range(reps):
                r = fn()
            ts.append((time.perf_counter() - t0) / reps)
        return sorted(ts)[runs // 2], r

    for n in (1024, 8192, 65536):
        s = I.make("comp", n, seed=5)
        bound = product.compressBound(n)
        b = buf(s)
        o = C.create_string_buffer(bound + 64)
        dt, r = clock(lambda: L.APE_LZ4_compress_default(b, o, n, bound))
        comp = o.raw[:r]
        er, ecomp = orc_compress(oracle, s)
        assert r == er and comp == ecomp           # the host codec = the reference's bytes
        cb = buf(comp)
        d = C.create_string_buffer(n + 64)
        dd, r2 = clock(lambda: L.APE_LZ4_decompress_safe(cb, d, r, n))
        assert r2 == n and d.raw[:n] == s
        with product.oneshot_on_gpu():
            gdt, gr = clock(lambda: L.APE_LZ4_compress_default(b, o, n, bound))
            assert gr > 0
            gcb = buf(o.raw[:gr])
            gdd, gr2 = clock(lambda: L.APE_LZ4_decompress_safe(gcb, d, gr, n))
            assert gr2 == n and d.raw[:n] == s
        # one host core, the restatement called with preallocated buffers
        ob = C.create_string_buffer(bound + 64)
        hc, _ = clock(lambda: oracle.orc_compress_default(b, ob, n, bound))
        hd, _ = clock(lambda: oracle.orc_decompress_safe(cb, d, r, n))
        print("one-shot n=%d: default (host codec) compress %.1f us, decompress %.1f us | GPU "
              "path compress %.1f us, decompress %.1f us | one host core (reference algorithm): "
              "compress %.1f us, decompress %.1f us" % (
                  n, dt * 1e6, dd * 1e6, gdt * 1e6, gdd * 1e6, hc * 1e6, hd * 1e6))
        # the default path is the host codec, not a GPU round trip: same order as one host
        # core (a loose bound on a shared host; the byte equality above is the hard check)
        assert dt <= 2.0 * hc + 20e-6 and dd <= 2.0 * hd + 20e-6
        assert gdt < 0.5 and gdd < 0.5


def test_host_batch_decode_huge_caps(cuda, product, golden, oracle):
    """host-buffer batch decode stages at most min(cap, 255 csize + 64) bytes per
    block while the kernel sees the caller's cap; with caps far above what a block can
    expand to, valid, mutated and truncated blocks return exactly the oracle's results."""
    import base64
    L = product.lib()
    rng = random.Random(11)
    blobs = [base64.b64decode(d["comp_b64"]) for d in golden["decode"]][:40]
    for i in range(20):
        _, c = orc_compress(oracle, I.make("comp", rng.randrange(1, 4000), seed=i))
        c = bytearray(c)
        if i % 2:
            c[rng.randrange(len(c))] = rng.randrange(256)
        blobs.append(bytes(c[:rng.randrange(1, len(c) + 1)] if i % 3 == 0 else c))
    cap = (1 << 20) + 3
    nb = len(blobs)
    keep = [buf(b) for b in blobs]
    outs = [C.create_string_buffer(cap + 64) for _ in blobs]
    res = (C.c_int * nb)()
    rc = L.APE_LZ4_decompress_safe_batch_host(
        (C.c_void_p * nb)(*[C.addressof(k) for k in keep]), (C.c_int * nb)(*map(len, blobs)),
        (C.c_void_p * nb)(*[C.addressof(o) for o in outs]), (C.c_int * nb)(*([cap] * nb)), res, nb)
    assert rc == 0
    for i, b in enumerate(blobs):
        er, eout = orc_decompress(oracle, b, cap)
        assert res[i] == er, i
        if er > 0 and not (i < 40 and golden["decode"][i]["has_offset0"]):
            assert outs[i].raw[:er] == eout, i
