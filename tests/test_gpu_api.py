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
