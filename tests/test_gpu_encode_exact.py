"""Greedy-exact GPU encode mode: APE_LZ4_compress_exact_batch_dev must
give LZ4_compress_generic's bytes and return value exactly (ref src/ape_lz4.c:530-755, via
compress_fast :789-808 / compress_fast_extState :758-786).

Checked against the golden encode KATs generated from the reference itself (default cap,
the limitedOutput caps and the accelerations they hold), against the oracle restatement and
the reference library itself (oracle/_ref, when present) on the benchmark blocks at random
caps, misaligned buffers, and accelerations including the reference's shift wrap."""
import ctypes as C
import random

import pytest

from gpuutil import alloc_out, fetch, ints, pack
from lz4util import I, blob_matches, buf, orc_compress, ref_lib, sha

pytestmark = pytest.mark.gpu


def run_exact(torch, amd, srcs, caps=None, accel=1, in_mis=None, out_mis=None):
    caps = [amd.compressBound(len(s)) for s in srcs] if caps is None else caps
    src, sptr, _ = pack(torch, srcs, misalign=in_mis)
    dst, dptr, doffs = alloc_out(torch, caps, misalign=out_mis)
    res = ints(torch, [-99] * len(srcs))
    sizes, capt = ints(torch, map(len, srcs)), ints(torch, caps)
    amd.compress_exact_ptr_batch(sptr, sizes, dptr, capt, res, accel)
    torch.cuda.synchronize()
    rs = res.cpu().tolist()
    return rs, [fetch(dst, o, r) for o, r in zip(doffs, rs)]


def ref_compress(src, cap, accel):
    """APE_LZ4_compress_fast of the reference library itself: (ret, dst[0:ret])."""
    ref = ref_lib()
    o = C.create_string_buffer(max(cap, 1) + 64)
    r = ref.APE_LZ4_compress_fast(buf(src), o, len(src), cap, accel)
    return r, o.raw[:max(r, 0)]


def test_exact_matches_golden_kats(cuda, product, golden):
    """Every encode KAT up to 64 KiB: compress_default bytes, the limitedOutput results and
    the acceleration results recorded from the reference."""
    kats = [e for e in golden["encode"] if e["n"] <= 65536]
    srcs = [I.make(e["content"], e["n"]) for e in kats]
    for s, e in zip(srcs, kats):
        assert I.sha(s) == e["in_sha256"]
    rs, comps = run_exact(cuda, product, srcs)
    for e, r, c in zip(kats, rs, comps):
        assert r == e["clen"] and blob_matches(e["comp"], c), (e["content"], e["n"], r)
    # limitedOutput: every recorded cap in one launch
    lim = [(s, l) for s, e in zip(srcs, kats) for l in e["limited"]]
    rs, comps = run_exact(cuda, product, [s for s, _ in lim], caps=[l["cap"] for _, l in lim])
    for (s, l), r, c in zip(lim, rs, comps):
        assert r == l["ret"] and sha(c) == l["sha256"], (len(s), l)
    # accelerations, one launch each
    accs = sorted({ac["accel"] for e in kats for ac in e["accel"]})
    for a in accs:
        sel = [(s, ac) for s, e in zip(srcs, kats) for ac in e["accel"] if ac["accel"] == a]
        rs, comps = run_exact(cuda, product, [s for s, _ in sel], accel=a)
        for (s, ac), r, c in zip(sel, rs, comps):
            assert r == ac["ret"] and sha(c) == ac["sha256"], (len(s), a)


def test_exact_benchmark_blocks_random_caps(cuda, product, oracle):
    """Config-3/config-2 shaped blocks (App. C), text and edge contents, misaligned in and
    out, at cap = compressBound, the exact size, one byte less and random caps below."""
    rng = random.Random(5)
    srcs = [I.synth_comp(65536, b) for b in range(24)] + \
           [I.synth_rand(4096, b) for b in range(8)] + \
           [I.synth_comp(4096, b) for b in range(8)] + \
           [I.make(c, rng.randrange(0, 65537), seed=k)
            for k, c in enumerate(["text", "zeros", "period7", "comp", "rand"] * 4)]
    exp = [orc_compress(oracle, s) for s in srcs]
    mis_in = [rng.randrange(16) for _ in srcs]
    mis_out = [rng.randrange(16) for _ in srcs]
    rs, comps = run_exact(cuda, product, srcs, in_mis=mis_in, out_mis=mis_out)
    assert rs == [r for r, _ in exp]
    assert comps == [c for _, c in exp]
    have_ref = ref_lib() is not None
    if have_ref:   # the reference library itself, not only its restatement
        for s, r, c in zip(srcs, rs, comps):
            assert ref_compress(s, product.compressBound(len(s)), 1) == (r, c)
    for caps in ([r for r, _ in exp],
                 [max(r - 1, 0) for r, _ in exp],
                 [rng.randrange(0, product.compressBound(len(s)) + 1) for s in srcs]):
        rs2, comps2 = run_exact(cuda, product, srcs, caps=caps, out_mis=mis_out)
        exp2 = [orc_compress(oracle, s, cap=k) for s, k in zip(srcs, caps)]
        assert rs2 == [r for r, _ in exp2], caps
        assert comps2 == [c for _, c in exp2]
        if have_ref:
            for s, k, r, c in zip(srcs, caps, rs2, comps2):
                assert ref_compress(s, k, 1) == (r, c)


@pytest.mark.parametrize("accel", [0, -3, 2, 3, 8, 65, 1 << 26, 1 << 30])
def test_exact_acceleration(cuda, product, oracle, accel):
    """compress_fast: acceleration < 1 is 1 (:762); the search step grows every 64 misses
    from acceleration << 6 (:597-600), in 32-bit arithmetic -- 1 << 26 and 1 << 30 wrap the
    shift to 0, which the reference turns into 64 probes of one position."""
    srcs = [I.synth_comp(65536, b) for b in range(8)] + [I.text(30000, 2), I.synth_rand(4096, 3)]
    rs, comps = run_exact(cuda, product, srcs, accel=accel)
    for s, r, c in zip(srcs, rs, comps):
        er, ec = orc_compress(oracle, s, accel=accel)
        assert (r, c) == (er, ec), (len(s), accel, r, er)


def test_exact_limits(cuda, product):
    """A block over the GPU limit: ERANGE; a negative cap: 0 (documented deviation)."""
    srcs = [bytes(65537), bytes(100), bytes(100)]
    rs, _ = run_exact(cuda, product, srcs, caps=[80000, -1, 0])
    assert rs == [product.ERANGE, 0, 0]
