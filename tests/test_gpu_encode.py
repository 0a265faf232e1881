"""GPU encoder: emits valid LZ4 v1.7.1 blocks.

Bar (north_star): "a valid LZ4 block that the reference decompresses to the original
bytes" -- every GPU-compressed block is decoded by the reference ITSELF (oracle/_ref, the
reference src/ape_lz4.c compiled from its own source, when present: always on the GPU box)
and by the oracle restatement (pinned to the reference by tests/test_oracle_golden.py):
cap = srcSize restores the input exactly, cap = srcSize - 1 fails with the same return
code in both; the output never exceeds compressBound, limited-output semantics hold (0 when
it does not fit), output is deterministic, and the compression ratio on the benchmark data
is reported next to the reference's.
"""
import ctypes as C
import os
import random

import pytest

from gpuutil import alloc_out, fetch, ints, pack
from lz4util import I, buf, orc_compress, orc_decompress, ref_lib, walk_ok

pytestmark = pytest.mark.gpu


def run_encode(torch, amd, srcs, caps=None, in_mis=None, out_mis=None):
    caps = [amd.compressBound(len(s)) for s in srcs] if caps is None else caps
    src, sptr, _ = pack(torch, srcs, misalign=in_mis)
    dst, dptr, doffs = alloc_out(torch, caps, misalign=out_mis)
    res = ints(torch, [0] * len(srcs))
    # keep every tensor referenced until the kernel has run (raw pointers escape
    # torch's stream-ordered allocator)
    sizes, capt = ints(torch, map(len, srcs)), ints(torch, caps)
    rc = amd.lib().APE_LZ4_compress_batch_dev(
        sptr.data_ptr(), sizes.data_ptr(), dptr.data_ptr(), capt.data_ptr(), res.data_ptr(),
        len(srcs), None)
    assert rc == 0, amd.gpu_last_error()
    torch.cuda.synchronize()
    rs = res.cpu().tolist()
    return rs, [fetch(dst, o, r) for o, r in zip(doffs, rs)]


def ref_decode(ref, comp, cap):
    """APE_LZ4_decompress_safe of the reference library itself: (ret, dst[0:ret])."""
    o = C.create_string_buffer(max(cap, 0) + 64)
    r = ref.APE_LZ4_decompress_safe(buf(comp), o, len(comp), cap)
    return r, o.raw[:max(r, 0)]


def check_valid(oracle, src, comp):
    n = len(src)
    r, out = orc_decompress(oracle, comp, n)
    assert r == n, (n, r)
    assert out == src
    walk_ok(comp)  # parses as a well-formed sequence list
    ref = ref_lib()
    if ref is not None:   # the reference decoder itself (oracle/_ref)
        assert ref_decode(ref, comp, n) == (n, src), n
        if n > 0:         # one byte short: a decode error, the same one in both
            rr, _ = ref_decode(ref, comp, n - 1)
            assert rr < 0 and rr == orc_decompress(oracle, comp, n - 1)[0], (n, rr)


def test_encoder_output_decoded_by_reference_itself(cuda, product, oracle):
    """the config-3 sample (64 x 64 KiB App. C blocks) plus 4 KiB random
    and compressible blocks and the edge sizes, compressed on the GPU, decoded by the
    reference library itself (cap = n: the input; cap = n - 1: the same error as the
    oracle's)."""
    if ref_lib() is None:
        pytest.skip("oracle/_ref (the reference built from its own source) not present")
    srcs = [I.synth_comp(65536, b) for b in range(64)] + \
           [I.synth_rand(4096, b) for b in range(64)] + \
           [I.synth_comp(4096, b) for b in range(64)] + \
           [I.make(c, n, seed=n) for c in ("comp", "text", "zeros", "rand")
            for n in (0, 1, 12, 13, 14, 15, 16, 17, 100, 4095, 65535, 65536)]
    rs, comps = run_encode(cuda, product, srcs)
    ref = ref_lib()
    for s, r, c in zip(srcs, rs, comps):
        assert 0 < r <= product.compressBound(len(s))
        assert ref_decode(ref, c, len(s)) == (len(s), s), len(s)
        if len(s):
            rr, _ = ref_decode(ref, c, len(s) - 1)
            assert rr < 0 and rr == orc_decompress(oracle, c, len(s) - 1)[0]


def test_golden_inputs_roundtrip(cuda, product, oracle):
    srcs = []
    for content in I.ENC_CONTENTS:
        for n in I.ENC_SIZES:
            if n <= 65536:
                srcs.append(I.make(content, n))
    rs, comps = run_encode(cuda, product, srcs)
    for s, r, c in zip(srcs, rs, comps):
        assert 0 < r <= product.compressBound(len(s)), len(s)
        check_valid(oracle, s, c)


def test_benchmark_blocks_ratio_and_roundtrip(cuda, product, oracle):
    srcs = [I.synth_comp(65536, b) for b in range(64)] + \
           [I.synth_rand(4096, b) for b in range(64)] + \
           [I.synth_comp(4096, b) for b in range(64)]
    rs, comps = run_encode(cuda, product, srcs)
    ref = [orc_compress(oracle, s)[0] for s in srcs]
    for s, c in zip(srcs, comps):
        check_valid(oracle, s, c)
    gpu_ratio = 64 * 65536 / sum(rs[:64])
    ref_ratio = 64 * 65536 / sum(ref[:64])
    print("64 KiB compressible ratio: gpu %.4f reference %.4f" % (gpu_ratio, ref_ratio))
    assert gpu_ratio >= 0.99 * ref_ratio   # a 2 % regression must fail
    assert rs[64:128] == [4114] * 64  # incompressible: one literal run, as the reference
    # and the GPU decoder restores them too
    from test_gpu_decode import run_decode
    drs, outs = run_decode(cuda, product, comps, [len(s) for s in srcs])
    assert drs == [len(s) for s in srcs] and outs == srcs


def test_limited_output(cuda, product, oracle):
    srcs = [I.make(c, n, seed=n) for c in ("comp", "text", "rand") for n in (100, 5000, 65536)]
    rs, comps = run_encode(cuda, product, srcs)
    rs2, comps2 = run_encode(cuda, product, srcs, caps=rs)
    assert rs2 == rs and comps2 == comps
    rs3, _ = run_encode(cuda, product, srcs, caps=[r - 1 for r in rs])
    assert rs3 == [0] * len(srcs)


def test_deterministic(cuda, product):
    srcs = [I.synth_comp(65536, b) for b in range(16)] + [I.text(65536, 3)]
    a = run_encode(cuda, product, srcs)
    b = run_encode(cuda, product, srcs)
    assert a == b


def test_misaligned_and_random_sizes(cuda, product, oracle):
    rng = random.Random(9)
    srcs = [I.make(rng.choice(["comp", "text", "rand", "zeros", "period7"]),
                   rng.randrange(0, 65537), seed=i) for i in range(96)]
    rs, comps = run_encode(cuda, product, srcs, in_mis=[i % 16 for i in range(96)],
                           out_mis=[(3 * i) % 16 for i in range(96)])
    for s, c in zip(srcs, comps):
        check_valid(oracle, s, c)


def test_pathological_runs(cuda, product, oracle):
    """Long matches exercise the cooperative extension path."""
    srcs = [bytes(65536), b"\xab" * 65536, (b"xyz" * 30000)[:65536],
            bytes(1000) + I.synth_rand(2000, 1) + bytes(62536)]
    rs, comps = run_encode(cuda, product, srcs)
    for s, c in zip(srcs, comps):
        check_valid(oracle, s, c)
    assert rs[0] < 400 and rs[1] < 400


def _boundary_copies(n, seed, lens):
    """Random bytes, then back-copies whose lengths sit on the encoder's measurement edges
    (C1 measures T and L to 12 bytes, stage 2 adds 64: lengths 11-13, 75-77; and the edges of
    the earlier 16- and 20-byte T: 15-17, 19-21, 79-81, 83-86), each followed by one random
    byte so the match ends exactly there.  Inside such a copy consecutive lanes share the
    offset: stage 2 measures the run's last lane and the others derive their lengths."""
    rng = random.Random(seed)
    out = bytearray(rng.randbytes(2048))
    while len(out) < n:
        ln = rng.choice(lens)
        off = rng.randrange(1, min(len(out), 65535))
        for _ in range(ln):
            out.append(out[-off])
        out.append(rng.randrange(256))
    return bytes(out[:n])


def test_stage2_measurement_edges(cuda, product, oracle):
    """Matches ending exactly at the producer's measured lengths (C1's 12/20 bytes, stage 2's
    +64) and chunks where more than 16 lanes are truncated (a second stage-2 pass): valid
    output, and the ratio close to the reference's on the same data."""
    lens = [11, 12, 13, 15, 16, 17, 19, 20, 21, 75, 76, 77, 79, 80, 81, 83, 84, 85, 86]
    srcs = [_boundary_copies(65536, s, lens) for s in range(16)] + \
           [_boundary_copies(65536, 100 + s, [79, 80, 81, 83, 84, 85, 86, 150, 300])
            for s in range(8)] + \
           [_boundary_copies(n, 200 + n, lens) for n in (150, 300, 1000, 4099, 65535)]
    rs, comps = run_encode(cuda, product, srcs)
    for s, r, c in zip(srcs, rs, comps):
        assert 0 < r <= product.compressBound(len(s)), len(s)
        check_valid(oracle, s, c)
    ours = sum(rs[:24])
    ref = sum(orc_compress(oracle, s)[0] for s in srcs[:24])
    # Copies of copies from uniform random offsets: here the reference's policy (walked
    # positions only, so the table keeps the original of a string a later short copy repeats)
    # beats the GPU's every-position table (the latest occurrence), measured +4.5 % at round 6
    # (the round-5 policy passed <= 1.03).  A stage-2 length cut short would cost far more.
    assert ours <= ref * 1.06, (ours, ref)


def test_odd_chunk_counts_and_tail_emission(cuda, product, oracle):
    """Blocks of 1..64 KiB at every residue of the 64-position chunk grid, odd and even chunk
    counts (the encoder's steps past the last chunk differ by parity), mixed content so the
    emitter has records pending at the end: every block valid and decoded by the oracle.  (A
    round-6 record-count bug in the last steps of odd-chunk blocks hung the GPU encoder fuzz;
    the pytest sizes had not reached it.)"""
    rng = random.Random(61)
    kinds = ["comp", "text", "period7", "rand"]
    sizes = [64 * c + r for c in (1, 2, 3, 5, 15, 16, 17, 63, 101, 255, 511, 1023)
             for r in (0, 1, 13, 37, 63)] + [rng.randrange(1, 65537) for _ in range(196)]
    srcs = []
    for i, n in enumerate(sizes):
        out = bytearray()
        while len(out) < n:
            out += I.make(kinds[(i + len(out)) % 4], min(n - len(out), rng.randrange(64, 4096)),
                          seed=rng.randrange(1 << 20))
        srcs.append(bytes(out[:n]))
    rs, comps = run_encode(cuda, product, srcs)
    for s, r, c in zip(srcs, rs, comps):
        assert 0 < r <= product.compressBound(len(s)), len(s)
        check_valid(oracle, s, c)


def test_block_limit(cuda, product):
    rs, _ = run_encode(cuda, product, [bytes(65537)])
    assert rs == [product.ERANGE]


ACCEL_RATIO_TOL = 0.01   # GPU >= (1 - tol) x reference at acceleration 1, 2, 4, 8


def test_acceleration(cuda, product, oracle):
    """compress_fast with acceleration > 1 (ref src/ape_lz4.c:789-808, step = searchMatchNb
    >> 6 from acceleration << 6, :597-600): valid blocks at a ratio that falls as the
    acceleration grows (the search probes every acceleration-th position after a match);
    acceleration <= 1 is compress_default's output byte for byte."""
    srcs = [I.synth_comp(65536, b) for b in range(32)] + \
           [I.make(c, n, seed=n) for c in ("text", "zeros", "rand", "period3")
            for n in (0, 13, 100, 4096, 65536)]
    src, sptr, _ = pack(cuda, srcs)
    caps = [product.compressBound(len(s)) for s in srcs]
    out = {}
    for accel in (1, 2, 4, 8, 1 << 30):
        dst, dptr, doffs = alloc_out(cuda, caps)
        res = ints(cuda, [0] * len(srcs))
        sizes, capt = ints(cuda, map(len, srcs)), ints(cuda, caps)
        product.compress_fast_ptr_batch(sptr, sizes, dptr, capt, res, accel)
        cuda.cuda.synchronize()
        rs = res.cpu().tolist()
        out[accel] = (rs, [fetch(dst, o, r) for o, r in zip(doffs, rs)])
        for s, c in zip(srcs, out[accel][1]):
            check_valid(oracle, s, c)
    rs1, comps1 = run_encode(cuda, product, srcs)
    assert out[1][1] == comps1
    ratio = {a: 32 * 65536 / sum(out[a][0][:32]) for a in out}
    # the reference's compress_fast on the same blocks (its probe pattern, step growth after
    # 64 misses included, is what the GPU walker follows: VERDICT r3 item 8)
    ref = {a: 32 * 65536 / sum(orc_compress(oracle, s, accel=a)[0] for s in srcs[:32])
           for a in (1, 2, 4, 8)}
    print("ratio by acceleration", {a: round(r, 4) for a, r in ratio.items()},
          "reference", {a: round(r, 4) for a, r in ref.items()})
    assert ratio[1] >= ratio[2] > ratio[4] > ratio[8] > ratio[1 << 30]
    # one-sided: the GPU's 6-byte key and near candidate compress App. C data better than
    # the reference's search (round 6: +7 % at a = 1); a ratio 1 % below the reference's fails
    for a in (1, 2, 4, 8):
        assert ratio[a] >= (1.0 - ACCEL_RATIO_TOL) * ref[a], (a, ratio[a], ref[a])
    # a huge acceleration probes only the three positions after each match end (and the
    # block's first three): little is found, but the blocks stay valid (checked above)
    assert ratio[1 << 30] < 1.5
    # the one-shot API routes acceleration too: the GPU path gives the batch's bytes, the
    # default (host codec) the reference's own
    with product.oneshot_on_gpu():
        r, c = product.compress_fast(srcs[0], acceleration=4)
    assert c == out[4][1][0]
    assert product.compress_fast(srcs[0], acceleration=4) == orc_compress(oracle, srcs[0], accel=4)


def test_destsize(cuda, product, oracle):
    """compress_destSize batched on the GPU (ref src/ape_lz4.c:843-1067): the output fits
    the target, decodes (oracle decompress_safe, cap = consumed) to exactly the consumed
    prefix, is compress_default's output when the block fits, and consumes about as much
    input as the reference's greedy cut (reported; aggregate >= 95 % of it for targets of
    at least 1000 bytes)."""
    import ctypes as C

    from lz4util import buf

    base = [I.synth_comp(65536, b) for b in range(6)] + \
           [I.make(c, n, seed=n) for c in ("text", "zeros", "rand", "period3")
            for n in (0, 1, 13, 100, 4096, 65536)]
    full_rs, full = run_encode(cuda, product, base)
    srcs, tgts = [], []
    for s, c in zip(base, full_rs):
        for t in (0, 1, 2, 10, 16, 17, 100, 1000, 5000, 20000, c - 1, c, c + 7,
                  product.compressBound(len(s))):
            srcs.append(s)
            tgts.append(t)
    src, sptr, _ = pack(cuda, srcs)
    dst, dptr, doffs = alloc_out(cuda, [max(t, 0) for t in tgts])
    sizes, tg = ints(cuda, map(len, srcs)), ints(cuda, tgts)
    res = ints(cuda, [-7] * len(srcs))
    product.compress_destSize_ptr_batch(sptr, sizes, dptr, tg, res)
    cuda.cuda.synchronize()
    rs, cons = res.cpu().tolist(), sizes.cpu().tolist()
    gpu_sum = ref_sum = 0
    full_by = {id(s): f for s, f in zip(base, full)}
    for i, (s, t) in enumerate(zip(srcs, tgts)):
        r, k = rs[i], cons[i]
        if t < 1:
            assert r == 0 and k == len(s), (i, t, r, k)
            continue
        assert 1 <= r <= t and 0 <= k <= len(s), (i, len(s), t, r, k)
        comp = fetch(dst, doffs[i], r)
        dr, out = orc_decompress(oracle, comp, k)
        assert dr == k and out == s[:k], (i, len(s), t, r, k, dr)
        walk_ok(comp)
        if t >= len(full_by[id(s)]):
            assert k == len(s) and comp == full_by[id(s)], (i, t)
        rsz = C.c_int(len(s))
        rd = C.create_string_buffer(t + 64)
        rr = oracle.orc_compress_destSize(buf(s), rd, C.byref(rsz), t)
        assert rr > 0
        if t >= 1000:
            gpu_sum += k
            ref_sum += rsz.value
    print("destSize consumed: GPU %d vs reference %d (%.4f)" % (gpu_sum, ref_sum,
                                                               gpu_sum / ref_sum))
    assert gpu_sum >= 0.95 * ref_sum


@pytest.mark.gpu
def test_destSize_scratch_form_matches_and_captures(cuda, product, oracle):
    """APE_LZ4_compress_destSize_batch_scratch_dev (caller-owned scratch, no allocation):
    the same results as the allocating form, with one-block scratch (a pass per block)
    and inside a captured HIP graph replayed twice."""
    srcs = [I.synth_comp(65536, b) for b in range(5)] + [I.make("text", 4096, seed=3)]
    tgts = [20000, 1000, 30000, 5000, 17, 600]
    src, sptr, _ = pack(cuda, srcs)
    tg = ints(cuda, tgts)

    def run(mode):
        dst, dptr, doffs = alloc_out(cuda, tgts)
        sizes = ints(cuda, map(len, srcs))
        res = ints(cuda, [-7] * len(srcs))
        if mode == "alloc":
            product.compress_destSize_ptr_batch(sptr, sizes, dptr, tg, res)
        else:
            nb = 1 if mode == "one" else len(srcs)
            scr = cuda.empty(product.destSize_scratch_size(nb), dtype=cuda.uint8, device="cuda")
            if mode == "graph":
                s = cuda.cuda.Stream()
                s.wait_stream(cuda.cuda.current_stream())
                g = cuda.cuda.CUDAGraph()
                sz0 = sizes.clone()
                with cuda.cuda.graph(g, stream=s):
                    product.compress_destSize_scratch_ptr_batch(sptr, sizes, dptr, tg, res, scr,
                                                                stream=s)
                for _ in range(2):
                    sizes.copy_(sz0)
                    g.replay()
            else:
                product.compress_destSize_scratch_ptr_batch(sptr, sizes, dptr, tg, res, scr)
        cuda.cuda.synchronize()
        rs, ks = res.cpu().tolist(), sizes.cpu().tolist()
        return rs, ks, [fetch(dst, o, max(r, 0)) for o, r in zip(doffs, rs)]

    ref = run("alloc")
    for mode in ("one", "all", "graph"):
        assert run(mode) == ref, mode
    for s, r, k, c in zip(srcs, *ref):
        assert r > 0
        dr, out = orc_decompress(oracle, c, k)
        assert dr == k and out == s[:k]


def _mixed_runs(n, seed):
    """Blocks whose sequences mix every emitter path: short literal runs and matches (the
    staged batch), literal runs longer than 16 bytes and match-length extensions of 3+
    bytes (written straight to dst), in random order, so that batches start and end at
    every alignment."""
    rng = random.Random(seed)
    out = bytearray(rng.randbytes(64))
    while len(out) < n:
        k = rng.random()
        if k < 0.15:
            out += rng.randbytes(rng.randrange(17, 300))           # long literal run
        elif k < 0.2:
            off = rng.randrange(1, min(len(out), 65535))
            for _ in range(rng.randrange(530, 2000)):                # long match
                out.append(out[-off])
        elif k < 0.6:
            out += rng.randbytes(rng.randrange(0, 16))
            off = rng.randrange(1, min(len(out), 65535))
            for _ in range(rng.randrange(4, 40)):
                out.append(out[-off])
        else:
            out.append(rng.randrange(256))
    return bytes(out[:n])


def test_emitter_batches_mixed(cuda, product, oracle):
    """The batched emitter (staging buffer carried across batches, big records written
    straight to dst, the partial chunk after them) on mixed sequences, aligned and
    misaligned dst, and caps at the exact size and one below."""
    srcs = [_mixed_runs(n, s) for s, n in enumerate([65536] * 12 + [300, 1000, 4097, 20000, 65535])]
    for mis in (None, [(7 * i) % 16 for i in range(len(srcs))]):
        rs, comps = run_encode(cuda, product, srcs, out_mis=mis)
        for s, r, c in zip(srcs, rs, comps):
            assert 0 < r <= product.compressBound(len(s))
            check_valid(oracle, s, c)
        rs2, comps2 = run_encode(cuda, product, srcs, caps=rs, out_mis=mis)
        assert rs2 == rs and comps2 == comps
        assert run_encode(cuda, product, srcs, caps=[r - 1 for r in rs], out_mis=mis)[0] == [0] * len(srcs)


def _start_echo_block(seed, n=65536):
    """Random bytes with a period-3 run at positions 1..11 (broken at 12) whose bytes from
    position 4 reappear at many interior positions.  Position 1 then sits in the table under
    the same 5 bytes as every echo, and its 4 bytes of backward context lie before the block:
    an interior step that took candidate 1 with the bytes of candidate 4 would measure a
    12-byte match where the true one from position 1 is 8 bytes long."""
    rng = random.Random(seed)
    b = bytearray(rng.randbytes(n))
    b[1:12] = (rng.randbytes(3) * 4)[:11]
    b[12] = b[9] ^ 0x5A
    e = bytes(b[4:17])
    for at in range(300 + seed % 64, n - 200, 997 + 13 * (seed % 7)):
        b[at:at + len(e)] = e
    return bytes(b)


def test_candidates_at_block_start(cuda, product, oracle):
    """Table entries for positions 1..3 (their backward context precedes the block) never
    corrupt a match found by an interior step: blocks that echo their first bytes many times
    round-trip through the oracle and the GPU decoder."""
    srcs = [_start_echo_block(s) for s in range(96)]
    rs, comps = run_encode(cuda, product, srcs)
    for s, r, c in zip(srcs, rs, comps):
        assert 0 < r <= product.compressBound(len(s))
        check_valid(oracle, s, c)


def test_many_blocks_gpu_roundtrip(cuda, product):
    """4096 x 64 KiB App. C blocks and 512 start-echo blocks: GPU encode, GPU decode, every
    byte compared (a rare bad match shows up at this sample size; the parity tests above
    decode smaller samples with the reference itself)."""
    import torch
    n, nb = 65536, 4096
    slot = (product.compressBound(n) + 15) // 16 * 16
    src = torch.empty((nb + 512, n), dtype=torch.uint8, device="cuda")
    product.synth_blocks(src[:nb], n, 7, 1)
    src[nb:] = torch.tensor(bytearray(b"".join(_start_echo_block(1000 + s) for s in range(512))),
                            dtype=torch.uint8).view(512, n).cuda()
    tot = nb + 512
    comp = torch.empty((tot, slot), dtype=torch.uint8, device="cuda")
    out = torch.empty((tot, n), dtype=torch.uint8, device="cuda")
    sizes = torch.full((tot,), n, dtype=torch.int32, device="cuda")
    csz = torch.zeros(tot, dtype=torch.int32, device="cuda")
    dres = torch.zeros(tot, dtype=torch.int32, device="cuda")
    product.compress_batch(src, sizes, comp, csz)
    product.decompress_batch(comp, csz, out, dres, dst_caps=sizes)
    torch.cuda.synchronize()
    bad = (dres != n).nonzero().flatten().tolist()
    assert not bad, bad[:8]
    same = (out == src).all(dim=1)
    assert bool(same.all()), (~same).nonzero().flatten().tolist()[:8]
