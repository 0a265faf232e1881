"""GPU decoder parity: bit-exact with the reference decompress_safe / _partial.

The bar (tier contract): identical return value for every block -- including the
negative -(consumed)-1 codes of malformed streams -- and identical dst[0:ret].
Streams with a zero match offset are excluded from content comparison only (the
reference then copies uninitialised dst bytes).
"""
import base64
import random

import pytest

from gpuutil import alloc_out, fetch, ints, pack
from lz4util import I, orc_compress, orc_decompress, sha

pytestmark = pytest.mark.gpu


def run_decode(torch, amd, comps, caps, targets=None, in_mis=None, out_mis=None):
    src, sptr, _ = pack(torch, comps, misalign=in_mis)
    dst, dptr, doffs = alloc_out(torch, caps, misalign=out_mis)
    res = ints(torch, [0] * len(comps))
    if targets is None:
        amd.decompress_ptr_batch(sptr, ints(torch, map(len, comps)), dptr, ints(torch, caps), res)
    else:
        amd.decompress_partial_batch(sptr, ints(torch, map(len, comps)), dptr,
                                     ints(torch, targets), ints(torch, caps), res)
    torch.cuda.synchronize()
    rs = res.cpu().tolist()
    outs = [fetch(dst, o, r) for o, r in zip(doffs, rs)]
    return rs, outs


def test_golden_decode_kats(cuda, product, golden):
    cases = golden["decode"]
    comps = [base64.b64decode(d["comp_b64"]) for d in cases]
    caps = [d["cap"] for d in cases]
    rs, outs = run_decode(cuda, product, comps, caps)
    for d, r, out in zip(cases, rs, outs):
        assert r == d["ret"], d["name"]
        if r > 0 and not d["has_offset0"]:
            assert sha(out) == d["out_sha256"], d["name"]
    tg = [d["partial"]["target"] for d in cases]
    rs, outs = run_decode(cuda, product, comps, caps, targets=tg)
    for d, r, out in zip(cases, rs, outs):
        assert r == d["partial"]["ret"], d["name"]
        if r > 0 and not d["has_offset0"]:
            assert sha(out) == d["partial"]["out_sha256"], d["name"]


def test_roundtrip_reference_streams(cuda, product, oracle):
    """Blocks compressed by the reference encoder decode bit-exactly on the GPU."""
    srcs = []
    for content in ("comp", "rand", "text", "zeros", "period3", "period7"):
        for n in (65536, 4096, 8192, 1000, 13, 65535, 30000):
            srcs.append(I.make(content, n, seed=n))
    for b in range(24):
        srcs.append(I.synth_comp(65536, 1000 + b))
    comps = [orc_compress(oracle, s)[1] for s in srcs]
    for caps in ([len(s) for s in srcs], [max(len(s) - 1, 0) for s in srcs],
                 [len(s) + 17 for s in srcs]):
        rs, outs = run_decode(cuda, product, comps, caps)
        for s, c, cap, r, out in zip(srcs, comps, caps, rs, outs):
            er, eout = orc_decompress(oracle, c, cap)
            assert r == er, (len(s), cap)
            if r > 0:
                assert out == eout


def test_fuzz_malformed_vs_oracle(cuda, product, oracle):
    rng = random.Random(1234)
    comps, caps, tg = [], [], []
    for k in range(3000):
        content = rng.choice(["comp", "text", "rand", "period3", "zeros", "byte"])
        n = rng.choice([16, 64, 300, 1000, 4096, 8192, 20000, 65536])
        _, c = orc_compress(oracle, I.make(content, n, seed=k))
        c = bytearray(c)
        for _ in range(rng.randrange(0, 5)):
            if c:
                c[rng.randrange(len(c))] = rng.randrange(256)
        if rng.random() < 0.2:
            c = c[:rng.randrange(len(c) + 1)]
        comps.append(bytes(c))
        cap = max(0, rng.choice([n, n - 1, n + 40, rng.randrange(n + 1), 65536]))
        if rng.random() < 0.05:   # negative caps: oend < dest in the reference
            cap = rng.choice([-1, -2, -13, -rng.randrange(1, 1 << 20)])
        caps.append(cap)
        tg.append(rng.randrange(-5, n + 40))
    for targets in (None, tg):
        rs, outs = run_decode(cuda, product, comps, caps, targets=targets)
        bad = []
        for i, (c, cap, r, out) in enumerate(zip(comps, caps, rs, outs)):
            er, eout = orc_decompress(oracle, c, cap, None if targets is None else targets[i])
            if r != er or (r > 0 and out != eout and not _has_off0(c)):
                bad.append((i, len(c), cap, r, er))
        assert not bad, bad[:10]


def _has_off0(c):
    import gen_golden
    return gen_golden.has_offset0(c)


def _dense_block(rng, nseq, p_long_lit, p_long_ml, p_ext):
    """A valid LZ4 block written token by token (no compressor): mostly 3-6-byte sequences
    (0-2 literals, a short match), so a 64-byte parse window holds up to 21 members and the
    lifting's 16-member round and its exits at every lane are exercised; literal lengths >= 15
    and match lengths with two or more extension bytes (the scalar path) at random places; a
    16-byte literal tail keeps every match clear of the block-end rules."""
    out, c = bytearray(), bytearray()

    def ext(v):
        while v >= 255:
            c.append(255)
            v -= 255
        c.append(v)

    for _ in range(nseq):
        r = rng.random()
        lit = rng.randrange(15, 300) if r < p_long_lit else rng.choice((0, 0, 0, 1, 2, 3, 14))
        if not out and lit == 0:
            lit = 1
        r = rng.random()
        if r < p_long_ml:
            ml = rng.randrange(19 + 255, 19 + 600)      # two or more extension bytes
        elif r < p_long_ml + p_ext:
            ml = rng.randrange(19, 19 + 254)            # one extension byte
        else:
            ml = rng.randrange(4, 19)
        off = rng.randrange(1, min(len(out) + lit, 65535) + 1)
        c.append((min(lit, 15) << 4) | min(ml - 4, 15))
        if lit >= 15:
            ext(lit - 15)
        lits = bytes(rng.randrange(256) for _ in range(lit))
        c += lits
        out += lits
        c += off.to_bytes(2, "little")
        if ml - 4 >= 15:
            ext(ml - 4 - 15)
        for _ in range(ml):
            out.append(out[-off])
    tail = bytes(rng.randrange(256) for _ in range(16))
    c.append(min(len(tail), 15) << 4)
    ext(len(tail) - 15)
    c += tail
    out += tail
    return bytes(c), bytes(out)


def test_dense_sequences_vs_oracle(cuda, product, oracle):
    """Hand-built blocks of dense short sequences (up to 21 per 64-byte window), with complex
    tokens at random positions, then cut short or mutated: return value (including every
    -(ip)-1) and bytes bit-exact with the oracle, for decompress_safe and _safe_partial."""
    rng = random.Random(77)
    comps, caps, tg, whole = [], [], [], []
    for k in range(240):
        mix = [(0.0, 0.0, 0.0), (0.02, 0.01, 0.05), (0.1, 0.05, 0.2)][k % 3]
        c, out = _dense_block(rng, rng.choice((3, 40, 400, 1500)), *mix)
        c = bytearray(c)
        if k % 4 == 1:
            for _ in range(rng.randrange(1, 4)):
                c[rng.randrange(len(c))] = rng.randrange(256)
        elif k % 4 == 2:
            c = c[:rng.randrange(1, len(c) + 1)]
        comps.append(bytes(c))
        caps.append(rng.choice((len(out), len(out), len(out) - 1, len(out) + 7)))
        tg.append(rng.randrange(0, len(out) + 8))
        whole.append(len(out) if k % 4 in (0, 3) and caps[-1] >= len(out) else None)
    for targets in (None, tg):
        rs, outs = run_decode(cuda, product, comps, caps, targets=targets)
        bad = []
        for i, (c, cap, r, o) in enumerate(zip(comps, caps, rs, outs)):
            er, eo = orc_decompress(oracle, c, cap, None if targets is None else targets[i])
            if r != er or (r > 0 and o != eo[:er] and not _has_off0(c)):
                bad.append((i, len(c), cap, r, er))
        assert not bad, bad[:10]
        if targets is None:   # the generator's blocks are valid: whole ones decode in full
            assert all(r == n for r, n in zip(rs, whole) if n is not None)
            assert sum(n is not None for n in whole) >= 60


def test_misaligned_buffers(cuda, product, oracle):
    rng = random.Random(5)
    srcs = [I.make(rng.choice(["comp", "text", "rand"]), rng.randrange(1, 65537), seed=i)
            for i in range(64)]
    comps = [orc_compress(oracle, s)[1] for s in srcs]
    rs, outs = run_decode(cuda, product, comps, [len(s) for s in srcs],
                          in_mis=[i % 16 for i in range(64)], out_mis=[(i * 7) % 16 for i in range(64)])
    assert rs == [len(s) for s in srcs]
    assert outs == srcs


def test_tiny_streams_every_alignment(cuda, product, oracle):
    """Compressed blocks of 1-14 bytes (whole and cut short) at all 16 source alignments: the
    staging loads read only dwords that intersect the block (a dword outside it re-reads the
    one holding byte 0); return value and bytes bit-exact with the oracle."""
    streams = []
    for n in range(0, 10):
        c = orc_compress(oracle, bytes(range(65, 65 + n)))[1]
        streams += [c[:k] for k in range(1, len(c) + 1)]
    comps, caps = [], []
    for c in streams:
        for cap in (16, 9):
            comps.append(c)
            caps.append(cap)
    mis = [i % 16 for i in range(len(comps))]
    rs, outs = run_decode(cuda, product, comps, caps, in_mis=mis, out_mis=[(3 * i) % 16 for i in range(len(comps))])
    for c, cap, r, o in zip(comps, caps, rs, outs):
        er, eo = orc_decompress(oracle, c, cap)
        assert r == er, (c, cap, r, er)
        if er > 0:
            assert o == eo[:er]


def test_blocks_beyond_64k(cuda, product, oracle):
    """The decoder has no block-size limit (only the 64 KiB offset window)."""
    srcs = [I.make("text", 70000), I.make("comp", 40000), I.make("rand", 200000, seed=3),
            I.make("zeros", 300000), I.make("period7", 131072), I.make("comp", 1 << 20, seed=9)]
    comps = [orc_compress(oracle, s)[1] for s in srcs]
    caps = [len(s) for s in srcs]
    rs, outs = run_decode(cuda, product, comps, caps)
    assert rs == caps
    assert outs == srcs
    # and an undersized cap fails exactly like the reference
    rs, _ = run_decode(cuda, product, comps, [c - 1 for c in caps])
    assert rs == [orc_decompress(oracle, c, n - 1)[0] for c, n in zip(comps, caps)]


def test_strided_batch_benchmark_layout(cuda, product, oracle):
    """The layout bench.py uses: fixed-stride slots, caps from the stride."""
    torch = cuda
    nb, n = 64, 65536
    slot = (n + n // 255 + 16 + 15) // 16 * 16
    srcs = [I.synth_comp(n, b) for b in range(nb)]
    comp = torch.zeros((nb, slot), dtype=torch.uint8, device="cuda")
    csz = []
    for b, s in enumerate(srcs):
        r, c = orc_compress(oracle, s)
        comp[b, :r] = torch.frombuffer(bytearray(c), dtype=torch.uint8).cuda()
        csz.append(r)
    out = torch.zeros((nb, n), dtype=torch.uint8, device="cuda")
    res = ints(torch, [0] * nb)
    product.decompress_batch(comp, ints(torch, csz), out, res)
    torch.cuda.synchronize()
    assert res.cpu().tolist() == [n] * nb
    host = out.cpu().numpy()
    for b in range(nb):
        assert host[b].tobytes() == srcs[b]


def test_decompress_fast(cuda, product, oracle):
    """decompress_fast (ref src/ape_lz4.c:1489): consumed bytes and output identical to the
    oracle on valid blocks with the exact original size, and the same error code when the
    size is short (the reference then stops inside the stream)."""
    import ctypes as C
    from lz4util import buf
    srcs = [I.make(c, n, seed=n) for c in ("comp", "text", "zeros", "rand", "period3")
            for n in (13, 14, 100, 300, 4096, 65536)]
    srcs += [I.synth_comp(65536, b) for b in range(8)]
    comps = [orc_compress(oracle, s)[1] for s in srcs]
    # the GPU encoder's blocks too
    src_t, sptr, _ = pack(cuda, srcs)
    caps0 = [product.compressBound(len(s)) for s in srcs]
    dst0, dptr0, doffs0 = alloc_out(cuda, caps0)
    res0 = ints(cuda, [0] * len(srcs))
    sizes0, capt0 = ints(cuda, map(len, srcs)), ints(cuda, caps0)
    product.compress_fast_ptr_batch(sptr, sizes0, dptr0, capt0, res0, 1)
    cuda.cuda.synchronize()
    comps += [fetch(dst0, o, r) for o, r in zip(doffs0, res0.cpu().tolist())]
    plains = srcs + srcs
    cases = []   # (comp, original size)
    for c, s in zip(comps, plains):
        cases.append((c, len(s)))
        for k in (1, 3, 8, 13, 100):
            if len(s) - k >= 0:
                cases.append((c, len(s) - k))
    blobs = [c for c, _ in cases]
    ins, iptr, _ = pack(cuda, blobs)
    osz = [n for _, n in cases]
    dst, dptr, doffs = alloc_out(cuda, [max(n, 1) for n in osz])
    res = ints(cuda, [0] * len(cases))
    product.decompress_fast_ptr_batch(iptr, ints(cuda, [len(b) for b in blobs]), dptr,
                                      ints(cuda, osz), res)
    cuda.cuda.synchronize()
    rs = res.cpu().tolist()
    for i, (c, n) in enumerate(cases):
        o = C.create_string_buffer(max(n, 1) + 64)
        er = oracle.orc_decompress_fast(buf(c), o, n)
        assert rs[i] == er, (i, n, len(c), rs[i], er)
        if er > 0:
            assert fetch(dst, doffs[i], n) == o.raw[:n], i


def test_decompress_fast_golden(cuda, product, golden):
    """The reference's own decompress_fast results (tests/golden, originalSize = n, n - 1)."""
    cases = [d for d in golden["decode"] if "fast" in d]
    comps = [base64.b64decode(d["comp_b64"]) for d in cases]
    ins, iptr, _ = pack(cuda, comps)
    osz = [d["fast"]["osize"] for d in cases]
    dst, dptr, doffs = alloc_out(cuda, [max(n, 1) for n in osz])
    res = ints(cuda, [0] * len(cases))
    product.decompress_fast_ptr_batch(iptr, ints(cuda, [len(c) for c in comps]), dptr,
                                      ints(cuda, osz), res)
    cuda.cuda.synchronize()
    for i, (d, r) in enumerate(zip(cases, res.cpu().tolist())):
        assert r == d["fast"]["ret"], d["name"]
        if r > 0:
            assert I.sha(fetch(dst, doffs[i], osz[i])) == d["fast"]["out_sha256"], d["name"]


def test_decompress_fast_garbage_stays_in_bounds(cuda, product, oracle):
    """decompress_fast on mutated and random inputs: the reference reads on without a bound
    (undefined there); the batch must stay inside each source's readable bound and dst,
    and return either an error or at most the bound."""
    rng = random.Random(17)
    blobs, osz = [], []
    for k in range(600):
        n = rng.choice([16, 100, 1000, 4096, 65536])
        c = bytearray(orc_compress(oracle, I.make(rng.choice(["comp", "text", "zeros"]), n,
                                                  seed=k))[1])
        for _ in range(rng.randint(1, 6)):
            c[rng.randrange(len(c))] = rng.randrange(256)
        if rng.random() < 0.3:
            c = c[:rng.randrange(1, len(c) + 1)]
        blobs.append(bytes(c))
        osz.append(n + rng.choice([0, 0, -3, 7, 300]))
    for k in range(100):
        blobs.append(bytes(rng.randrange(256) for _ in range(rng.randrange(1, 600))))
        osz.append(rng.randrange(1, 5000))
    ins, iptr, _ = pack(cuda, blobs, extra=0)
    dst, dptr, doffs = alloc_out(cuda, osz)
    res = ints(cuda, [0] * len(blobs))
    product.decompress_fast_ptr_batch(iptr, ints(cuda, [len(b) for b in blobs]), dptr,
                                      ints(cuda, osz), res)
    cuda.cuda.synchronize()
    for b, r in zip(blobs, res.cpu().tolist()):
        assert r <= len(b)


def test_negative_capacity(cuda, product, oracle):
    """decompress_safe / _partial / _fast with a negative capacity: the
    reference fails the first sequence (oend < dest) and writes nothing; same code here,
    and the canary check proves nothing was written."""
    import ctypes as C
    from lz4util import buf
    srcs = [I.make(c, n, seed=n) for c in ("comp", "text", "rand", "zeros") for n in (13, 100, 4096, 65536)]
    comps = [orc_compress(oracle, s)[1] for s in srcs]
    comps += [b"\xf0" + b"\xff" * 40 + b"\x00", b"\x00", b"\x1f\x41\x01\x00"]
    caps = [-1, -5, -65536, -(1 << 30)]
    cases = [(c, cap) for c in comps for cap in caps]
    blobs = [c for c, _ in cases]
    cps = [cap for _, cap in cases]
    rs, _ = run_decode(cuda, product, blobs, cps)
    assert rs == [orc_decompress(oracle, c, cap)[0] for c, cap in cases]
    rs, _ = run_decode(cuda, product, blobs, cps, targets=[abs(cap) for cap in cps])
    assert rs == [orc_decompress(oracle, c, cap, abs(cap))[0] for c, cap in cases]
    ins, iptr, _ = pack(cuda, blobs)
    dst, dptr, doffs = alloc_out(cuda, [0] * len(cases))
    res = ints(cuda, [0] * len(cases))
    product.decompress_fast_ptr_batch(iptr, ints(cuda, [len(b) for b in blobs]), dptr,
                                      ints(cuda, cps), res)
    cuda.cuda.synchronize()
    exp = [oracle.orc_decompress_fast(buf(c), C.create_string_buffer(64), cap) for c, cap in cases]
    assert res.cpu().tolist() == exp


def _ref_lib():
    import ctypes as C
    import os
    p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                     "oracle", "_ref", "libape_lz4_ref.so")
    if not os.path.exists(p):
        pytest.skip("oracle/_ref (the reference built from its own source) not present")
    return C.CDLL(p)


@pytest.mark.parametrize("cfg", ["config3_comp64k", "config2_rand4k"])
def test_benchmark_blocks_vs_reference_itself(cuda, product, cfg):
    """decode reference-compressed benchmark blocks (BASELINE config 3:
    App. C gen_comp 64 KiB; config 2: gen_rand 4 KiB) on the GPU and compare the return
    value and bytes with the reference decoder itself (oracle/_ref, compiled from
    src/ape_lz4.c), at the exact cap and one byte short."""
    import ctypes as C
    from lz4util import buf
    ref = _ref_lib()
    torch = cuda
    n, kind, nb, first = ((65536, 1, 192, 1048576 - 96) if cfg == "config3_comp64k"
                          else (4096, 0, 512, 262144 - 256))
    t = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    product.synth_blocks(t, n, first, kind)
    torch.cuda.synchronize()
    host = t.cpu().numpy()
    bound = product.compressBound(n)
    comps = []
    for b in range(nb):
        o = C.create_string_buffer(bound + 64)
        r = ref.APE_LZ4_compress_default(buf(host[b].tobytes()), o, n, bound)
        assert r > 0
        comps.append(o.raw[:r])
    if kind == 0:
        assert {len(c) for c in comps} == {4114}
    for cap in (n, n - 1):
        rs, outs = run_decode(cuda, product, comps, [cap] * nb)
        for b, (c, r, out) in enumerate(zip(comps, rs, outs)):
            o = C.create_string_buffer(cap + 64)
            er = ref.APE_LZ4_decompress_safe(buf(c), o, len(c), cap)
            assert r == er, (b, cap, r, er)
            if er > 0:
                assert out == o.raw[:er] == host[b].tobytes()[:er], (b, cap)


def test_final_token_literal_run_ignores_bytes_past_src(cuda, product, oracle):
    """a token with literal length 15 as the last input byte (`[0xFF]`, csize 1).
    The reference reads one byte past src there (ref src/ape_lz4.c:1330-1337) and returns
    -(csize + 1) - 1 whatever it holds; the GPU decoder's staging masks everything beyond
    csize, so the byte that follows in memory (varied here) cannot matter either.  (Only a
    first token can be the last byte: after a sequence the safe checks leave >= 4 bytes.)"""
    cases = []
    for blob in (b"\xff", b"\xf0", b"\xf7", b"\x10a\xf0", b"\x10a\xff"):
        for after in (b"\x00", b"\xff", b"\x05" * 40):
            for cap in (1, 64, 4096):
                cases.append((blob, after, cap))
    stored = [b + a for b, a, _ in cases]
    ins, iptr, _ = pack(cuda, stored)
    sizes = ints(cuda, [len(b) for b, _, _ in cases])
    caps = [c for _, _, c in cases]
    for partial in (False, True):
        dst, dptr, _ = alloc_out(cuda, caps)
        res = ints(cuda, [0] * len(cases))
        if partial:
            product.decompress_partial_batch(iptr, sizes, dptr, ints(cuda, [10] * len(cases)),
                                             ints(cuda, caps), res)
        else:
            product.decompress_ptr_batch(iptr, sizes, dptr, ints(cuda, caps), res)
        cuda.cuda.synchronize()
        got = res.cpu().tolist()
        exp = [orc_decompress(oracle, b, cap, 10 if partial else None)[0] for b, _, cap in cases]
        assert got == exp, [(c[0], c[2], g, e) for c, g, e in zip(cases, got, exp) if g != e]
        assert all(g == -3 for (b, _, _), g in zip(cases, got) if len(b) == 1), got


def test_long_literal_runs_all_modes(cuda, product, oracle):
    """Round 5 parses a literal length with one extension byte (15..269) in the vector windows:
    blocks dominated by such runs (and some of 270+, two extension bytes: the scalar path), long
    enough to restage many times, so runs straddle every staging boundary (a run whose offset
    bytes lie past the staged input is complex).  decompress_safe at cap n / n - 1 / n + 7, cut
    short and mutated; _safe_partial at random targets; decompress_fast at n and n - 3; and the
    same blocks through usingDict with a history dictionary: results and bytes vs the oracle."""
    import ctypes as C
    from lz4util import buf
    from test_gpu_stream import gpu_dict_decode, orc_dict_decode
    rng = random.Random(2025)
    blocks = [_dense_block(rng, rng.choice((5, 60, 300, 900)), 0.55, 0.01, 0.2) for _ in range(48)]
    comps, caps, tg, plains = [], [], [], []
    for k, (c, out) in enumerate(blocks):
        for v in range(3):
            cc = bytearray(c)
            if v == 1:
                cc = cc[:rng.randrange(1, len(cc) + 1)]
            elif v == 2:
                for _ in range(rng.randrange(1, 3)):
                    cc[rng.randrange(len(cc))] = rng.randrange(256)
            comps.append(bytes(cc))
            caps.append(rng.choice((len(out), len(out) - 1, len(out) + 7)) if v else len(out))
            tg.append(rng.randrange(0, len(out) + 8))
            plains.append(out)
    for targets in (None, tg):
        rs, outs = run_decode(cuda, product, comps, caps, targets=targets)
        bad = []
        for i, (c, cap, r, o) in enumerate(zip(comps, caps, rs, outs)):
            er, eo = orc_decompress(oracle, c, cap, None if targets is None else targets[i])
            if r != er or (r > 0 and o != eo[:er] and not _has_off0(c)):
                bad.append((i, len(c), cap, r, er))
        assert not bad, bad[:10]
        if targets is None:   # the unmodified blocks decode in full
            assert all(rs[3 * k] == len(out) and outs[3 * k] == out for k, (_, out) in enumerate(blocks))
    # decompress_fast on the valid blocks, exact size and 3 short
    cases = [(c, len(out) - d) for c, out in blocks for d in (0, 3) if len(out) - d > 0]
    blobs = [c for c, _ in cases]
    ins, iptr, _ = pack(cuda, blobs)
    osz = [n for _, n in cases]
    dst, dptr, doffs = alloc_out(cuda, osz)
    res = ints(cuda, [0] * len(cases))
    product.decompress_fast_ptr_batch(iptr, ints(cuda, [len(b) for b in blobs]), dptr,
                                      ints(cuda, osz), res)
    cuda.cuda.synchronize()
    rs = res.cpu().tolist()
    for i, (c, n) in enumerate(cases):
        o = C.create_string_buffer(max(n, 1) + 64)
        er = oracle.orc_decompress_fast(buf(c), o, n)
        assert rs[i] == er, (i, n, len(c), rs[i], er)
        if er > 0:
            assert fetch(dst, doffs[i], n) == o.raw[:n], i
    # usingDict: the same blocks after a random history (matches stay inside their own output)
    dicts = [bytes(rng.randrange(256) for _ in range(rng.choice((0, 100, 5000, 70000))))
             for _ in blocks]
    got = gpu_dict_decode(cuda, product, [c for c, _ in blocks], [len(o) for _, o in blocks],
                          dicts, False)
    for (c, out), d, g in zip(blocks, dicts, got):
        assert g == orc_dict_decode(oracle, c, len(out), d) == (len(out), out)
