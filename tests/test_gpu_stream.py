"""Chained-stream path on the GPU: usingDict decode parity and
withPrefix encode round trips.

The reference socket compresses 8 KiB chunks with compress_fast_continue against the
previous <= 64 KiB of the stream and decodes them with decompress_safe_continue
(ref src/ape_socket.c:832-857, :1386-1421; src/ape_lz4.c:1160-1220, :1555-1584).  The
oracle's streaming restatement (pinned by the golden socket-stream KATs,
tests/test_oracle_golden.py::test_stream_kats) produces the chunks and is the checker
for every decode; the GPU decode must match orc_decompress_safe_usingDict bit for bit
(return value and dst[0:ret]), and every GPU-encoded chunk must decode with it to the
original bytes.
"""
import ctypes as C
import random

import numpy as np
import pytest

from lz4util import I, buf

pytestmark = pytest.mark.gpu

CHUNK = 8192


def stream_plain(n, seed):
    return I.make("comp", n, seed=seed)


def oracle_stream_chunks(oracle, plain, chunk=CHUNK):
    """Compress `plain` as the reference TX does (compress_fast_continue per chunk)."""
    s = C.c_void_p(oracle.orc_createStream())
    pb = buf(plain)
    out = []
    for pos in range(0, len(plain), chunk):
        ln = min(chunk, len(plain) - pos)
        cap = oracle.orc_compressBound(ln)
        ob = C.create_string_buffer(cap + 64)
        r = oracle.orc_compress_fast_continue(s, C.byref(pb, pos), ob, ln, cap, 1)
        assert r > 0
        out.append((pos, ln, ob.raw[:r]))
    oracle.orc_freeStream(s)
    return out


def orc_dict_decode(oracle, comp, cap, dict_bytes):
    d = buf(dict_bytes)
    o = C.create_string_buffer(max(cap, 1) + 64)
    r = oracle.orc_decompress_safe_usingDict(buf(comp), o, len(comp), cap, d, len(dict_bytes))
    return r, o.raw[:max(r, 0)]


def gpu_dict_decode(torch, amd, comps, caps, dicts, adjacent):
    """Decode comps[i] with dictionary dicts[i]; adjacent=True places each dictionary
    right before its output slot (the reference's prefix / withPrefix64k forms)."""
    n = len(comps)
    # inputs
    coff, pos = [], 0
    for c in comps:
        coff.append(pos)
        pos += len(c) + 64
    hin = np.zeros(pos + 64, np.uint8)
    for o, c in zip(coff, comps):
        hin[o:o + len(c)] = np.frombuffer(c, np.uint8)
    din = torch.from_numpy(hin).cuda()
    # outputs (+ dictionaries)
    doff, ooff, pos = [], [], 0
    for d, cap in zip(dicts, caps):
        pos = (pos + 15) // 16 * 16
        if adjacent:
            doff.append(pos)
            pos += len(d)
            ooff.append(pos)
            pos += cap + 64
        else:
            ooff.append(pos)
            pos += cap + 64
    hout = np.full(pos + 64, 0xCD, np.uint8)
    if adjacent:
        for o, d in zip(doff, dicts):
            hout[o:o + len(d)] = np.frombuffer(d, np.uint8)
    dout = torch.from_numpy(hout).cuda()
    if adjacent:
        dptr = [dout.data_ptr() + o for o in doff]
    else:
        dpos, pos2 = [], 0
        for d in dicts:
            pos2 = (pos2 + 7) // 8 * 8 + 3      # odd placement
            dpos.append(pos2)
            pos2 += len(d) + 64
        hd = np.zeros(pos2 + 64, np.uint8)
        for o, d in zip(dpos, dicts):
            hd[o:o + len(d)] = np.frombuffer(d, np.uint8)
        ddict = torch.from_numpy(hd).cuda()
        dptr = [ddict.data_ptr() + o for o in dpos]
    t = lambda v: torch.tensor(v, dtype=torch.int64, device="cuda")
    ti = lambda v: torch.tensor(v, dtype=torch.int32, device="cuda")
    res = ti([0] * n)
    amd.decompress_dict_batch(t([din.data_ptr() + o for o in coff]), ti([len(c) for c in comps]),
                              t([dout.data_ptr() + o for o in ooff]), ti(caps), t(dptr),
                              ti([len(d) for d in dicts]), res)
    torch.cuda.synchronize()
    r = res.cpu().tolist()
    host = dout.cpu().numpy()
    return [(r[i], host[ooff[i]:ooff[i] + max(r[i], 0)].tobytes()) for i in range(n)]


@pytest.mark.parametrize("adjacent", [False, True])
def test_dict_decode_socket_stream(oracle, product, cuda, adjacent):
    """Every chunk of a compress_fast_continue stream, decoded with its history."""
    plain = stream_plain(400000, seed=7)
    chunks = oracle_stream_chunks(oracle, plain)
    comps, caps, dicts = [], [], []
    for pos, ln, c in chunks:
        comps.append(c)
        caps.append(ln)
        dicts.append(plain[max(0, pos - 65536):pos])
    got = gpu_dict_decode(cuda, product, comps, caps, dicts, adjacent)
    for (pos, ln, c), d, (r, b) in zip(chunks, dicts, got):
        exp = orc_dict_decode(oracle, c, ln, d)
        assert exp == (ln, plain[pos:pos + ln])
        assert (r, b) == exp, pos


def test_dict_decode_short_dicts_and_mutations(oracle, product, cuda):
    """Dictionaries shorter than the history the stream used (offset check of :1375 with
    lowLimit = dst - dictSize), and mutated / truncated chunks: identical return codes."""
    plain = stream_plain(200000, seed=11)
    chunks = oracle_stream_chunks(oracle, plain)
    rng = random.Random(5)
    comps, caps, dicts = [], [], []
    for pos, ln, c in chunks[1:]:
        for dsz in (0, 1, 100, 4096, 65535, 65536):
            d = plain[max(0, pos - dsz):pos]
            comps.append(c)
            caps.append(ln + rng.choice([0, 0, 7, 300]))
            dicts.append(d)
        for _ in range(6):
            m = bytearray(c)
            for _ in range(rng.randint(1, 4)):
                m[rng.randrange(len(m))] = rng.randrange(256)
            if rng.random() < 0.3:
                m = m[:rng.randrange(1, len(m))]
            comps.append(bytes(m))
            caps.append(ln)
            dicts.append(plain[max(0, pos - rng.choice([10, 30000, 65536])):pos])
    got = gpu_dict_decode(cuda, product, comps, caps, dicts, adjacent=False)
    for i, (c, cap, d) in enumerate(zip(comps, caps, dicts)):
        assert got[i] == orc_dict_decode(oracle, c, cap, d), i


def gpu_prefix_encode(torch, amd, plain, starts, lens, prefixes):
    """Compress plain[s:s+l] with the preceding `prefix` bytes as history (one device
    copy of the whole stream, so the history lies right before each chunk)."""
    n = len(starts)
    dplain = torch.from_numpy(np.frombuffer(plain + b"\0" * 64, np.uint8).copy()).cuda()
    caps = [amd.compressBound(l) for l in lens]
    ooff, pos = [], 0
    for cap in caps:
        ooff.append(pos)
        pos += (cap + 64 + 15) // 16 * 16
    dout = torch.zeros(pos + 64, dtype=torch.uint8, device="cuda")
    t = lambda v: torch.tensor(v, dtype=torch.int64, device="cuda")
    ti = lambda v: torch.tensor(v, dtype=torch.int32, device="cuda")
    res = ti([0] * n)
    amd.compress_prefix_batch(t([dplain.data_ptr() + s for s in starts]), ti(lens), ti(prefixes),
                              t([dout.data_ptr() + o for o in ooff]), ti(caps), res)
    torch.cuda.synchronize()
    r = res.cpu().tolist()
    host = dout.cpu().numpy()
    return [host[ooff[i]:ooff[i] + max(r[i], 0)].tobytes() if r[i] > 0 else r[i] for i in range(n)]


def test_prefix_encode_socket_stream(oracle, product, cuda):
    """8 KiB chunks with the previous 64 KiB as history: each decodes with
    decompress_safe_usingDict (= the receiver's decompress_safe_continue) to the chunk,
    and the history pays (ratio well above independent chunks)."""
    plain = stream_plain(600000, seed=3)
    starts = list(range(0, len(plain), CHUNK))
    lens = [min(CHUNK, len(plain) - s) for s in starts]
    pre = [min(s, 65536) for s in starts]
    outs = gpu_prefix_encode(cuda, product, plain, starts, lens, pre)
    indep = gpu_prefix_encode(cuda, product, plain, starts, lens, [0] * len(starts))
    tot = tot0 = 0
    for s, l, p, c, c0 in zip(starts, lens, pre, outs, indep):
        assert isinstance(c, bytes) and isinstance(c0, bytes)
        assert orc_dict_decode(oracle, c, l, plain[s - p:s]) == (l, plain[s:s + l]), s
        assert orc_dict_decode(oracle, c0, l, b"") == (l, plain[s:s + l]), s
        tot += len(c)
        tot0 += len(c0)
    ratio, ratio0 = len(plain) / tot, len(plain) / tot0
    # the reference's own chained stream on the same data, for scale
    ref = sum(len(c) for _, _, c in oracle_stream_chunks(oracle, plain))
    assert ratio > 1.5 * ratio0, (ratio, ratio0)
    assert ratio >= 0.9 * len(plain) / ref, (ratio, len(plain) / ref)


def test_prefix_encode_edges(oracle, product, cuda):
    """Chunk sizes 0..64 KiB against prefixes 0..64 KiB (history trimmed so that history
    + chunk fit one 64 KiB window), tiny and incompressible chunks, then the
    reference's decoder with the full history as dictionary."""
    plain = stream_plain(200000, seed=9) + I.make("rand", 70000, seed=4) + stream_plain(140000, 5)
    rng = random.Random(1)
    starts, lens, pre = [], [], []
    for l in (0, 1, 5, 12, 13, 14, 63, 64, 65, 127, 128, 300, 4096, 8192, 30000, 65535, 65536):
        for p in (0, 1, 63, 64, 100, 4095, 40000, 65536):
            s = rng.randrange(65536, len(plain) - l)
            starts.append(s)
            lens.append(l)
            pre.append(p)
    outs = gpu_prefix_encode(cuda, product, plain, starts, lens, pre)
    for s, l, p, c in zip(starts, lens, pre, outs):
        assert isinstance(c, bytes), (l, p, c)
        assert orc_dict_decode(oracle, c, l, plain[s - p:s]) == (l, plain[s:s + l]), (l, p)
        # the decoder never needs more history than given: a longer dictionary agrees
        assert orc_dict_decode(oracle, c, l, plain[max(0, s - 65536):s]) == (l, plain[s:s + l])


def test_prefix_encode_then_gpu_dict_decode(oracle, product, cuda):
    """GPU TX -> GPU RX round trip of a whole stream (both sides batched)."""
    plain = stream_plain(300000, seed=21)
    starts = list(range(0, len(plain), CHUNK))
    lens = [min(CHUNK, len(plain) - s) for s in starts]
    pre = [min(s, 65536) for s in starts]
    outs = gpu_prefix_encode(cuda, product, plain, starts, lens, pre)
    got = gpu_dict_decode(cuda, product, outs, lens, [plain[s - p:s] for s, p in zip(starts, pre)],
                          adjacent=False)
    for s, l, (r, b) in zip(starts, lens, got):
        assert (r, b) == (l, plain[s:s + l])
