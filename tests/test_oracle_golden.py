"""Pin the oracle (CPU restatement) against the reference's own outputs.

tests/golden/lz4_golden.json was produced by running the reference src/ape_lz4.c
(oracle/_ref, see tests/golden/gen_golden.py).  Every encode KAT, every decode
KAT (valid, crafted-malformed and mutated streams; full and partial decoding)
and the socket-style stream KATs must match bit for bit.
"""
import base64
import ctypes as C

import pytest

from lz4util import I, blob_matches, buf, orc_compress, orc_decompress, sha


def test_constants(oracle, golden):
    assert oracle.orc_versionNumber() == golden["version"] == 10701
    assert oracle.orc_sizeofState() == golden["sizeofState"] == 16416


def test_encode_kats(oracle, golden):
    for e in golden["encode"]:
        src = I.make(e["content"], e["n"])
        assert I.sha(src) == e["in_sha256"], e["content"]
        assert oracle.orc_compressBound(e["n"]) == e["bound"]
        r, comp = orc_compress(oracle, src)
        assert r == e["clen"], (e["content"], e["n"])
        assert blob_matches(e["comp"], comp), (e["content"], e["n"])
        for lim in e["limited"]:
            lr, lcomp = orc_compress(oracle, src, cap=lim["cap"])
            assert lr == lim["ret"] and sha(lcomp) == lim["sha256"], (e["content"], e["n"], lim)
        for ac in e["accel"]:
            ar, acomp = orc_compress(oracle, src, accel=ac["accel"])
            assert ar == ac["ret"] and sha(acomp) == ac["sha256"]


def test_decode_kats(oracle, golden):
    for d in golden["decode"]:
        comp = base64.b64decode(d["comp_b64"])
        r, out = orc_decompress(oracle, comp, d["cap"])
        assert r == d["ret"], d["name"]
        if r > 0 and not d["has_offset0"]:
            assert sha(out) == d["out_sha256"], d["name"]
        p = d["partial"]
        pr, pout = orc_decompress(oracle, comp, d["cap"], p["target"])
        assert pr == p["ret"], d["name"]
        if pr > 0 and not d["has_offset0"]:
            assert sha(pout) == p["out_sha256"], d["name"]


def test_decode_fast_kats(oracle, golden):
    """decompress_fast (ref :1489) on the reference's own results (valid streams,
    originalSize = n and n - 1)."""
    n = 0
    for d in golden["decode"]:
        if "fast" not in d:
            continue
        comp, f = base64.b64decode(d["comp_b64"]), d["fast"]
        out = C.create_string_buffer(max(f["osize"], 1) + 64)
        r = oracle.orc_decompress_fast(buf(comp), out, f["osize"])
        assert r == f["ret"], d["name"]
        if r > 0:
            assert sha(out.raw[:f["osize"]]) == f["out_sha256"], d["name"]
        n += 1
    assert n > 200


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_stream_kats(oracle, golden, idx):
    st = golden["stream"][idx]
    msgs = [I.make(st["content"], st["msg_len"], seed=s) for s in st["seeds"]]
    s = C.c_void_p(oracle.orc_createStream())
    dictbuf = C.create_string_buffer(65536)
    frames, keep = [], []
    for msg in msgs:
        mb = buf(msg)
        keep.append(mb)
        pos = 0
        while pos < len(msg):
            ln = min(8192, len(msg) - pos)
            ob = C.create_string_buffer(8240 + 64)
            r = oracle.orc_compress_fast_continue(s, C.byref(mb, pos), ob, ln, 8240, 1)
            frames.append(ob.raw[:r])
            pos += ln
        oracle.orc_saveDict(s, dictbuf, 65536)
    assert [base64.b64encode(f).decode() for f in frames] == st["frames_b64"]
    # RX replay through a 64 KiB ring
    ds = C.c_void_p(oracle.orc_createStreamDecode())
    ring = C.create_string_buffer(65536)
    rp, rets, plain = 0, [], b""
    for fr in frames:
        tmp = C.create_string_buffer(8192 + 64)
        r = oracle.orc_decompress_safe_continue(ds, buf(fr), tmp, len(fr), 8192)
        rets.append(r)
        if r <= 0:
            break
        plain += tmp.raw[:r]
        if rp + r > 65536:
            keepn = 65536 - r
            C.memmove(ring, C.byref(ring, rp - keepn), keepn)
            rp = keepn
        C.memmove(C.byref(ring, rp), tmp, r)
        rp += r
        oracle.orc_setStreamDecode(ds, ring, rp)
    assert rets == st["dec_rets"]
    assert sha(plain) == st["plain_sha256"] and st["plain_ok"]


def test_synth_matches_spec(oracle):
    """oracle/synth.c == tests/golden/inputs.py."""
    for kind, fn in ((0, I.synth_rand), (1, I.synth_comp)):
        for n, b in ((65536, 7), (4096, 123)):
            out = C.create_string_buffer(n)
            oracle.synth_blocks(out, n, C.c_longlong(n), C.c_longlong(b), 1, kind)
            assert out.raw == fn(n, b)


def test_benchmark_data_ratio(oracle):
    """The compressible generator reproduces the survey's ratio (~3.15 at 64 KiB)."""
    n, nb = 65536, 8
    src = C.create_string_buffer(n * nb)
    oracle.synth_blocks(src, n, C.c_longlong(n), C.c_longlong(0), nb, 1)
    tot = 0
    out = C.create_string_buffer(n + n // 255 + 16)
    for b in range(nb):
        tot += oracle.orc_compress_default(C.byref(src, b * n), out, n, n + n // 255 + 16)
    assert 3.05 < n * nb / tot < 3.25
