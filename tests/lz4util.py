"""Small helpers shared by the tests (no product or oracle logic here)."""
import base64
import ctypes as C
import hashlib
import os

import inputs as I

_REF = []


def ref_lib():
    """oracle/_ref/libape_lz4_ref.so -- the reference src/ape_lz4.c compiled from its own
    source by oracle/Makefile (a checker, like the oracle), or None when it was not built."""
    if not _REF:
        p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         "oracle", "_ref", "libape_lz4_ref.so")
        _REF.append(C.CDLL(p) if os.path.exists(p) else None)
    return _REF[0]


def buf(b, pad=64):
    return C.create_string_buffer(bytes(b) + b"\0" * pad, len(b) + pad)


def blob_matches(blob, data):
    if "b64" in blob:
        return base64.b64decode(blob["b64"]) == data
    return blob["len"] == len(data) and blob["sha256"] == hashlib.sha256(data).hexdigest()


def sha(b):
    return hashlib.sha256(b).hexdigest()


def orc_compress(orc, src, cap=None, accel=None):
    n = len(src)
    bound = orc.orc_compressBound(n)
    cap = bound if cap is None else cap
    out = C.create_string_buffer(max(cap, 1) + 64)
    if accel is None:
        r = orc.orc_compress_default(buf(src), out, n, cap)
    else:
        r = orc.orc_compress_fast(buf(src), out, n, cap, accel)
    return r, out.raw[:max(r, 0)]


def orc_decompress(orc, comp, cap, target=None):
    out = C.create_string_buffer(max(cap, 0) + 64)
    if target is None:
        r = orc.orc_decompress_safe(buf(comp), out, len(comp), cap)
    else:
        r = orc.orc_decompress_safe_partial(buf(comp), out, len(comp), target, cap)
    return r, out.raw[:max(r, 0)]


def walk_ok(comp):
    """Structural LZ4 walk used by encoder tests: returns list of (lit, off, mlen)."""
    seqs, ip, n = [], 0, len(comp)
    while True:
        tok = comp[ip]
        ip += 1
        lit = tok >> 4
        if lit == 15:
            while True:
                s = comp[ip]
                ip += 1
                lit += s
                if s != 255:
                    break
        ip += lit
        if ip == n:
            seqs.append((lit, 0, 0))
            return seqs
        off = comp[ip] | (comp[ip + 1] << 8)
        ip += 2
        ml = tok & 15
        if ml == 15:
            while True:
                s = comp[ip]
                ip += 1
                ml += s
                if s != 255:
                    break
        seqs.append((lit, off, ml + 4))


__all__ = ["I", "buf", "blob_matches", "sha", "orc_compress", "orc_decompress", "walk_ok"]
