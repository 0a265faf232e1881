"""Deterministic input generators shared by the golden-fixture generator and the tests.

Pure Python (no oracle, no reference), so a fixture's input can be rebuilt anywhere
from its (content, size) pair; every fixture also stores the input's sha256.
`synth_rand` / `synth_comp` restate SURVEY.md Appendix C (the benchmark data).
"""
import hashlib
import random

M64 = (1 << 64) - 1


def _xs(s):
    s ^= (s << 13) & M64
    s ^= s >> 7
    s ^= (s << 17) & M64
    return s


def seed_of(block):
    return (block * 0x9E3779B97F4A7C15 + 1) & M64


def synth_rand(n, block):
    s = seed_of(block)
    out = bytearray()
    while len(out) < n:
        s = _xs(s)
        out += s.to_bytes(8, "little")
    return bytes(out[:n])


def synth_comp(n, block):
    s = seed_of(block)
    out = bytearray()
    i = 0
    while i < n:
        s = _xs(s)
        r = s
        if i >= 64 and (r & 3) != 0:
            ln = 4 + ((r >> 32) % 60)
            win = min(i, 65535)
            off = 1 + ((r >> 8) % win)
            for _ in range(ln):
                if i >= n:
                    break
                out.append(out[i - off])
                i += 1
        else:
            ln = 1 + ((r >> 8) % 16)
            for _ in range(ln):
                if i >= n:
                    break
                s = _xs(s)
                out.append(ord("a") + (s & 15))
                i += 1
    return bytes(out)


_WORDS = [b"the", b"lz4", b"block", b"socket", b"buffer", b"event", b"loop", b"gpu",
          b"stream", b"dictionary", b"compress", b"nidium", b"ape", b"  ", b"\n", b"{",
          b"}", b"\"key\": ", b"0123", b"value"]


def text(n, seed=0):
    rng = random.Random(1000 + seed)
    parts = []
    size = 0
    while size < n:
        w = rng.choice(_WORDS)
        parts.append(w)
        size += len(w)
    return b"".join(parts)[:n]


def make(content, n, seed=0):
    """content in: zeros, byte, periodK (K=2..8), rand, comp, text."""
    if content == "zeros":
        return bytes(n)
    if content == "byte":
        return b"\x41" * n
    if content.startswith("period"):
        k = int(content[6:])
        pat = bytes(range(1, k + 1))
        return (pat * (n // k + 1))[:n]
    if content == "rand":
        return synth_rand(n, seed)
    if content == "comp":
        return synth_comp(n, seed)
    if content == "text":
        return text(n, seed)
    raise ValueError(content)


def sha(b):
    return hashlib.sha256(b).hexdigest()


ENC_SIZES = [0, 1, 4, 5, 12, 13, 14, 15, 16, 17, 100, 255, 256, 4095, 4096, 8192, 65535,
             65536, 65546, 65547]
ENC_CONTENTS = ["zeros", "byte", "period2", "period3", "period7", "rand", "comp", "text"]
