#!/usr/bin/env python3
"""Time-bounded GPU encoder fuzz against the oracle (TEST INFRASTRUCTURE, run by hand on a GPU
box; the pytest suite runs bounded forms in tests/test_gpu_encode.py and test_gpu_encode_exact.py).

Blocks of 0 B .. 64 KiB spliced from 1-4 pieces of App. C / text / random / periodic / zero
content, at capacities around the reference's own compressed size (size - 1, size, size + 1),
the bound, bound - 1, 0 and random values, through two product entry points:
  * APE_LZ4_compress_fast_batch_dev (the chunk encoder; acceleration 1, 2 or 8): 0 <= ret <= cap,
    a nonzero block decodes with the oracle to the input, a capacity >= compressBound never
    fails, an empty input returns what the oracle returns;
  * APE_LZ4_compress_exact_batch_dev (greedy-exact mode): ret and bytes equal to the oracle's
    compress_fast at the same capacity (limitedOutput) and acceleration;
  * APE_LZ4_compress_withPrefix_batch_dev (round 6): chunks of 0 .. 64 KiB of a mixed stream with
    0 .. 64 KiB of the stream before them as history, every block decoded by the oracle's
    decompress_safe_usingDict with that history to the chunk.
Canaries around every dst slot are checked per batch (nothing written outside dst[0:cap)).

  python3 tests/fuzz/gpu_encode_fuzz.py SECONDS [SEED]
prints one progress line per batch and a JSON summary; exit 1 on the first mismatch."""
import ctypes
import json

import numpy as np
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
sys.path[:0] = [TESTS, os.path.join(TESTS, "golden"), os.path.dirname(TESTS)]

import inputs as I  # noqa: E402
from gpuutil import alloc_out, check_canaries, fetch, ints, pack  # noqa: E402
from lz4util import orc_compress, orc_decompress  # noqa: E402

KINDS = ["comp", "text", "rand", "period3", "zeros", "byte"]


def block(rng):
    n = rng.choice([0, 1, 12, 13, 64, 300, 1000, 4096, 8192, 20000, 65535, 65536,
                    rng.randrange(65537)])
    out = bytearray()
    while len(out) < n:
        out += I.make(rng.choice(KINDS), rng.randrange(1, n + 1), seed=rng.randrange(1 << 30))
    return bytes(out[:n])


def fail(what, **kw):
    print(json.dumps(dict(mismatch=what, **kw)), flush=True)
    sys.exit(1)


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 20261
    import torch
    import libapenetwork_amd as amd
    if not torch.cuda.is_available():
        sys.exit("no GPU")
    orc = ctypes.CDLL(os.path.join(os.path.dirname(TESTS), "oracle", "liblz4_oracle.so"))
    rng = random.Random(seed)
    t0, nb, checked = time.time(), 0, {"chunk": 0, "exact": 0, "prefix": 0}
    while time.time() - t0 < seconds:
        srcs = [block(rng) for _ in range(1000)]
        accel = rng.choice([1, 1, 1, 2, 8])
        caps, refs = [], []
        for s in srcs:
            bound = amd.compressBound(len(s))
            r, c = orc_compress(orc, s, accel=accel)
            refs.append((r, c))
            caps.append(max(0, rng.choice([bound, bound, r, r - 1, r + 1, bound - 1, 0,
                                           rng.randrange(bound + 1)])))
        src, sptr, _ = pack(torch, srcs)
        sizes, capt = ints(torch, map(len, srcs)), ints(torch, caps)
        for mode in ("chunk", "exact"):
            dst, dptr, doffs = alloc_out(torch, caps)
            res = ints(torch, [0] * len(srcs))
            if mode == "chunk":
                amd.compress_fast_ptr_batch(sptr, sizes, dptr, capt, res, accel)
            else:
                amd.compress_exact_ptr_batch(sptr, sizes, dptr, capt, res, accel)
            torch.cuda.synchronize()
            rs = res.cpu().tolist()
            for i, (s, cap, r) in enumerate(zip(srcs, caps, rs)):
                out = fetch(dst, doffs[i], r)
                info = dict(mode=mode, batch=nb, block=i, n=len(s), cap=cap, accel=accel, gpu=r)
                if mode == "exact":
                    er, ec = orc_compress(orc, s, cap=cap, accel=accel)
                    if r != er or out != ec:
                        fail("exact", oracle=er, **info)
                    continue
                if r < 0 or r > max(cap, 0):
                    fail("range", **info)
                if len(s) == 0:
                    er, _ = orc_compress(orc, s, cap=cap, accel=accel)
                    if r != er:
                        fail("empty", oracle=er, **info)
                    continue
                if r == 0:
                    if cap >= amd.compressBound(len(s)):
                        fail("failed at the bound", **info)
                    continue
                dr, dout = orc_decompress(orc, out, len(s))
                if dr != len(s) or dout != s:
                    fail("roundtrip", decoded=dr, **info)
            check_canaries()
            checked[mode] += len(srcs)
        # withPrefix: chunks of one stream against the bytes before them
        plain = b"".join(srcs[:160])[:3 << 20]
        if len(plain) > 70000:
            starts, lens, pres = [], [], []
            for _ in range(400):
                ln = rng.choice([0, 1, 13, 64, 300, 4096, 8192, 65536, rng.randrange(65537)])
                st = rng.randrange(0, len(plain) - ln + 1)
                pres.append(min(st, rng.choice([0, 64, 4096, 65536, rng.randrange(65537)])))
                starts.append(st)
                lens.append(ln)
            dplain = torch.from_numpy(np.frombuffer(plain + bytes(64), np.uint8).copy()).cuda()
            pcaps = [amd.compressBound(ln) for ln in lens]
            dst, dptr, doffs = alloc_out(torch, pcaps)
            res = ints(torch, [0] * len(starts))
            amd.compress_prefix_batch(
                torch.tensor([dplain.data_ptr() + st for st in starts], dtype=torch.int64, device="cuda"),
                ints(torch, lens), ints(torch, pres), dptr, ints(torch, pcaps), res)
            torch.cuda.synchronize()
            rs = res.cpu().tolist()
            for i, (st, ln, pr, r) in enumerate(zip(starts, lens, pres, rs)):
                info = dict(mode="prefix", batch=nb, block=i, n=ln, prefix=pr, gpu=r)
                if r <= 0 or r > pcaps[i]:
                    if not (ln == 0 and r == 1):
                        fail("range", **info)
                comp = fetch(dst, doffs[i], r)
                d = ctypes.create_string_buffer(plain[st - pr:st] + b"\0", pr + 1)
                o = ctypes.create_string_buffer(ln + 64)
                dr = orc.orc_decompress_safe_usingDict(ctypes.c_char_p(comp + bytes(16)), o, len(comp),
                                                       ln, d, pr)
                if dr != ln or o.raw[:ln] != plain[st:st + ln]:
                    fail("prefix roundtrip", decoded=dr, **info)
            check_canaries()
            checked["prefix"] += len(starts)
        nb += 1
        print("batch %d: %d blocks x 2 modes, %.0f s" % (nb, checked["chunk"], time.time() - t0),
              flush=True)
    print(json.dumps({"seconds": round(time.time() - t0, 1), "seed": seed, "batches": nb,
                      "blocks_checked": checked, "mismatches": 0, "canaries": "intact"}), flush=True)


if __name__ == "__main__":
    main()
