#!/usr/bin/env python3
"""Time-bounded GPU decoder fuzz against the oracle (TEST INFRASTRUCTURE, run by hand on a GPU
box; the pytest suite runs the bounded form, tests/test_gpu_decode.py::test_fuzz_malformed_vs_oracle).

Batches of reference-compressed blocks (App. C / text / random / periodic / zero contents,
16 B .. 64 KiB), mutated -- byte flips, truncation, a run of 255 length bytes spliced in,
an offset zeroed or pushed past the output, a token's nibbles rewritten -- are decoded by
the product's decompress_safe and decompress_safe_partial batch entry points and compared
with the oracle: the return value of every block (the negative -(ip)-1 codes included), the
bytes dst[0:ret], and the canaries around every dst slot (nothing written outside dst[0:cap)).
Streams with a zero offset are compared by return value only.

  python3 tests/fuzz/gpu_decode_fuzz.py SECONDS [SEED]
prints one progress line per batch and a JSON summary; exit 1 on the first mismatch."""
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
sys.path[:0] = [TESTS, os.path.join(TESTS, "golden"), os.path.dirname(TESTS)]

import ctypes  # noqa: E402

import gen_golden  # noqa: E402
import inputs as I  # noqa: E402
from gpuutil import alloc_out, check_canaries, fetch, ints, pack  # noqa: E402
from lz4util import orc_compress, orc_decompress  # noqa: E402


def mutate(rng, c):
    c = bytearray(c)
    for _ in range(rng.randrange(0, 4)):
        if not c:
            break
        kind = rng.randrange(6)
        i = rng.randrange(len(c))
        if kind == 0:
            c[i] = rng.randrange(256)
        elif kind == 1:
            c[i] ^= 1 << rng.randrange(8)
        elif kind == 2:
            c[i:i] = b"\xff" * rng.randrange(1, 40)
        elif kind == 3 and i + 2 <= len(c):
            c[i:i + 2] = b"\x00\x00"
        elif kind == 4 and i + 2 <= len(c):
            c[i:i + 2] = rng.choice((b"\xff\xff", b"\x01\x00", bytes((rng.randrange(256), 0xFF))))
        else:
            c[i] = (rng.randrange(16) << 4) | rng.randrange(16)
    if rng.random() < 0.2:
        c = c[:rng.randrange(len(c) + 1)]
    return bytes(c)


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 20260
    import torch
    import libapenetwork_amd as amd
    if not torch.cuda.is_available():
        sys.exit("no GPU")
    orc = ctypes.CDLL(os.path.join(os.path.dirname(TESTS), "oracle", "liblz4_oracle.so"))
    rng = random.Random(seed)
    t0, nb, blocks, checked = time.time(), 0, 0, {"safe": 0, "partial": 0}
    while time.time() - t0 < seconds:
        comps, caps, tg = [], [], []
        for k in range(2000):
            content = rng.choice(["comp", "text", "rand", "period3", "zeros", "byte"])
            n = rng.choice([16, 64, 300, 1000, 4096, 8192, 20000, 65536])
            _, c = orc_compress(orc, I.make(content, n, seed=rng.randrange(1 << 30)))
            comps.append(mutate(rng, c) if rng.random() < 0.9 else c)
            cap = max(0, rng.choice([n, n - 1, n + 40, rng.randrange(n + 1), 65536]))
            if rng.random() < 0.03:
                cap = -rng.randrange(1, 1 << 20)
            caps.append(cap)
            tg.append(rng.randrange(-5, n + 40))
        src, sptr, _ = pack(torch, comps)
        for mode, targets in (("safe", None), ("partial", tg)):
            dst, dptr, doffs = alloc_out(torch, caps)
            res = ints(torch, [0] * len(comps))
            if targets is None:
                amd.decompress_ptr_batch(sptr, ints(torch, map(len, comps)), dptr, ints(torch, caps), res)
            else:
                amd.decompress_partial_batch(sptr, ints(torch, map(len, comps)), dptr,
                                             ints(torch, targets), ints(torch, caps), res)
            torch.cuda.synchronize()
            rs = res.cpu().tolist()
            for i, (c, cap, r) in enumerate(zip(comps, caps, rs)):
                er, eout = orc_decompress(orc, c, cap, None if targets is None else targets[i])
                if r != er or (r > 0 and fetch(dst, doffs[i], r) != eout and not gen_golden.has_offset0(c)):
                    print(json.dumps({"mismatch": mode, "batch": nb, "block": i, "csize": len(c),
                                      "cap": cap, "target": None if targets is None else targets[i],
                                      "gpu": r, "oracle": er, "hex": c[:256].hex()}), flush=True)
                    sys.exit(1)
            check_canaries()
            checked[mode] += len(comps)
        nb += 1
        blocks += len(comps)
        print("batch %d: %d blocks x 2 modes, %.0f s" % (nb, blocks, time.time() - t0), flush=True)
    print(json.dumps({"seconds": round(time.time() - t0, 1), "seed": seed, "batches": nb,
                      "decodes_checked": checked, "mismatches": 0, "canaries": "intact"}), flush=True)


if __name__ == "__main__":
    main()
