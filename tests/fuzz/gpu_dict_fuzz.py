#!/usr/bin/env python3
"""Time-bounded GPU usingDict-decoder fuzz against the oracle (TEST INFRASTRUCTURE, run by hand
on a GPU box; the pytest suite runs the bounded form, tests/test_gpu_stream.py).

Chained streams (compress_fast_continue per chunk, the reference socket TX, on the oracle) of
mixed content; every chunk is decoded by APE_LZ4_decompress_safe_usingDict_batch_dev with its
history -- the whole 64 KiB, or cut short (the offset check against dst - dictSize), in a
separate buffer or adjacent to the output (the prefix form) -- and compared with the oracle's
decompress_safe_usingDict: return value and bytes.  Most chunks are mutated (byte flips,
truncation, spliced 255 runs, offsets pushed past the history); capacities are the chunk
size, one less, more, or random.  Streams with a zero offset are compared by return value.

  python3 tests/fuzz/gpu_dict_fuzz.py SECONDS [SEED]"""
import ctypes as C
import json
import os
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
sys.path[:0] = [TESTS, os.path.join(TESTS, "golden"), os.path.dirname(TESTS)]

import gen_golden  # noqa: E402
import inputs as I  # noqa: E402
from gpu_decode_fuzz import mutate  # noqa: E402
from test_gpu_stream import gpu_dict_decode, oracle_stream_chunks, orc_dict_decode  # noqa: E402

KINDS = ["comp", "comp", "text", "rand", "period3", "zeros"]


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 20262
    import torch
    import libapenetwork_amd as amd
    if not torch.cuda.is_available():
        sys.exit("no GPU")
    orc = C.CDLL(os.path.join(os.path.dirname(TESTS), "oracle", "liblz4_oracle.so"))
    orc.orc_createStream.restype = C.c_void_p
    rng = random.Random(seed)
    t0, nb, checked = time.time(), 0, 0
    while time.time() - t0 < seconds:
        comps, caps, dicts = [], [], []
        while len(comps) < 1500:
            plain = bytearray()
            n = rng.randrange(20000, 300000)
            while len(plain) < n:
                plain += I.make(rng.choice(KINDS), rng.randrange(1000, 70000), seed=rng.randrange(1 << 30))
            plain = bytes(plain[:n])
            chunk = rng.choice([8192, 8192, 4096, 16384, 65536])
            for pos, ln, c in oracle_stream_chunks(orc, plain, chunk):
                comps.append(mutate(rng, c) if rng.random() < 0.7 else c)
                caps.append(max(0, rng.choice([ln, ln, ln - 1, ln + 100, rng.randrange(ln + 1)])))
                d = plain[max(0, pos - 65536):pos]
                if rng.random() < 0.3:
                    d = d[len(d) - rng.randrange(len(d) + 1):]
                dicts.append(d)
        adjacent = rng.random() < 0.5
        got = gpu_dict_decode(torch, amd, comps, caps, dicts, adjacent)
        for i, (c, cap, d, (r, b)) in enumerate(zip(comps, caps, dicts, got)):
            er, eb = orc_dict_decode(orc, c, cap, d)
            if r != er or (r > 0 and b != eb and not gen_golden.has_offset0(c)):
                print(json.dumps({"mismatch": "usingDict", "batch": nb, "block": i, "csize": len(c),
                                  "cap": cap, "dict": len(d), "adjacent": adjacent, "gpu": r,
                                  "oracle": er}), flush=True)
                sys.exit(1)
        nb += 1
        checked += len(comps)
        print("batch %d: %d chunks, %.0f s" % (nb, checked, time.time() - t0), flush=True)
    print(json.dumps({"seconds": round(time.time() - t0, 1), "seed": seed, "batches": nb,
                      "chunks_checked": checked, "mismatches": 0}), flush=True)


if __name__ == "__main__":
    main()
