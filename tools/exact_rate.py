#!/usr/bin/env python3
"""exact_rate.py -- DESIGN TOOL: throughput of the greedy-exact encode mode
(APE_LZ4_compress_exact_batch_dev) next to the product encoder on the same App. C blocks,
and a byte-for-byte check of a sample against the oracle restatement.

  python tools/exact_rate.py [nblocks]
"""
import ctypes as C
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import libapenetwork_amd as amd  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    n = 65536
    assert amd.gpu_init() == 0, amd.gpu_last_error()
    slot = (amd.compressBound(n) + 15) // 16 * 16
    src = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    amd.synth_blocks(src, n, 0, 1)
    comp = torch.zeros((nb, slot), dtype=torch.uint8, device="cuda")
    sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
    caps = torch.full((nb,), slot, dtype=torch.int32, device="cuda")
    res = torch.zeros(nb, dtype=torch.int32, device="cuda")
    sp = torch.tensor([src.data_ptr() + i * n for i in range(nb)], dtype=torch.int64, device="cuda")
    dp = torch.tensor([comp.data_ptr() + i * slot for i in range(nb)], dtype=torch.int64,
                      device="cuda")
    out = {}
    for name, fn in (("exact", lambda: amd.compress_exact_ptr_batch(sp, sizes, dp, caps, res, 1)),
                     ("product", lambda: amd.compress_fast_ptr_batch(sp, sizes, dp, caps, res, 1))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        out[name] = (dt, int(res.to(torch.int64).sum().item()))
        if name == "exact":   # byte check of a sample against the oracle restatement
            orc = C.CDLL(os.path.join(ROOT, "oracle", "liblz4_oracle.so"))
            bad = 0
            for i in range(0, nb, max(1, nb // 16)):
                s = src[i].cpu().numpy().tobytes()
                o = C.create_string_buffer(slot + 64)
                r = orc.orc_compress_default(C.create_string_buffer(s + b"\0" * 64, n + 64), o, n, slot)
                g = comp[i, :int(res[i].item())].cpu().numpy().tobytes()
                bad += (r != int(res[i].item()) or o.raw[:r] != g)
            out["sample_mismatches"] = bad
    for name in ("exact", "product"):
        dt, tot = out[name]
        print("%-8s %6d blocks: %9.2f ms  %8.2f GiB/s  ratio %.4f" % (
            name, nb, dt * 1e3, nb * n / dt / 2**30, nb * n / tot))
    print("exact vs oracle sample mismatches:", out["sample_mismatches"])


if __name__ == "__main__":
    main()
