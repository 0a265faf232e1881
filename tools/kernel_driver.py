#!/usr/bin/env python3
"""Run lz4_encode_kernel and lz4_decode_kernel once each over N synthetic blocks
(for rocprofv3 --kernel-trace / --pmc).  usage: kernel_driver.py [nblocks] [kind]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import libapenetwork_amd as amd
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    kind = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    n = 65536
    slot = (amd.compressBound(n) + 15) // 16 * 16
    src = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    amd.synth_blocks(src, n, 0, kind)
    comp = torch.empty((nb, slot), dtype=torch.uint8, device="cuda")
    out = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
    csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
    dres = torch.zeros(nb, dtype=torch.int32, device="cuda")
    for _ in range(reps):
        amd.compress_batch(src, sizes, comp, csz)
        amd.decompress_batch(comp, csz, out, dres, dst_caps=sizes)
    torch.cuda.synchronize()
    print("ok", bool((dres == n).all()), "ratio %.4f" % (nb * n / max(1, int(csz.sum()))))


if __name__ == "__main__":
    main()
