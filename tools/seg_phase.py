#!/usr/bin/env python3
"""DIAGNOSTIC (GPU box): per-phase cycles of the segment encoder (stats build:
make -C libapenetwork_amd/csrc stats), averaged per block: workgroup thread 0's s_memtime
between the barriers that close each phase."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("APE_LZ4_LIB", os.path.join(ROOT, "libapenetwork_amd", "libape_lz4_amd_stats.so"))
os.environ["APE_LZ4_ENCODER"] = "seg"
sys.path.insert(0, ROOT)
NAMES = ["load", "index", "parse (thread 0's lanes)", "parse (wait for the slowest wave)",
         "splice", "sizes + offsets", "emit", "", "", "", "(blocks)"]


def main():
    import torch
    import libapenetwork_amd as amd
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    kind = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    n = 65536
    L = amd.lib()
    L.APE_LZ4_debug_stats.argtypes = [C.c_int, C.c_void_p, C.c_int]
    slot = (amd.compressBound(n) + 15) // 16 * 16
    src = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    amd.synth_blocks(src, n, 0, kind)
    comp = torch.empty((nb, slot), dtype=torch.uint8, device="cuda")
    sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
    csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
    amd.compress_batch(src, sizes, comp, csz)   # warm-up
    torch.cuda.synchronize()
    out = (C.c_ulonglong * 16)()
    L.APE_LZ4_debug_stats(2, out, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    amd.compress_batch(src, sizes, comp, csz)
    e1.record()
    torch.cuda.synchronize()
    L.APE_LZ4_debug_stats(2, out, 0)
    blocks = out[10] or 1
    print("segment encoder, %d blocks (kind %d): %.3f ms, ratio %.4f" % (
        nb, kind, e0.elapsed_time(e1), nb * n / csz.sum().item()))
    tot = sum(out[i] for i in range(7))
    for i in range(7):
        print("  %-36s %9.0f cycles/block  %5.1f %%" % (NAMES[i], out[i] / blocks, 100.0 * out[i] / max(tot, 1)))
    print("  wave 0 per block: probes (max lane) %.1f, binary-search steps %.1f, extension steps %.1f,"
          " catch-up steps %.1f, probes (all lanes) %.0f" % tuple(out[i] / blocks for i in (11, 12, 13, 14, 15)))


if __name__ == "__main__":
    main()
