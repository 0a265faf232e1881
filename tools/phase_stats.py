#!/usr/bin/env python3
"""Per-phase cycle breakdown of the LZ4 kernels (diagnostic build only).

Loads libapenetwork_amd/libape_lz4_amd_stats.so (make -C libapenetwork_amd/csrc stats),
whose kernels accumulate s_memtime cycles of workgroup thread 0 per phase, and prints
the average cycles per block for each phase next to the kernel's HIP-event time.
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("APE_LZ4_LIB", os.path.join(ROOT, "libapenetwork_amd", "libape_lz4_amd_stats.so"))
sys.path.insert(0, ROOT)

DEC = ["parse", "copy", "(batches)", "(passes after round 1)", "(restages)", "(coop matches)",
       "(window slides)", "[copy] slides", "[copy] ballots + literals", "[copy] round 1", "(blocks)",
       "[copy] dependent passes", "[copy] flushes", "", "", ""]
ENC = ["W walk", "W publish", "E write", "W wait end", "W wait mid", "P A+B+C1",
       "P wait mid", "P C2 + S2 + R", "P wait end", "P load waits", "(steps x3 waves)",
       "(members)", "E prepare",
       "(blocks)", "E wait mid", "E wait end"]


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
    out = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
    csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
    dres = torch.zeros(nb, dtype=torch.int32, device="cuda")
    buf = (C.c_ulonglong * 16)()
    for which, name, fn, labels in (
            (1, "encode", lambda: amd.compress_batch(src, sizes, comp, csz), ENC),
            (0, "decode", lambda: amd.decompress_batch(comp, csz, out, dres, dst_caps=sizes), DEC)):
        fn()
        torch.cuda.synchronize()
        L.APE_LZ4_debug_stats(which, buf, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        L.APE_LZ4_debug_stats(which, buf, 1)
        ms = e0.elapsed_time(e1)
        vals = list(buf)
        blocks = vals[labels.index("(blocks)")]
        print("%s: %d blocks, %.2f ms, %.1f GB/s (in+out bytes)" % (
            name, nb, ms, (nb * n + int(csz.sum())) / ms / 1e6))
        tot = sum(v for i, v in enumerate(vals)
                  if labels[i] and not labels[i].startswith(("(", "[")) and labels[i] != "-")
        for i, lab in enumerate(labels):
            if not lab or lab == "-":
                continue
            per = vals[i] / max(blocks, 1)
            if lab.startswith("("):
                if vals[i] or not lab.startswith("(pending") and "owner" not in lab and "S0" not in lab:
                    print("   %-22s %12.1f per block" % (lab, per))
            else:
                print("   %-22s %12.0f cyc/block  %5.1f%%" % (lab, per, 100.0 * vals[i] / max(tot, 1)))
    print("verified:", bool((dres == n).all()), "ratio %.4f" % (nb * n / int(csz.sum())))


if __name__ == "__main__":
    main()
