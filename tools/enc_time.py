#!/usr/bin/env python3
"""enc_time.py -- DESIGN TOOL (GPU box): median HIP-event time of compress_batch over 131072 App. C
blocks for the library APE_LZ4_LIB names (a variant built by tools/enc_variant.sh or make variant);
for variants whose output is not a valid block (sensitivity builds), where tools/ab_inproc.py stops."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libapenetwork_amd as amd
nb, n = 131072, 65536
slot = (amd.compressBound(n) + 15) // 16 * 16
src = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
for b0 in range(0, nb, 1 << 16):
    amd.synth_blocks(src[b0:b0 + (1 << 16)], n, b0, 1)
comp = torch.empty((nb, slot), dtype=torch.uint8, device="cuda")
sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
ts = []
for i in range(8):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); amd.compress_batch(src, sizes, comp, csz); e1.record(); torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
ts = sorted(ts[1:])
print(os.path.basename(os.environ.get("APE_LZ4_LIB", "base")), "encode ms median %.3f min %.3f" % (ts[len(ts) // 2], ts[0]))
