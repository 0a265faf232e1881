#!/usr/bin/env python3
"""DIAGNOSTIC: which golden decode KATs make the GPU decoder write outside dst[0:cap)
(full / partial / fast), one batch per mode, slot-by-slot canary report."""
import base64
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import numpy as np
import torch

import libapenetwork_amd as amd
from gpuutil import CANARY, alloc_out, ints, pack

d = json.load(open(os.path.join(ROOT, "tests", "golden", "lz4_golden.json")))["decode"]
comps = [base64.b64decode(c["comp_b64"]) for c in d]
caps = [c["cap"] for c in d]
for mode in ("full", "partial"):
    src, sptr, _ = pack(torch, comps)
    dst, dptr, doffs = alloc_out(torch, caps)
    res = ints(torch, [0] * len(comps))
    if mode == "full":
        amd.decompress_ptr_batch(sptr, ints(torch, map(len, comps)), dptr, ints(torch, caps), res)
    else:
        amd.decompress_partial_batch(sptr, ints(torch, map(len, comps)), dptr,
                                     ints(torch, [c["partial"]["target"] for c in d]),
                                     ints(torch, caps), res)
    torch.cuda.synchronize()
    h = dst.cpu().numpy()
    rs = res.cpu().tolist()
    ends = doffs[1:] + [h.shape[0]]
    for i, (o, c, e) in enumerate(zip(doffs, caps, ends)):
        tail = h[o + max(c, 0):e]
        bad = np.nonzero(tail != CANARY)[0]
        if bad.size:
            print(mode, i, d[i]["name"], "cap", c, "ret", rs[i], "exp",
                  d[i]["ret"] if mode == "full" else d[i]["partial"]["ret"],
                  "bad bytes past cap:", bad.size, "first +%d" % bad[0], "comp", comps[i][:24].hex())
