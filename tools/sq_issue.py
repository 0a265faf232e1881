#!/usr/bin/env python3
"""Summarise the SQ instruction-issue PMC passes of tools/sq_passes.sh (diagnostic).

Reads gpurun_out/sq/p*/run_{counter_collection,kernel_trace}.csv (16384 x 64 KiB blocks, one
launch of each kernel) and writes profiles/sq_issue.json plus the raw counter CSVs
(profiles/<tag>_sq_p1.csv, <tag>_sq_p2.csv; tag = $PROFILE_TAG, default r2).  Derived per kernel:
  valu_pipe_busy = SQ_ACTIVE_INST_VALU (quad-cycles, summed over waves) / (SIMDs x cycles / 4)
  salu_busy, lds_busy: SQ_ACTIVE_INST_SCA / _LDS normalised the same way (per SIMD)
with cycles = kernel duration x 2.4 GHz (MI355X_MICROARCH.md: max clock 2400 MHz; SQ_ACTIVE_INST_*
count quad-cycles), 256 CUs x 4 SIMDs.
usage: python3 tools/sq_issue.py [nblocks]"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS, CLK = 1024, 2.4e9


def kind(name):
    return "lz4_encode_kernel" if "encode" in name else (("lz4_decode_coop_kernel" if "coop" in name else "lz4_decode_kernel") if "decode" in name else None)


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    base = os.environ.get("SQ_DIR", os.path.join(ROOT, "gpurun_out", "sq"))
    cnt = collections.defaultdict(dict)
    dur = collections.defaultdict(list)
    for p in sorted(glob.glob(os.path.join(base, "p*"))):
        for f in glob.glob(os.path.join(p, "*counter_collection.csv")):
            acc = collections.defaultdict(float)
            for r in csv.DictReader(open(f)):
                k = kind(r["Kernel_Name"])
                if k:
                    acc[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            for (k, c), v in acc.items():
                cnt[k][c] = v
            shutil.copy(f, os.path.join(ROOT, "profiles", "%s_sq_%s.csv" % (os.environ.get("PROFILE_TAG", "r2"), os.path.basename(p))))
        for f in glob.glob(os.path.join(p, "*kernel_trace.csv")):
            for r in csv.DictReader(open(f)):
                k = kind(r["Kernel_Name"])
                if k:
                    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    out = {"_note": __doc__.split("\n\n")[1].strip(), "blocks": nb}
    for k, c in cnt.items():
        t = sum(dur[k]) / max(len(dur[k]), 1)
        cyc = t * CLK
        units = nb * 1024 if "encode" in k else nb   # encoder: per 64-position step; decoder: per block
        out[k] = {
            "duration_ms": round(t * 1e3, 3),
            "valu_pipe_busy": round(c.get("SQ_ACTIVE_INST_VALU", 0) / (SIMDS * cyc / 4), 3),
            "salu_busy": round(c.get("SQ_ACTIVE_INST_SCA", 0) / (SIMDS * cyc / 4), 3),
            "lds_busy": round(c.get("SQ_ACTIVE_INST_LDS", 0) / (SIMDS * cyc / 4), 3),
            ("valu_insts_per_step" if "encode" in k else "valu_insts_per_block"):
                round(c.get("SQ_INSTS_VALU", 0) / units, 1),
            ("salu_insts_per_step" if "encode" in k else "salu_insts_per_block"):
                round(c.get("SQ_INSTS_SALU", 0) / units, 1),
            "counters": {n: v for n, v in sorted(c.items())},
        }
    with open(os.path.join(ROOT, "profiles", os.environ.get("SQ_JSON", "sq_issue.json")), "w") as f:
        json.dump(out, f, indent=1)
    for k in ("lz4_encode_kernel", "lz4_decode_kernel", "lz4_decode_coop_kernel"):
        if k in out:
            print(k, {a: b for a, b in out[k].items() if a != "counters"})


if __name__ == "__main__":
    main()
