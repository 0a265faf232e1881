#!/usr/bin/env python3
"""Summarise tools/pmc_traffic.sh: HBM bytes per block and per launch of each codec kernel
-> profiles/pmc_traffic.json (read by bench.py for roofline.traffic)."""
import csv
import glob
import json
import os
import shutil
import sys

TAG = os.environ.get("PROFILE_TAG", "r2")

nb = int(sys.argv[1])
out = {"_note": ("rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE and --pmc TCC_EA0_RDREQ"
                 "{,_32B,_64B,_128B} in separate passes over `bench.py --blocks %d --steps 1 "
                 "--warmup 0` (input %.1f GiB, past the 256 MiB Infinity Cache).  fetch = read "
                 "request bytes (32 n32 + 64 n64 + 128 n128), measured; FETCH_SIZE x 2 beside it "
                 "(the calibrated factor for this access shape: profiles/fetch_calib.json -- "
                 "every L2 miss is a 128-B request, gathers included); KB -> bytes, per launch / "
                 "blocks.  Raw: profiles/%s_pmc_fetch_size.csv, _write_size.csv, _rdreq.csv"
                 % (nb, nb * 65536 / 2**30, TAG)),
       "blocks": nb}
vals = {}
for c, dst in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
    files = glob.glob("gpurun_out/pmc_%s/*counter_collection.csv" % c) + \
        glob.glob("gpurun_out/pmc_%s/*/*counter_collection.csv" % c)
    shutil.copy(files[0], "profiles/%s_pmc_%s.csv" % (TAG, c.lower()))
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            name = ("lz4_encode_kernel" if "encode" in k else
                    "lz4_decode_kernel" if "decode" in k else None)
            if name and r["Counter_Name"] == c:
                vals.setdefault(name, {}).setdefault(dst, []).append(float(r["Counter_Value"]))
req = {}
rfiles = glob.glob("gpurun_out/pmc_RDREQ/*counter_collection.csv") + \
    glob.glob("gpurun_out/pmc_RDREQ/*/*counter_collection.csv")
if rfiles:
    shutil.copy(rfiles[0], "profiles/%s_pmc_rdreq.csv" % TAG)
for f in rfiles:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        name = ("lz4_encode_kernel" if "encode" in k else
                "lz4_decode_kernel" if "decode" in k else None)
        w = {"TCC_EA0_RDREQ_32B": 32, "TCC_EA0_RDREQ_64B": 64, "TCC_EA0_RDREQ_128B": 128}.get(
            r["Counter_Name"])
        if name and w:
            req.setdefault(name, {}).setdefault(r["Dispatch_Id"], 0.0)
            req[name][r["Dispatch_Id"]] += w * float(r["Counter_Value"])
for name, d in vals.items():
    fs2 = sum(d.get("fetch", [0])) / max(len(d.get("fetch", [1])), 1) * 1024 * 2
    fetch = (sum(req[name].values()) / len(req[name])) if name in req else fs2
    write = sum(d.get("write", [0])) / max(len(d.get("write", [1])), 1) * 1024
    out[name] = {"fetch_bytes_per_block": round(fetch / nb, 1),
                 "fetch_size_x2_per_block": round(fs2 / nb, 1),
                 "fetch_source": "request bytes" if name in req else "FETCH_SIZE x 2",
                 "write_bytes_per_block": round(write / nb, 1),
                 "bytes_per_block": round((fetch + write) / nb, 1)}
json.dump(out, open("profiles/pmc_traffic.json", "w"), indent=1)
print(json.dumps(out, indent=1))
