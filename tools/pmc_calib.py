#!/usr/bin/env python3
"""Summarise tools/fetch_calib.sh (gpurun_out/calib) -> profiles/fetch_calib.json: FETCH_SIZE
and the L2 memory-side read requests by size (TCC_EA0_RDREQ_32B/_64B/_128B) for access shapes
of known byte counts (tools/ubench/fetch_calib.hip), and the factor that turns FETCH_SIZE into
bytes for each shape."""
import csv
import json
import os
import shutil

D = "gpurun_out/calib"
known = json.loads(open(os.path.join(D, "known.json")).read().strip().splitlines()[-1])
names = {"stream16": "stream16", "gather<0>": "gather16", "gather<1>": "gather20",
         "gather<2>": "gather16h"}


def per_kernel(path):
    out = {}
    for r in csv.DictReader(open(path)):
        k = next((v for s, v in names.items() if s in r["Kernel_Name"]), None)
        if k:
            out.setdefault(k, {})
            out[k][r["Counter_Name"]] = out[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


fetch = per_kernel(os.path.join(D, "fetch", "run_counter_collection.csv"))
req = per_kernel(os.path.join(D, "req", "run_counter_collection.csv"))
dur = {}
for r in csv.DictReader(open(os.path.join(D, "trace", "run_kernel_stats.csv"))):
    k = next((v for s, v in names.items() if s in r["Name"]), None)
    if k:
        dur[k] = float(r["AverageNs"])
res = {"_note": "tools/ubench/fetch_calib.hip on one MI355X: every kernel reads a 4 GiB buffer "
                "(past the 256 MiB Infinity Cache), each line once (gather16h: each 64-B half "
                "once); FETCH_SIZE is reported in KB; request bytes = 32 n32 + 64 n64 + 128 n128 "
                "from TCC_EA0_RDREQ_{32B,64B,128B} (one --pmc pass of 4 TCC counters).  Raw: "
                "profiles/fetch_calib_*.csv",
       "known": known}
for k in ("stream16", "gather16", "gather20", "gather16h"):
    f = fetch[k]["FETCH_SIZE"] * 1024
    q = req[k]
    rb = 32 * q.get("TCC_EA0_RDREQ_32B", 0) + 64 * q.get("TCC_EA0_RDREQ_64B", 0) + \
        128 * q.get("TCC_EA0_RDREQ_128B", 0)
    acc = known[k]["accesses"]
    res[k] = {"fetch_size_bytes": round(f), "request_bytes": round(rb),
              "requests": round(q["TCC_EA0_RDREQ"]), "requests_128B": round(q.get("TCC_EA0_RDREQ_128B", 0)),
              "request_bytes_per_access": round(rb / acc, 2),
              "factor_request_over_fetch_size": round(rb / f, 4),
              "kernel_ns": dur.get(k), "request_GBps": round(rb / dur[k], 1) if dur.get(k) else None}
res["conclusion"] = ("every L2 miss is one 128-B request whatever the access shape (a 16-B "
                     "gather, a 16+4-B unaligned gather, 16 B per 64-B half): request bytes = "
                     "2 x FETCH_SIZE for all four shapes, so the encoder's scattered candidate "
                     "gathers take the same x2 as streaming reads; traffic is measured directly "
                     "as request bytes (tools/pmc_traffic.sh RDREQ pass)")
json.dump(res, open("profiles/fetch_calib.json", "w"), indent=1)
shutil.copy(os.path.join(D, "fetch", "run_counter_collection.csv"), "profiles/fetch_calib_fetch_size.csv")
shutil.copy(os.path.join(D, "req", "run_counter_collection.csv"), "profiles/fetch_calib_rdreq.csv")
shutil.copy(os.path.join(D, "trace", "run_kernel_stats.csv"), "profiles/fetch_calib_kernel_stats.csv")
print(json.dumps(res, indent=1))
