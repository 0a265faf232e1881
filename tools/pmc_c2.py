#!/usr/bin/env python3
"""pmc_c2.py -- DESIGN TOOL: config 2's decode kernel HBM bytes per launch from the
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `bench.py --rand4k --steps 1 --warmup 0`
(tools/gpu_refresh.sh B) next to its algorithmic bytes and rocprofv3 kernel time.
FETCH_SIZE is corrected x2 (profiles/fetch_calib.json: every request counts 64 B on gfx950,
the codec's requests are 128 B); WRITE_SIZE as reported.  KB = 1024 B.
  python3 tools/pmc_c2.py TAG   -> profiles/TAG_config2_pmc.json"""
import csv
import json
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r5"
out = {"_note": __doc__.strip()}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = [r for r in csv.DictReader(open("gpurun_out/pmc_c2_%s/run_counter_collection.csv" % c))
            if "lz4_decode_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c]
    v = [float(r["Counter_Value"]) * 1024.0 for r in rows]
    out[c] = {"launches": len(v), "bytes_per_launch_raw": v[-1] if v else None}
f = out["FETCH_SIZE"]["bytes_per_launch_raw"] * 2.0
w = out["WRITE_SIZE"]["bytes_per_launch_raw"]
line = json.load(open("gpurun_out/rand4k_%s.json" % tag))
alg = line["roofline"]["bytes_per_launch"]
ms = [float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open("gpurun_out/prof_c2_%s/run_kernel_stats.csv" % tag))
      if "lz4_decode_kernel" in r["Name"]]
out.update({"fetch_bytes_per_launch": f, "write_bytes_per_launch": w, "traffic_bytes": f + w,
            "algorithmic_bytes": alg, "traffic_over_algorithmic": round((f + w) / alg, 3),
            "rocprof_avg_launch_ms": ms[0] if ms else None,
            "bench_event_avg_launch_ms": line["roofline"]["avg_launch_ms"],
            "achieved_GBps_rocprof": round(alg / (ms[0] * 1e-3) / 1e9, 1) if ms else None,
            "bench_line": {k: line[k] for k in ("value", "unit", "verified")}})
json.dump(out, open("profiles/%s_config2_pmc.json" % tag, "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "_note"}, indent=1))
