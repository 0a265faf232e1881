#!/bin/bash
# Texture-path occupancy of the encoder (diagnostic): TA / TD busy vs GPU active and the
# L1 tag accesses, for the product encoder and APE_LZ4_ENCODER=v2, one PMC pass each.
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
NB=${1:-16384}
for v in v1 v2; do
  APE_LZ4_ENCODER=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TD_BUSY_avr GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/ta/$v -o run --output-format csv -- python3 tools/kernel_driver.py $NB 1 > gpurun_out/ta_$v.log 2>&1 || { echo "pass $v failed"; tail -5 gpurun_out/ta_$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for v in ("v1", "v2"):
    for f in glob.glob("gpurun_out/ta/%s/**/*counter_collection.csv" % v, recursive=True):
        d = {}
        for r in csv.DictReader(open(f)):
            if "encode" not in r["Kernel_Name"]: continue
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        print(v, {k: round(x, 1) for k, x in d.items()},
              "TA busy frac %.3f" % (d.get("TA_BUSY_avr", 0) / max(d.get("GRBM_GUI_ACTIVE", 1), 1)),
              "TD busy frac %.3f" % (d.get("TD_BUSY_avr", 0) / max(d.get("GRBM_GUI_ACTIVE", 1), 1)))
PY
