#!/bin/bash
# Memory-path counters of the encoder (diagnostic), product (v1) vs APE_LZ4_ENCODER=v2:
# pass 1 L1->L2 requests and L2 hits/misses/busy, pass 2 the texture-address stalls.
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
NB=${1:-16384}
i=0
for grp in "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum TCC_BUSY_avr GRBM_GUI_ACTIVE" \
           "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for v in v1 v2; do
    APE_LZ4_ENCODER=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/mem/$v/p$i -o run --output-format csv -- python3 tools/kernel_driver.py $NB 1 > gpurun_out/mem_${v}_$i.log 2>&1 || { echo "pass $v $i failed"; tail -5 gpurun_out/mem_${v}_$i.log; exit 1; }
  done
done
python3 - $NB <<'PY'
import csv, glob, sys
nb = int(sys.argv[1])
for v in ("v1", "v2"):
    d = {}
    for f in glob.glob("gpurun_out/mem/%s/**/*counter_collection.csv" % v, recursive=True):
        for r in csv.DictReader(open(f)):
            if "encode" not in r["Kernel_Name"]: continue
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    steps = nb * 1028.0
    print(v, {k: (round(x / steps, 2) if "GRBM" not in k and "BUSY" not in k else round(x, 1)) for k, x in d.items()}, "(per block-step)")
PY
