#!/bin/bash
# SQ instruction mix of the product encoder (v1) vs the three-role one (APE_LZ4_ENCODER=v2),
# two PMC passes each over tools/kernel_driver.py (diagnostic).
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
NB=${1:-16384}
for v in v2 v1; do
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
             "SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM" ; do
    i=$((i+1))
    APE_LZ4_ENCODER=$v timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/sqc/$v/p$i -o run --output-format csv -- python3 tools/kernel_driver.py $NB 1 > gpurun_out/sqc_${v}_p$i.log 2>&1 || { echo "pass $v $i failed"; tail -5 gpurun_out/sqc_${v}_p$i.log; exit 1; }
  done
done
python3 - $NB <<'PY'
import csv, glob, collections, sys
nb = int(sys.argv[1]); steps = 1028
for v in ("v2", "v1"):
    agg = collections.defaultdict(float)
    dur = []
    for f in glob.glob('gpurun_out/sqc/%s/p*/**/*counter_collection.csv' % v, recursive=True):
        for r in csv.DictReader(open(f)):
            if 'encode' in r['Kernel_Name']:
                agg[r['Counter_Name']] += float(r['Counter_Value'])
    for f in glob.glob('gpurun_out/sqc/%s/p*/**/*kernel_trace.csv' % v, recursive=True):
        for r in csv.DictReader(open(f)):
            if 'encode' in r['Kernel_Name']:
                dur.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
    per = {k: round(val / (nb * steps), 1) for k, val in sorted(agg.items())}
    print(v, "kernel ms", [round(d, 2) for d in dur], "per block-step:", per)
PY
