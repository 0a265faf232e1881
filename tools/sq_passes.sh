#!/bin/bash
# SQ instruction-mix / wait-state PMC passes over tools/kernel_driver.py (diagnostic).
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
NB=${1:-16384}
SQ=${SQ_DIR:-gpurun_out/sq}   # (APE_LZ4_LIB selects a variant library)
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
grep -o "SQ_[A-Z_0-9]*" gpurun_out/counters.txt | sort -u > gpurun_out/sq_counters.txt
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $SQ/p$i -o run --output-format csv -- python3 tools/kernel_driver.py $NB 1 > gpurun_out/sq_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sq_p$i.log; exit 1; }
done
SQ_DIR=$SQ python3 - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.environ['SQ_DIR'] + '/p*/*counter_collection.csv') + glob.glob(os.environ['SQ_DIR'] + '/p*/*/*counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        k = 'enc' if 'encode' in k else ('dec' if 'decode' in k else None)
        if k: agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in agg.items():
    print(k, {c: '%.4g' % v for c, v in sorted(d.items())})
PY
