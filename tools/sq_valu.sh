#!/bin/bash
# VALU issue occupancy counters for the encoder / decoder (diagnostic).
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
V=${1:-}
[ -n "$V" ] && export APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_$V.so
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_CYCLES SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_SALU SQ_INSTS_SALU SQ_WAVE_CYCLES -d gpurun_out/sqv -o run --output-format csv -- python3 tools/kernel_driver.py 16384 1 > gpurun_out/sqv.log 2>&1 || { tail -5 gpurun_out/sqv.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob('gpurun_out/sqv/*counter_collection.csv') + glob.glob('gpurun_out/sqv/*/*counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        k = 'enc' if 'encode' in k else ('dec' if 'decode' in k else None)
        if k: agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in agg.items():
    print(k, {c: '%.4g' % v for c, v in sorted(d.items())})
PY
