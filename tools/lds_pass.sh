#!/bin/bash
# LDS stall counters of the codec kernels (diagnostic), one PMC pass over NB blocks.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
NB=${NB:-16384}
rm -rf gpurun_out/lds
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS -d gpurun_out/lds -o run --output-format csv -- python3 tools/kernel_driver.py $NB 1 > gpurun_out/lds.log 2>&1 || { tail -5 gpurun_out/lds.log; exit 1; }
python3 - $NB <<'PY'
import csv, glob, collections, sys
nb = int(sys.argv[1])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
dur = {}
for f in glob.glob('gpurun_out/lds/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        k = 'enc' if 'encode' in k else ('dec' if 'decode' in k else None)
        if k: agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in agg.items():
    print(k, {c: '%.4g' % (v / nb) for c, v in sorted(d.items())}, "(per block)")
PY
