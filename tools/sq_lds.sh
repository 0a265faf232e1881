#!/bin/bash
# LDS PMC pass (diagnostic): unaligned stalls, bank / address conflicts and LDS activity of the
# encode and decode kernels over tools/kernel_driver.py (one rocprofv3 --pmc run).
#   bash tools/sq_lds.sh [nblocks]      (APE_LZ4_LIB selects a variant library)
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
NB=${1:-16384}
OUT=${SQ_DIR:-gpurun_out/sqlds}
rm -rf $OUT
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_LDS -d $OUT -o run --output-format csv -- python3 tools/kernel_driver.py $NB 1 > gpurun_out/sqlds.log 2>&1 || { echo "pass failed"; tail -5 gpurun_out/sqlds.log; exit 1; }
OUT=$OUT NB=$NB python3 - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.environ['OUT'] + '/*counter_collection.csv') + glob.glob(os.environ['OUT'] + '/*/*counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        k = 'enc' if 'encode' in k else ('dec' if 'decode' in k else None)
        if k: agg[k][r['Counter_Name']] += float(r['Counter_Value'])
nb = float(os.environ['NB'])
for k, d in agg.items():
    print(k, ' '.join('%s=%.0f' % (c.replace('SQ_', ''), v / nb) for c, v in sorted(d.items())), '(per block)')
PY
