#!/bin/bash
# SQ / LDS PMC passes of the segment encoder (diagnostic): instruction mix, waits, LDS
# conflicts and stalls, one counter group per rocprofv3 run over tools/kernel_driver.py.
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
NB=${1:-16384}
SQ=${SQ_DIR:-gpurun_out/sqs}
export APE_LZ4_ENCODER=seg
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_LDS_DATA_FIFO_FULL" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $SQ/p$i -o run --output-format csv -- python3 tools/kernel_driver.py $NB 1 > gpurun_out/sqs_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sqs_p$i.log; exit 1; }
done
SQ_DIR=$SQ NB=$NB python3 - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(float)
for f in glob.glob(os.environ['SQ_DIR'] + '/p*/*counter_collection.csv') + glob.glob(os.environ['SQ_DIR'] + '/p*/*/*counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'encode_seg' in r['Kernel_Name']:
            agg[r['Counter_Name']] += float(r['Counter_Value'])
nb = float(os.environ['NB'])
for c, v in sorted(agg.items()):
    print('%-28s %14.4g  per block %12.1f' % (c, v, v / nb))
PY
