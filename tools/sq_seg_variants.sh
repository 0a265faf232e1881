#!/bin/bash
# VALU / SALU / LDS instructions per block and kernel time of segment-encoder variant builds
# (diagnostic): usage sq_seg_variants.sh v1 v2 ...  ("base" = the product library)
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
export APE_LZ4_ENCODER=seg
NB=16384
for V in "$@"; do
  L=$PWD/libapenetwork_amd/libape_lz4_amd_$V.so; [ "$V" = base ] && L=$PWD/libapenetwork_amd/libape_lz4_amd.so
  D=gpurun_out/sqv_$V
  APE_LZ4_LIB=$L timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $D -o run --output-format csv -- python3 tools/kernel_driver.py $NB 1 > $D.log 2>&1 || { echo "$V failed"; tail -5 $D.log; exit 1; }
  D=$D NB=$NB V=$V python3 - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(float); dur = []
for f in glob.glob(os.environ['D'] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'encode_seg' in r['Kernel_Name']: agg[r['Counter_Name']] += float(r['Counter_Value'])
for f in glob.glob(os.environ['D'] + '/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'encode_seg' in r['Kernel_Name']: dur.append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
nb = float(os.environ['NB'])
print('%-10s %s  kernel %.3f ms' % (os.environ['V'], '  '.join('%s %.1fK' % (c.replace('SQ_INSTS_', '').replace('SQ_', ''), v / nb / 1e3) for c, v in sorted(agg.items())), min(dur) if dur else -1))
PY
done
