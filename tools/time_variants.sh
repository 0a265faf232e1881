#!/bin/bash
# Kernel times (rocprofv3 kernel trace) of library variants on tools/kernel_driver.py (diagnostic).
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_$v.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/tv_$v -o run --output-format csv -- python3 tools/kernel_driver.py ${NB:-16384} 1 > gpurun_out/tv_$v.log 2>&1 || exit 1
  python3 -c "
import csv,glob
d={}
for f in glob.glob('gpurun_out/tv_$v/*kernel_trace.csv') + glob.glob('gpurun_out/tv_$v/*/*kernel_trace.csv'):
    for r in csv.DictReader(open(f)):
        k='enc' if 'encode' in r['Kernel_Name'] else ('dec' if 'decode' in r['Kernel_Name'] else None)
        if k: d[k]=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
print('$v', d, [l for l in open('gpurun_out/tv_$v.log').read().split('\n') if l.startswith('ok')])
"
done
