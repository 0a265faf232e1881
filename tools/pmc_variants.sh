#!/bin/bash
# VALU/SALU counts and kernel time of the encoder for experimental library variants (diagnostic).
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/pv_$v -o run --output-format csv -- python3 tools/kernel_driver.py 4096 1 > gpurun_out/pv_$v.log 2>&1 || exit 1
  echo "== $v $(tail -1 gpurun_out/pv_$v.log)"
  python3 tools/pmc_sum.py gpurun_out/pv_$v 4096 | grep encode
  python3 -c "
import csv,glob
for f in glob.glob('gpurun_out/pv_$v/*/run_kernel_trace.csv'):
    for r in csv.DictReader(open(f)):
        if 'encode' in r['Kernel_Name']: print('   encode kernel us', (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000)
"
done
