#!/bin/bash
# GPU parity tests, then per-variant encoder/decoder kernel time + VALU/SALU counts.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/iter_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_$v.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/tv_$v -o run --output-format csv -- python3 tools/kernel_driver.py 16384 1 > gpurun_out/tv_$v.log 2>&1 || exit 1
  APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/pv_$v -o run --output-format csv -- python3 tools/kernel_driver.py 4096 1 > gpurun_out/pv_$v.log 2>&1 || exit 1
  python3 - "$v" <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
t = {}
for f in glob.glob('gpurun_out/tv_%s/*kernel_trace.csv' % v) + glob.glob('gpurun_out/tv_%s/*/*kernel_trace.csv' % v):
    for r in csv.DictReader(open(f)):
        k = 'enc' if 'encode' in r['Kernel_Name'] else ('dec' if 'decode' in r['Kernel_Name'] else None)
        if k: t[k] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
c = collections.defaultdict(float)
for f in glob.glob('gpurun_out/pv_%s/*counter_collection.csv' % v) + glob.glob('gpurun_out/pv_%s/*/*counter_collection.csv' % v):
    for r in csv.DictReader(open(f)):
        k = 'enc' if 'encode' in r['Kernel_Name'] else ('dec' if 'decode' in r['Kernel_Name'] else None)
        if k: c[(k, r['Counter_Name'])] += float(r['Counter_Value'])
steps = 4096 * 1024
log = open('gpurun_out/tv_%s.log' % v).read().strip().split('\n')
ok = [l for l in log if l.startswith('ok')]
print('%-10s enc %.2f ms  dec %.2f ms  | enc/step VALU %.0f SALU %.0f LDS %.0f | dec/blk VALU %.0f SALU %.0f | %s' % (
    v, t.get('enc', 0), t.get('dec', 0), c[('enc', 'SQ_INSTS_VALU')] / steps, c[('enc', 'SQ_INSTS_SALU')] / steps,
    c[('enc', 'SQ_INSTS_LDS')] / steps, c[('dec', 'SQ_INSTS_VALU')] / 4096, c[('dec', 'SQ_INSTS_SALU')] / 4096,
    ok[-1] if ok else log[-1][-60:]))
PY
done
