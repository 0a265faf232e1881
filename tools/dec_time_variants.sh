#!/bin/bash
# Decode/encode kernel times of library variants over NB blocks (diagnostic):
# tools/dec_time_variants.sh base v1 v2 ...   ("base" = the product library)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
for v in "$@"; do
  lib=$PWD/libapenetwork_amd/libape_lz4_amd_$v.so
  [ "$v" = base ] && lib=$PWD/libapenetwork_amd/libape_lz4_amd.so
  rm -rf gpurun_out/tv_$v
  APE_LZ4_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/tv_$v -o run --output-format csv -- python3 tools/kernel_driver.py ${NB:-65536} 1 2 > gpurun_out/tv_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/tv_$v.log; exit 1; }
  python3 - $v <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
d = collections.defaultdict(list)
for f in glob.glob('gpurun_out/tv_%s/**/*kernel_trace.csv' % v, recursive=True):
    for r in csv.DictReader(open(f)):
        k = 'enc' if 'encode' in r['Kernel_Name'] else ('dec' if 'decode' in r['Kernel_Name'] else None)
        if k: d[k].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
ok = [l for l in open('gpurun_out/tv_%s.log' % v).read().split('\n') if l.startswith('ok')]
print(v, {k: [round(x, 3) for x in vv] for k, vv in d.items()}, ok)
PY
done
