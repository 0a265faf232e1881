#!/bin/bash
# Kernel-time A/B of library variants (diagnostic): each variant runs REPS launches of the
# encoder and decoder on 16384 x 64 KiB blocks under rocprofv3 --kernel-trace, the variants
# interleaved ROUNDS times; prints the median kernel times per variant.
# usage: bash tools/ab_time.sh v1 v2 ...   (libapenetwork_amd/libape_lz4_amd_<v>.so)
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
ROUNDS=${ROUNDS:-3}; REPS=${REPS:-3}
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_$v.so timeout -k 10 120 rocprofv3 --kernel-trace \
      -d gpurun_out/ab_${v}_$r -o run --output-format csv -- python3 tools/kernel_driver.py 16384 1 $REPS \
      > gpurun_out/ab_${v}_$r.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab_${v}_$r.log; exit 1; }
  done
done
python3 - "$@" <<'PY'
import csv, glob, sys, statistics
for v in sys.argv[1:]:
    t = {'enc': [], 'dec': []}
    for f in glob.glob('gpurun_out/ab_%s_*/*kernel_trace.csv' % v) + glob.glob('gpurun_out/ab_%s_*/*/*kernel_trace.csv' % v):
        for r in csv.DictReader(open(f)):
            k = 'enc' if 'encode' in r['Kernel_Name'] else ('dec' if 'decode' in r['Kernel_Name'] else None)
            if k: t[k].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
    print('%-10s enc median %.3f ms (n=%d, min %.3f max %.3f)  dec median %.3f ms' % (
        v, statistics.median(t['enc']), len(t['enc']), min(t['enc']), max(t['enc']), statistics.median(t['dec'])))
PY
