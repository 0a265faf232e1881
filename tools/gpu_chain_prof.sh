#!/bin/bash
# GPU box: kernel + memory-copy trace of the chained-socket leg (where its GPU time goes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/chainprof -o run --output-format csv -- python3 -u bench.py --sock-chained --no-cpu-baseline > gpurun_out/chainprof.json 2> gpurun_out/chainprof.err || { tail -5 gpurun_out/chainprof.err; exit 1; }
cat gpurun_out/chainprof.json
for f in gpurun_out/chainprof/*kernel_stats.csv gpurun_out/chainprof/*/*kernel_stats.csv gpurun_out/chainprof/*memory_copy_stats.csv gpurun_out/chainprof/*/*memory_copy_stats.csv; do [ -f "$f" ] && { echo "== $f"; cut -c1-200 "$f" | head -12; }; done
exit 0
