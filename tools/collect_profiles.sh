#!/bin/bash
# Copy a tools/gpu_refresh.sh run's results from gpurun_out/ into profiles/ (run here).
set -e
TAG=${1:-r2}
cd "$(dirname "$0")/.."
cp gpurun_out/bench_$TAG.json profiles/${TAG}_bench.json
cp gpurun_out/prof_$TAG/run_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
for f in stream rand4k e2e sock; do
  [ -f gpurun_out/${f}_$TAG.json ] && cp gpurun_out/${f}_$TAG.json profiles/${TAG}_$f.json
done
PROFILE_TAG=$TAG python3 tools/sq_issue.py 16384
PROFILE_TAG=$TAG python3 tools/pmc_traffic.py 65536
