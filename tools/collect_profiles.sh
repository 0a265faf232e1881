#!/bin/bash
# Copy a refresh_profiles.sh run's results from gpurun_out/ into profiles/ (run here).
set -e
TAG=${1:-r1}
cd "$(dirname "$0")/.."
cp gpurun_out/bench_$TAG.json profiles/r1_bench.json
cp gpurun_out/prof_$TAG/run_kernel_stats.csv profiles/r1_kernel_stats.csv
cp gpurun_out/stream_$TAG.json profiles/r1_stream.json
cp gpurun_out/rand4k_$TAG.json profiles/r1_rand4k.json
cp gpurun_out/e2e_$TAG.json profiles/r1_e2e.json
python3 tools/sq_issue.py 16384
python3 tools/pmc_traffic.py 65536
