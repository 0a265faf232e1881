#!/bin/bash
# Full bench.py line + rocprofv3 kernel stats of the same command (round profile).
# usage: bash tools/gpu_bench.sh TAG
set -o pipefail
TAG=${1:-r2}
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --no-config2 --no-config5 > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err || exit 1
cat gpurun_out/bench_prof_$TAG.json
