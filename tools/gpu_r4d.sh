#!/bin/bash
# GPU box: gather-rate microbenchmark, memory-system passes (5 groups), config 5 A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/gather_rate > gpurun_out/gather_rate.json 2> gpurun_out/gather_rate.err
echo "gather rc=$?"; cat gpurun_out/gather_rate.json
bash tools/mem_passes.sh 16384
