#!/bin/bash
# GPU box: full -m gpu suite, config 5 and the chained-socket leg, memory-system passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r4c.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_r4c.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --sock > gpurun_out/sock_r4c.json 2> gpurun_out/sock_r4c.err
echo "sock rc=$?"; cut -c1-1500 gpurun_out/sock_r4c.json
timeout -k 10 400 python -u bench.py --sock-chained > gpurun_out/chain_r4c.json 2> gpurun_out/chain_r4c.err
echo "chain rc=$?"; cut -c1-2000 gpurun_out/chain_r4c.json; tail -3 gpurun_out/chain_r4c.err
bash tools/mem_passes.sh 16384
