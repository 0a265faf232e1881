#!/bin/bash
# HBM traffic of the codec kernels: rocprofv3 FETCH_SIZE and WRITE_SIZE in separate
# passes (MI355X_MICROARCH.md: they do not fit one pass) over a 65536-block bench run
# (4 GiB of input, well past the 256 MiB Infinity Cache), then per-block bytes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
NB=${1:-65536}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- python3 bench.py --blocks $NB --steps 1 --warmup 0 --no-cpu-baseline --no-config2 --no-config5 --verify-sample 0 > gpurun_out/pmc_$c.log 2>&1 || { echo "pass $c failed"; tail -5 gpurun_out/pmc_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $NB
