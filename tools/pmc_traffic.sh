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
# request sizes of the same run (true bytes = 32 n32 + 64 n64 + 128 n128; FETCH_SIZE tallies
# every request at 64 B on gfx950: tools/ubench/fetch_calib.hip)
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B -d gpurun_out/pmc_RDREQ -o run --output-format csv -- python3 bench.py --blocks $NB --steps 1 --warmup 0 --no-cpu-baseline --no-config2 --no-config5 --verify-sample 0 > gpurun_out/pmc_RDREQ.log 2>&1 || { echo "pass RDREQ failed"; tail -5 gpurun_out/pmc_RDREQ.log; exit 1; }
python3 tools/pmc_traffic.py $NB
