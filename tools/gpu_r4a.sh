#!/bin/bash
# GPU box: -m gpu suite, smoke, the 2-rank self-launch rehearsal of `bench.py --gpus 2` on
# one device (with rank 0's cpu_baseline), then the default bench line.  Each step under its
# own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r4}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_$TAG.log; echo "smoke rc=$rc"
[ $rc -eq 0 ] || exit $rc
APE_BENCH_DEVICE=0 timeout -k 10 500 python -u bench.py --gpus 2 --blocks 131072 --steps 3 \
    --no-config2 --no-config5 > gpurun_out/rehearse2_$TAG.json 2> gpurun_out/rehearse2_$TAG.err
rc=$?; tail -3 gpurun_out/rehearse2_$TAG.err; echo "rehearse rc=$rc"; cut -c1-300 gpurun_out/rehearse2_$TAG.json
[ $rc -eq 0 ] || exit $rc
if [ "$2" = "bench" ]; then
  timeout -k 10 600 python -u bench.py --steps 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; tail -3 gpurun_out/bench_$TAG.err; echo "bench rc=$rc"; cut -c1-600 gpurun_out/bench_$TAG.json
fi
exit $rc
