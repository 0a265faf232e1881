#!/bin/bash
# GPU box: -m gpu suite, then the 2-rank rehearsal of `bench.py --gpus 2` on one device.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
grep "one-shot n=" gpurun_out/pytest_gpu.log | head -3
python -u -m pytest tests/test_gpu_api.py -m gpu -q -s -k latency --timeout 300 > gpurun_out/latency.log 2>&1; grep "one-shot" gpurun_out/latency.log
APE_BENCH_DEVICE=0 timeout -k 10 400 python -u bench.py --gpus 2 --blocks 131072 --steps 3 \
    > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
rc=$?; tail -3 gpurun_out/rehearse2.err; echo "rehearse rc=$rc"; cut -c1-400 gpurun_out/rehearse2.json
[ $rc -eq 0 ] || exit $rc
exit 0
