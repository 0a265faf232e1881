#!/bin/bash
# GPU box (diagnostic iteration): decoder parity tests, then kernel times of one
# encode + decode launch over NB blocks (rocprofv3 kernel trace + stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_decode.py tests/test_gpu_frames.py tests/test_gpu_stream.py}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pt_dec.log 2>&1
rc=$?; tail -15 gpurun_out/pt_dec.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/kt
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o run --output-format csv \
    -- python3 tools/kernel_driver.py ${NB:-65536} 1 2 > gpurun_out/kt.log 2>&1
rc=$?; tail -2 gpurun_out/kt.log; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find gpurun_out/kt -name '*kernel_stats.csv' | xargs cat | cut -d, -f1-8
