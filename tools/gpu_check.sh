set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -3 gpurun_out/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o run --output-format csv -- python3 tools/kernel_driver.py 65536 1 2 > gpurun_out/kt.log 2>&1 && cat gpurun_out/kt.log | tail -2 && find gpurun_out/kt -name '*kernel_stats.csv' | xargs cat | cut -c1-40,200-
