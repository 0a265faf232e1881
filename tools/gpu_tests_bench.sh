#!/bin/bash
# GPU box: the -m gpu suite, smoke(), then the default bench line (one call, each step
# under its own time limit; stops at the first failure).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; echo "smoke rc=$rc"
[ $rc -eq 0 ] || exit $rc
if [ "$1" = "bench" ]; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; tail -3 gpurun_out/bench.err; echo "bench rc=$rc"; cat gpurun_out/bench.json | cut -c1-600
fi
exit $rc
