#!/bin/bash
# Profile refresh at a commit (GPU box), in two calls that each fit gpurun's limit.
# Results land under gpurun_out/; tools/collect_profiles.sh TAG copies the common ones into
# profiles/.
#   part A: GPU parity suite + smoke, the bench line + rocprofv3 kernel stats of the same
#           command, SQ issue passes, PMC traffic passes (FETCH_SIZE, WRITE_SIZE, requests)
#   part B: memory-pipeline passes (TA/TD busy), phase timers, config 2 (rocprofv3 kernel
#           time + FETCH_SIZE / WRITE_SIZE passes of bench.py --rand4k), --stream, --e2e,
#           --sock-chained
#   usage: bash tools/gpu_refresh.sh A|B [TAG]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PART=${1:-A}
TAG=${2:-r6}
if [ "$PART" = A ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -20 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_$TAG.log
  timeout -k 10 200 python -u -m pytest tests/test_gpu_encode.py -m gpu -q -s -k acceleration --timeout 120 --timeout-method thread > gpurun_out/accel_$TAG.log 2>&1 || exit 1
  grep "ratio by acceleration" gpurun_out/accel_$TAG.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
  bash tools/gpu_bench.sh $TAG || exit 1
  bash tools/sq_passes.sh 16384 > gpurun_out/sq_$TAG.txt 2>&1 || { tail -5 gpurun_out/sq_$TAG.txt; exit 1; }
  bash tools/pmc_traffic.sh 65536 > gpurun_out/pmc_$TAG.txt 2>&1 || { tail -5 gpurun_out/pmc_$TAG.txt; exit 1; }
  cat gpurun_out/pmc_$TAG.txt
else
  bash tools/mem_passes.sh 16384 > gpurun_out/mem_$TAG.txt 2>&1 || { tail -5 gpurun_out/mem_$TAG.txt; exit 1; }
  timeout -k 10 300 python3 tools/phase_stats.py 16384 > gpurun_out/phase_$TAG.txt 2>&1 || { tail -5 gpurun_out/phase_$TAG.txt; exit 1; }
  # config 2: kernel time and HBM bytes of the decode-only 4 KiB random-block line
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_$TAG -o run --output-format csv -- python3 -u bench.py --rand4k > gpurun_out/rand4k_$TAG.json 2> gpurun_out/rand4k_$TAG.err || { tail -5 gpurun_out/rand4k_$TAG.err; exit 1; }
  cat gpurun_out/rand4k_$TAG.json
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/pmc_c2_$c -o run --output-format csv -- python3 bench.py --rand4k --steps 1 --warmup 0 > gpurun_out/pmc_c2_$c.log 2>&1 || { echo "config-2 pass $c failed"; tail -5 gpurun_out/pmc_c2_$c.log; exit 1; }
  done
  timeout -k 10 400 python3 -u bench.py --stream > gpurun_out/stream_$TAG.json 2> gpurun_out/stream_$TAG.err || exit 1
  timeout -k 10 300 python3 -u bench.py --e2e > gpurun_out/e2e_$TAG.json 2> gpurun_out/e2e_$TAG.err || exit 1
  timeout -k 10 400 python3 -u bench.py --sock-chained > gpurun_out/sockc_$TAG.json 2> gpurun_out/sockc_$TAG.err || exit 1
  cat gpurun_out/stream_$TAG.json gpurun_out/e2e_$TAG.json gpurun_out/sockc_$TAG.json
fi
