#!/bin/bash
# Round-4 profile refresh at the final commit (GPU box).  Results land under gpurun_out/;
# tools/collect_profiles.sh r4 copies the common ones into profiles/.
#   bench line + rocprofv3 kernel stats of the same command, --sock-chained line,
#   SQ issue passes, PMC traffic passes (FETCH_SIZE, WRITE_SIZE, request sizes),
#   per-role encoder instruction counts (NOWALK / NOEMIT variants), phase timers,
#   request bytes at 8 encoder blocks per CU (8192-entry table), --stream/--rand4k/--e2e.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r4}
NB=65536
# the GPU parity suite and smoke() first (acceleration ratios printed into their own log)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -20 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_encode.py -m gpu -q -s -k acceleration --timeout 120 --timeout-method thread > gpurun_out/accel_$TAG.log 2>&1 || exit 1
grep "ratio by acceleration" gpurun_out/accel_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
bash tools/gpu_bench.sh $TAG || exit 1
# config-4 self-launch rehearsal: two ranks of `bench.py --gpus 2` on the one device
APE_BENCH_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus 2 --blocks 131072 > gpurun_out/rehearse2_$TAG.json 2> gpurun_out/rehearse2_$TAG.err || { tail -5 gpurun_out/rehearse2_$TAG.err; exit 1; }
cat gpurun_out/rehearse2_$TAG.json
timeout -k 10 400 python3 -u bench.py --sock-chained > gpurun_out/sockc_$TAG.json 2> gpurun_out/sockc_$TAG.err || exit 1
cat gpurun_out/sockc_$TAG.json
bash tools/sq_passes.sh 16384 > gpurun_out/sq_$TAG.txt 2>&1 || { tail -5 gpurun_out/sq_$TAG.txt; exit 1; }
bash tools/pmc_traffic.sh $NB > gpurun_out/pmc_$TAG.txt 2>&1 || { tail -5 gpurun_out/pmc_$TAG.txt; exit 1; }
NB=16384 bash tools/sq_variant.sh base nowalk noemit > gpurun_out/sq_roles_$TAG.txt 2>&1 || { tail -5 gpurun_out/sq_roles_$TAG.txt; exit 1; }
cat gpurun_out/sq_roles_$TAG.txt
timeout -k 10 300 python3 tools/phase_stats.py 16384 > gpurun_out/phase_$TAG.txt 2>&1 || { tail -5 gpurun_out/phase_$TAG.txt; exit 1; }
APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_t8192.so timeout -s KILL 240 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B -d gpurun_out/pmc_RDREQ_t8192 -o run --output-format csv -- python3 bench.py --blocks $NB --steps 1 --warmup 0 --no-cpu-baseline --no-config2 --no-config5 --verify-sample 0 > gpurun_out/pmc_RDREQ_t8192.log 2>&1 || { echo "t8192 pass failed"; tail -5 gpurun_out/pmc_RDREQ_t8192.log; exit 1; }
timeout -k 10 400 python3 -u bench.py --stream > gpurun_out/stream_$TAG.json 2> gpurun_out/stream_$TAG.err || exit 1
timeout -k 10 300 python3 -u bench.py --rand4k > gpurun_out/rand4k_$TAG.json 2> gpurun_out/rand4k_$TAG.err || exit 1
timeout -k 10 300 python3 -u bench.py --e2e > gpurun_out/e2e_$TAG.json 2> gpurun_out/e2e_$TAG.err || exit 1
cat gpurun_out/stream_$TAG.json gpurun_out/rand4k_$TAG.json gpurun_out/e2e_$TAG.json
