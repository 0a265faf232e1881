set -o pipefail
TAG=r2
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/sq_passes.sh 16384 > gpurun_out/sq_$TAG.txt 2>&1 || { tail -5 gpurun_out/sq_$TAG.txt; exit 1; }
NB=65536
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- python3 bench.py --blocks $NB --steps 1 --warmup 0 --no-cpu-baseline --no-config2 --no-config5 --verify-sample 0 > gpurun_out/pmc_$c.log 2>&1 || { echo "pass $c failed"; tail -5 gpurun_out/pmc_$c.log; exit 1; }
done
timeout -k 10 400 python3 -u bench.py --stream > gpurun_out/stream_$TAG.json 2> gpurun_out/stream_$TAG.err || exit 1
timeout -k 10 300 python3 -u bench.py --rand4k > gpurun_out/rand4k_$TAG.json 2> gpurun_out/rand4k_$TAG.err || exit 1
timeout -k 10 300 python3 -u bench.py --e2e > gpurun_out/e2e_$TAG.json 2> gpurun_out/e2e_$TAG.err || exit 1
timeout -k 10 300 python3 -u bench.py --sock > gpurun_out/sock_$TAG.json 2> gpurun_out/sock_$TAG.err || exit 1
cat gpurun_out/stream_$TAG.json gpurun_out/rand4k_$TAG.json gpurun_out/e2e_$TAG.json gpurun_out/sock_$TAG.json | cut -c1-300
