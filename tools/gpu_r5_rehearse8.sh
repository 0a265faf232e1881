set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
APE_BENCH_DEVICE=0 timeout -k 10 700 python3 -u bench.py --gpus 8 --blocks 131072 > gpurun_out/rehearse8_r5.json 2> gpurun_out/rehearse8_r5.err || { tail -20 gpurun_out/rehearse8_r5.err; exit 1; }
cat gpurun_out/rehearse8_r5.json
