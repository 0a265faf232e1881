#!/bin/bash
# Config-4 rehearsal on ONE MI355X (GPU box): `bench.py --gpus 8` self-launches 8 ranks, all on
# device 0 (APE_BENCH_DEVICE=0), each with its contiguous share of the blocks.  Default: the
# configuration's full size, 1,048,576 x 64 KiB blocks = 131,072 per rank, ~24 GiB of device
# memory per rank (192 GiB in all).  It exercises the N > 1 path end to end; the 8-GPU number
# itself stays unmeasured (8 ranks share one GPU here).
#   usage: bash tools/gpu_rehearse8.sh TAG [BLOCKS]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r6}
NB=${2:-1048576}
APE_BENCH_DEVICE=0 timeout -k 10 900 python3 -u bench.py --gpus 8 --blocks $NB > gpurun_out/rehearse8_$TAG.json 2> gpurun_out/rehearse8_$TAG.err || { tail -20 gpurun_out/rehearse8_$TAG.err; exit 1; }
cat gpurun_out/rehearse8_$TAG.json
