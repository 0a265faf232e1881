#!/bin/bash
# GPU box: the start-echo encoder test on the product and on a library rebuilt with the
# round-4 TFREE bug (positions 1..3 inserted; it must fail there), then the encoder A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_tfbug.so timeout -k 10 200 python -u -m pytest tests/test_gpu_encode.py -m gpu -q --timeout 120 --timeout-method thread -k "block_start or many_blocks" > gpurun_out/tfbug_tests.log 2>&1
echo "bug library (must fail): rc=$?"; tail -3 gpurun_out/tfbug_tests.log
bash tools/gpu_ab2.sh "$@"
