#!/bin/bash
# GPU box, round 4: tests + smoke + 2-rank rehearsal + bench (tools/gpu_r4a.sh), the
# acceleration ratios of the product and the in-chunk-candidate variant, the chained-socket
# leg, FETCH calibration.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_r4a.sh r4a bench || exit $?
for lib in libape_lz4_amd.so libape_lz4_amd_accl.so; do
  APE_LZ4_LIB=$PWD/libapenetwork_amd/$lib timeout -k 10 120 python -u -m pytest tests/test_gpu_encode.py -m gpu -q -s -k acceleration --timeout 100 --timeout-method thread > gpurun_out/accel_$lib.log 2>&1
  echo "accel $lib rc=$?"; grep "ratio by acceleration" gpurun_out/accel_$lib.log
done
timeout -k 10 300 python -u bench.py --sock-chained > gpurun_out/chain_r4a.json 2> gpurun_out/chain_r4a.err
echo "chain rc=$?"; cut -c1-700 gpurun_out/chain_r4a.json; tail -3 gpurun_out/chain_r4a.err
bash tools/fetch_calib.sh
