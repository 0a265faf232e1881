#!/bin/bash
# GPU box: acceleration ratios (test_acceleration prints GPU vs reference) for the product and
# the variant that keeps the in-chunk candidate at acceleration > 1; then the chain tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for lib in libape_lz4_amd.so libape_lz4_amd_accl.so; do
  APE_LZ4_LIB=$PWD/libapenetwork_amd/$lib timeout -k 10 120 python -u -m pytest tests/test_gpu_encode.py -m gpu -q -s -k acceleration --timeout 100 --timeout-method thread > gpurun_out/accel_$lib.log 2>&1
  echo "accel $lib rc=$?"; grep "ratio by acceleration" gpurun_out/accel_$lib.log
done
timeout -k 10 300 python -u -m pytest tests/test_sock.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/sock_tests.log 2>&1
echo "sock tests rc=$?"; tail -3 gpurun_out/sock_tests.log
timeout -k 10 300 python -u bench.py --sock-chained > gpurun_out/chain_r4b.json 2> gpurun_out/chain_r4b.err
echo "chain rc=$?"; cut -c1-600 gpurun_out/chain_r4b.json; tail -3 gpurun_out/chain_r4b.err
timeout -k 10 120 ./tools/ubench/host_sock > gpurun_out/host_sock.json 2> gpurun_out/host_sock.err
echo "host_sock rc=$?"; cat gpurun_out/host_sock.json
timeout -k 10 400 python3 tools/ab_inproc.py 131072 7 base t6432w8 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_t6432w8.log
echo "ab rc=$?"; cat gpurun_out/ab_t6432w8.log
timeout -k 10 300 python -u bench.py --sock > gpurun_out/sock_r4a.json 2> gpurun_out/sock_r4a.err
echo "sock rc=$?"; cut -c1-900 gpurun_out/sock_r4a.json
