#!/bin/bash
# GPU box: chain parity tests, then the chained-socket leg with the looping RX decode on / off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sock.py tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/chain_ab3_tests.log 2>&1 || { tail -8 gpurun_out/chain_ab3_tests.log; exit 1; }
tail -1 gpurun_out/chain_ab3_tests.log
for rep in 1 2 3; do
  for lp in 1 0; do
    APE_LZ4_CHAIN_LOOP=$lp timeout -k 10 200 python3 -u bench.py --sock-chained --no-cpu-baseline > gpurun_out/chainab3_${lp}_$rep.json 2> gpurun_out/chainab3_${lp}_$rep.err || { tail -3 gpurun_out/chainab3_${lp}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/chainab3_${lp}_$rep.json')); s=d['split_ms']; print('loop $lp rep $rep', d['value'], d['verified'], 'rx_gpu_wait', round(s['rx_gpu_wait_ms']), 'rx_read', round(s['rx_read_ms']), 'tx_gpu_wait', round(s['tx_gpu_wait_ms']))"
  done
done
