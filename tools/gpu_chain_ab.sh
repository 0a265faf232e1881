#!/bin/bash
# GPU box: chained-socket leg A/B over environment settings (stream priorities, parts),
# alternating, two runs each; prints value and the RX split per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sock.py -m gpu -x -q --timeout 120 --timeout-method thread -k chain > gpurun_out/chain_ab_tests.log 2>&1 || { tail -5 gpurun_out/chain_ab_tests.log; exit 1; }
tail -1 gpurun_out/chain_ab_tests.log
for rep in 1 2; do
  for cfg in "1 4" "0 4" "1 8" "0 8"; do
    set -- $cfg
    APE_LZ4_CHAIN_PRIO=$1 APE_LZ4_CHAIN_THREADS=$2 timeout -k 10 200 python3 -u bench.py --sock-chained --no-cpu-baseline > gpurun_out/chainab_$1_$2_$rep.json 2> gpurun_out/chainab_$1_$2_$rep.err || { tail -3 gpurun_out/chainab_$1_$2_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/chainab_$1_$2_$rep.json')); s=d['split_ms']; print('prio $1 parts $2 rep $rep', d['value'], d['verified'], 'rx_total', round(s['rx_total_ms']), 'rx_gpu_wait', round(s['rx_gpu_wait_ms']), 'rx_read', round(s['rx_read_ms']), 'tx_gpu_wait', round(s['tx_gpu_wait_ms']))"
  done
done
