#!/bin/bash
# GPU box: chained-socket leg over part counts (priorities on), and 4 parts with 8 hardware queues.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for p in 2 3 4 6; do
    APE_LZ4_CHAIN_THREADS=$p timeout -k 10 200 python3 -u bench.py --sock-chained --no-cpu-baseline > gpurun_out/chainab2_$p_$rep.json 2> gpurun_out/chainab2_$p_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/chainab2_$p_$rep.json')); s=d['split_ms']; print('parts $p rep $rep', d['value'], d['verified'], 'rx_gpu_wait', round(s['rx_gpu_wait_ms']), 'rx_read', round(s['rx_read_ms']))"
  done
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 -u bench.py --sock-chained --no-cpu-baseline > gpurun_out/chainab2_q8_$rep.json 2> gpurun_out/chainab2_q8_$rep.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/chainab2_q8_$rep.json')); s=d['split_ms']; print('parts 4 hwq 8 rep $rep', d['value'], d['verified'], 'rx_gpu_wait', round(s['rx_gpu_wait_ms']), 'rx_read', round(s['rx_read_ms']))"
done
