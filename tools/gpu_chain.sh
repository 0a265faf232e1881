#!/bin/bash
# GPU box: socket + chain parity tests, then the chained leg (and config 5).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sock.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/chain_tests.log 2>&1
rc=$?; tail -3 gpurun_out/chain_tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for t in 4 8; do
  APE_LZ4_CHAIN_THREADS=$t timeout -k 10 400 python -u bench.py --sock-chained ${CPU:---no-cpu-baseline} > gpurun_out/chain_t$t.json 2> gpurun_out/chain_t$t.err
  echo "chain t$t rc=$?"; python3 -c "import json;d=json.load(open('gpurun_out/chain_t$t.json'));print(d['value'],d['wall_s'],d['verified'],(d['cpu_baseline'] or {}).get('value'),json.dumps(d['split_ms']))"
done
timeout -k 10 300 python -u bench.py --sock --no-cpu-baseline > gpurun_out/sock_r4f.json 2> gpurun_out/sock_r4f.err
echo "sock rc=$?"; python3 -c "import json;d=json.load(open('gpurun_out/sock_r4f.json'));print(d['value'],d['wire_GBps'],d['ceiling_GBps'],d['ceiling_cold_GBps'])"
