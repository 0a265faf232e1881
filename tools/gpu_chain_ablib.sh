#!/bin/bash
# GPU box: chain parity tests on the product, then the chained-socket leg alternating between
# library variants (usage: gpu_chain_ablib.sh v1 v2 ...; "base" = the product), three runs each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sock.py tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/chain_ablib_tests.log 2>&1 || { tail -8 gpurun_out/chain_ablib_tests.log; exit 1; }
tail -1 gpurun_out/chain_ablib_tests.log
for rep in 1 2 3; do
  for v in "$@"; do
    lib=$PWD/libapenetwork_amd/libape_lz4_amd_$v.so; [ "$v" = base ] && lib=$PWD/libapenetwork_amd/libape_lz4_amd.so
    APE_LZ4_LIB=$lib timeout -k 10 200 python3 -u bench.py --sock-chained --no-cpu-baseline > gpurun_out/chainablib_${v}_$rep.json 2> gpurun_out/chainablib_${v}_$rep.err || { tail -3 gpurun_out/chainablib_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/chainablib_${v}_$rep.json')); s=d['split_ms']; print('$v rep $rep', d['value'], d['verified'], {k: round(x) for k, x in s.items()})"
  done
done
