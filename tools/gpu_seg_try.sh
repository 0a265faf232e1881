#!/bin/bash
# Segment-parallel encoder try-out (GPU box): encoder parity suite with APE_LZ4_ENCODER=seg,
# then the bench at 65536 blocks with each encoder.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-seg1}
APE_LZ4_ENCODER=seg timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_enc_tests.log 2>&1
rc=$?; tail -30 gpurun_out/${TAG}_enc_tests.log; [ $rc -eq 0 ] || exit $rc
for E in seg chunk; do
  APE_LZ4_ENCODER=$E timeout -k 10 200 python3 -u bench.py --blocks 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-config2 --no-config5 > gpurun_out/${TAG}_bench_$E.json 2> gpurun_out/${TAG}_bench_$E.err || { tail -5 gpurun_out/${TAG}_bench_$E.err; exit 1; }
done
python3 -c "
import json
for f in ('seg','chunk'):
    d=json.loads(open('gpurun_out/${TAG}_bench_%s.json'%f).read().strip().splitlines()[-1]); print(f, d['value'], d['encode_ms'], d['decode_ms'], d['ratio'], d.get('verified'))
"
