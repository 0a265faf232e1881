#!/bin/bash
# Decoder change check (GPU box): decode/frame/stream parity suites, then a bench line with the
# config-2 leg (16384 x 64 KiB headline blocks: decode_ms) ; stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-d}
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_frames.py tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_dec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_dec_tests.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/${TAG}_dec_tests.log; exit $rc; }
timeout -k 10 300 python3 -u bench.py --blocks 131072 --steps 3 --warmup 1 --no-cpu-baseline --no-config5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); c=d.get('config2') or {}
print('headline', d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], '| config2', c.get('value'), c.get('ms_per_step') or c.get('decode_ms'), c.get('roofline', {}).get('frac') if isinstance(c.get('roofline'), dict) else '')
"
