#!/bin/bash
# Segment encoder quick check (GPU box): decode-verified debug cases on the product build,
# phase timers (stats build), and the seg-vs-chunk bench pair at 65536 blocks.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-q}
bash tools/gpu_seg_debug.sh base || exit 1
timeout -k 10 120 python3 tools/seg_phase.py 16384 1 || exit 1
for E in seg chunk; do
  APE_LZ4_ENCODER=$E timeout -k 10 200 python3 -u bench.py --blocks 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-config2 --no-config5 > gpurun_out/${TAG}_bench_$E.json 2> gpurun_out/${TAG}_bench_$E.err || { tail -5 gpurun_out/${TAG}_bench_$E.err; exit 1; }
done
python3 -c "
import json
for f in ('seg','chunk'):
    d=json.loads(open('gpurun_out/${TAG}_bench_%s.json'%f).read().strip().splitlines()[-1]); print(f, d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'ratio', d['ratio'], d.get('verified'))
"
