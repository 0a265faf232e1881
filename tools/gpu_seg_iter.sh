#!/bin/bash
# Segment encoder iteration (GPU box): the encoder parity suite with APE_LZ4_ENCODER=seg,
# its phase timers (stats build), then the seg / chunk bench pair at 65536 blocks.  (The
# stage-2 edge test bounds the size at 1.03 x the reference's on boundary-copy data, which
# the segment encoder exceeds: 277145 vs 264236 B.)
#   bash tools/gpu_seg_iter.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-it}
APE_LZ4_ENCODER=seg timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -m gpu -x -q -k "not stage2_measurement_edges" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_enc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_enc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/seg_phase.py 16384 1 > gpurun_out/${TAG}_phase.txt 2>&1 || { tail -5 gpurun_out/${TAG}_phase.txt; exit 1; }
cat gpurun_out/${TAG}_phase.txt
for E in seg chunk; do
  APE_LZ4_ENCODER=$E timeout -k 10 200 python3 -u bench.py --blocks 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-config2 --no-config5 > gpurun_out/${TAG}_bench_$E.json 2> gpurun_out/${TAG}_bench_$E.err || { tail -5 gpurun_out/${TAG}_bench_$E.err; exit 1; }
done
python3 -c "
import json
for f in ('seg','chunk'):
    d=json.loads(open('gpurun_out/${TAG}_bench_%s.json'%f).read().strip().splitlines()[-1]); print(f, d['value'], 'enc', d['encode_ms'], 'dec', d['decode_ms'], 'ratio', d['ratio'], d.get('verified'))
"
