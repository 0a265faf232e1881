set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
APE_LZ4_ENCODER=seg timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/seg1_enc_tests.log 2>&1; echo "tests rc=$?"; tail -30 gpurun_out/seg1_enc_tests.log
APE_LZ4_ENCODER=seg timeout -k 10 200 python3 -u bench.py --blocks 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-config2 --no-config5 > gpurun_out/seg1_bench_seg.json 2> gpurun_out/seg1_bench_seg.err; echo "bench seg rc=$?"; tail -3 gpurun_out/seg1_bench_seg.err
APE_LZ4_ENCODER=chunk timeout -k 10 200 python3 -u bench.py --blocks 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-config2 --no-config5 > gpurun_out/seg1_bench_chunk.json 2> gpurun_out/seg1_bench_chunk.err; echo "bench chunk rc=$?"
python3 -c "
import json
for f in ('seg','chunk'):
    try:
        d=json.loads(open('gpurun_out/seg1_bench_%s.json'%f).read().strip().splitlines()[-1]); print(f, d['value'], d['encode_ms'], d['decode_ms'], d['ratio'], d.get('verified'))
    except Exception as e: print(f, 'ERR', e)
"
