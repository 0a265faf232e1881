#!/bin/bash
# GPU box: encoder tests, then the A/B of the product encoder (round 1's, the default)
# vs the three-role v2 one (APE_LZ4_ENCODER=v2) on a reduced bench (131072 blocks);
# each step time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_api.py -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_enc.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_enc.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
B=${1:-131072}
APE_LZ4_ENCODER=v2 timeout -k 10 200 python -u bench.py --blocks $B --steps 3 --no-cpu-baseline --no-config2 --no-config5 \
    > gpurun_out/ab_v2.json 2> gpurun_out/ab_v2.err || exit 1
timeout -k 10 200 python -u bench.py --blocks $B --steps 3 --no-cpu-baseline --no-config5 \
    --no-config2 > gpurun_out/ab_v1.json 2> gpurun_out/ab_v1.err || exit 1
python3 - <<'PY'
import json
for v in ("v1", "v2"):
    d = json.load(open("gpurun_out/ab_%s.json" % v))
    print(v, "value", d["value"], "enc_ms", d["encode_ms"], "dec_ms", d["decode_ms"], "ratio", d["ratio"],
          "verified", d["verified"], "oracle", d["oracle_sample_ok"])
PY
