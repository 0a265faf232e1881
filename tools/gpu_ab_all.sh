set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_decode.py tests/test_gpu_stream.py tests/test_gpu_frames.py tests/test_sock.py tests/test_gpu_api.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_both_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ab_both_tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/ab_inproc.py "$@" 2>&1 | grep -v amdgpu.ids
