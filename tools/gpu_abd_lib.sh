#!/bin/bash
# GPU box: decoder/stream/frame/socket parity suites on a VARIANT library (APE_LZ4_LIB), then an
# interleaved in-process A/B (tools/ab_inproc.py).  usage: gpu_abd_lib.sh VARIANT NB ROUNDS v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
V=$1; shift
APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_stream.py tests/test_gpu_frames.py tests/test_sock.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abdl_tests.log 2>&1
rc=$?; tail -3 gpurun_out/abdl_tests.log; echo "tests ($V) rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/ab_inproc.py "$@" 2>&1 | grep -v amdgpu.ids
