#!/bin/bash
# usage: gpu_ab.sh NB ROUNDS variants...   (+ encoder tests of the first non-base variant via APE_LZ4_LIB)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$TESTV" ]; then
  APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_$TESTV.so timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/test_$TESTV.log 2>&1
  rc=$?; tail -3 gpurun_out/test_$TESTV.log; echo "tests($TESTV) rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python3 tools/ab_inproc.py "$@" 2>&1 | grep -v amdgpu.ids
