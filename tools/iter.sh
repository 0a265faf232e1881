#!/bin/bash
# Quick GPU iteration: GPU parity tests, then kernel times of the listed variants.
# usage: bash tools/iter.sh [variant ...]   (variant "" = the product library)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/iter_pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/time_variants.sh "$@"
