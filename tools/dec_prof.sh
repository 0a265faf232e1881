#!/bin/bash
# GPU box (diagnostic): decoder phase stats (stats build) and the SQ instruction passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/phase_stats.py ${NB:-16384} > gpurun_out/phase.log 2>&1
rc=$?; cat gpurun_out/phase.log | grep -v "^W2"; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/sq
timeout -k 10 400 bash tools/sq_passes.sh ${NB:-16384} 2>&1 | grep -v "^W2" | cut -c1-2000
