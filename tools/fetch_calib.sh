#!/bin/bash
# GPU box: FETCH_SIZE calibration for the encoder's access shape (tools/ubench/fetch_calib.hip):
# one --pmc pass per counter group, kernel durations from the same runs.  Results under
# gpurun_out/calib/; tools/pmc_calib.py turns them into profiles/fetch_calib.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/calib
B=tools/ubench/fetch_calib
[ -x $B ] || /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o $B tools/ubench/fetch_calib.hip || exit 1
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/calib/avail.txt 2>&1 || echo "list-avail rc=$?"
grep -o "TCC_EA0_RD[A-Z0-9_]*\|TCC_BUBBLE[A-Z0-9_]*\|TCC_EA_RD[A-Z0-9_]*" gpurun_out/calib/avail.txt | sort -u > gpurun_out/calib/tcc_rd.txt || true
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/calib/fetch -o run --output-format csv -- ./$B > gpurun_out/calib/known.json 2> gpurun_out/calib/fetch.err || { echo "FETCH pass failed"; tail -3 gpurun_out/calib/fetch.err; exit 1; }
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d gpurun_out/calib/trace -o run --output-format csv -- ./$B > /dev/null 2> gpurun_out/calib/trace.err || { echo "trace pass failed"; exit 1; }
# request sizes: 4 TCC counters, one pass (the TCC block's limit)
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B -d gpurun_out/calib/req -o run --output-format csv -- ./$B > /dev/null 2> gpurun_out/calib/req.err || { echo "req pass failed"; tail -3 gpurun_out/calib/req.err; exit 1; }
cat gpurun_out/calib/known.json
find gpurun_out/calib -name "*counter_collection.csv" | head
