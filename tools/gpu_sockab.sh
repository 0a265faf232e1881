#!/bin/bash
# GPU box: config 5 A/B on one box -- the product vs the round-3-style socket loop
# (libape_lz4_amd_oldsock.so: two slots, D2H of the frames), alternating, 2 runs each; then the
# chained leg.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  for v in base oldsock; do
    if [ $v = base ]; then L=$PWD/libapenetwork_amd/libape_lz4_amd.so; else L=$PWD/libapenetwork_amd/libape_lz4_amd_$v.so; fi
    APE_LZ4_LIB=$L timeout -k 10 300 python -u bench.py --sock --no-cpu-baseline > gpurun_out/sockab_${v}_$i.json 2> gpurun_out/sockab_${v}_$i.err
    echo "$v $i rc=$?"; python3 -c "import json;d=json.load(open('gpurun_out/sockab_${v}_$i.json'));print(d['value'],d['wire_GBps'],d['ceiling_GBps'],d['ceiling_cold_GBps'],json.dumps(d['split_ms']))"
  done
done
timeout -k 10 400 python -u bench.py --sock-chained > gpurun_out/chain_r4e.json 2> gpurun_out/chain_r4e.err
echo "chain rc=$?"; python3 -c "import json;d=json.load(open('gpurun_out/chain_r4e.json'));print(d['value'],d['wall_s'],d['verified'],d['cpu_baseline']['value'],json.dumps(d['split_ms']))"
