#!/bin/bash
# Memory-system PMC passes over tools/kernel_driver.py (DIAGNOSTIC): is the encoder bound by
# the texture/L1 path or the L2 (busy fractions, request counts, stalls)?  One --pmc pass per
# group (block limits: TA 2, TCP 4, TCC 4, GRBM 2).  Results: gpurun_out/mem/p*/.
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
NB=${1:-16384}
OUT=gpurun_out/mem
i=0
for grp in "GRBM_GUI_ACTIVE GRBM_TA_BUSY TA_TA_BUSY TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY" \
           "GRBM_GUI_ACTIVE TCC_REQ TCC_HIT TCC_MISS TCC_BUSY" \
           "GRBM_GUI_ACTIVE TCC_TAG_STALL TCC_EA0_RDREQ_LEVEL TCC_EA0_RDREQ TCC_READ" \
           "GRBM_GUI_ACTIVE TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_TCR_TCP_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TCP_UTCL1_TRANSLATION_MISS TCP_TOTAL_CACHE_ACCESSES" \
           "GRBM_GUI_ACTIVE TA_TOTAL_WAVEFRONTS TCP_UTCL1_REQUEST TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_STALL_MULTI_MISS TCP_TCP_TA_ADDR_STALL_CYCLES" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 tools/kernel_driver.py $NB 1 > gpurun_out/mem_p$i.log 2>&1 || { echo "mem pass $i failed"; tail -5 gpurun_out/mem_p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob('gpurun_out/mem/p*/*counter_collection.csv') + glob.glob('gpurun_out/mem/p*/*/*counter_collection.csv'):
    p = f.split('/')[2]
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        k = 'enc' if 'encode' in k else ('dec' if 'decode' in k else None)
        if k: agg[k][p + ':' + r['Counter_Name']] += float(r['Counter_Value'])
for k, d in agg.items():
    print(k, {c: '%.4g' % v for c, v in sorted(d.items())})
PY
