#!/bin/bash
# SQ instruction counts per block of library variants (diagnostic): tools/sq_variant.sh v1 v2 ...
# ("base" = the product library)
cd "$GRAFT_REPO_ROOT" || exit 1
for v in "$@"; do
  lib=$PWD/libapenetwork_amd/libape_lz4_amd_$v.so
  [ "$v" = base ] && lib=$PWD/libapenetwork_amd/libape_lz4_amd.so
  rm -rf gpurun_out/sqv_$v
  SQ_DIR=gpurun_out/sqv_$v APE_LZ4_LIB=$lib timeout -k 10 300 bash tools/sq_passes.sh ${NB:-16384} > gpurun_out/sqv_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/sqv_$v.log; exit 1; }
  python3 - $v ${NB:-16384} <<'PY'
import sys, re, ast
v, nb = sys.argv[1], int(sys.argv[2])
for line in open("gpurun_out/sqv_%s.log" % v):
    if line.startswith(("enc ", "dec ")):
        k, d = line.split(" ", 1)
        d = ast.literal_eval(d)
        f = lambda c: float(d.get(c, 0)) / nb
        print(v, k, "VALU %.0f SALU %.0f LDS %.0f VMEM %.0f BR %.0f per block; wait/wave %.2f" % (
            f("SQ_INSTS_VALU"), f("SQ_INSTS_SALU"), f("SQ_INSTS_LDS"), f("SQ_INSTS_VMEM"),
            f("SQ_INSTS_BRANCH"), float(d["SQ_WAIT_ANY"]) / float(d["SQ_WAVE_CYCLES"])))
PY
done
