#!/bin/bash
# Decoder A/B (diagnostic): per library variant, the kernel times (trace) and the
# FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) over tools/kernel_driver.py with
# NB blocks (65536 = 4 GiB of input, past the Infinity Cache).  "base" = the product.
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
NB=${NB:-65536}
for v in "$@"; do
  lib=$PWD/libapenetwork_amd/libape_lz4_amd_$v.so
  [ "$v" = base ] && lib=$PWD/libapenetwork_amd/libape_lz4_amd.so
  for c in none FETCH_SIZE WRITE_SIZE; do
    pm=""; [ $c != none ] && pm="--pmc $c"
    APE_LZ4_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace $pm -d gpurun_out/dv_${v}_$c -o run --output-format csv -- python3 tools/kernel_driver.py $NB 1 > gpurun_out/dv_${v}_$c.log 2>&1 || { echo "$v $c failed"; tail -3 gpurun_out/dv_${v}_$c.log; exit 1; }
  done
  python3 - $v $NB <<'PY'
import csv, glob, sys
v, nb = sys.argv[1], int(sys.argv[2])
out = {}
for c in ("none", "FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob("gpurun_out/dv_%s_%s/**/*.csv" % (v, c), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            kk = "enc" if "encode" in k else ("dec" if "decode" in k else None)
            if not kk: continue
            if "kernel_trace" in f and c == "none":
                out[kk + "_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            if "counter_collection" in f:
                val = float(r["Counter_Value"])
                key = "%s_%s" % (kk, c)
                out[key] = out.get(key, 0.0) + val
for kk in ("enc", "dec"):
    if kk + "_FETCH_SIZE" in out:   # KB, 128-B requests tallied at 64 B on gfx950
        out[kk + "_fetch_B_per_block"] = round(out.pop(kk + "_FETCH_SIZE") * 1024 * 2 / nb)
    if kk + "_WRITE_SIZE" in out:
        out[kk + "_write_B_per_block"] = round(out.pop(kk + "_WRITE_SIZE") * 1024 / nb)
print(v, out, open("gpurun_out/dv_%s_none.log" % v).read().strip().split("\n")[-1])
PY
done
