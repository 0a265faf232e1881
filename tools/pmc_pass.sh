#!/bin/bash
# PMC passes over tools/kernel_driver.py (one counter group per pass, kernel trace only).
# usage: bash tools/pmc_pass.sh OUTDIR NBLOCKS "GROUP1" "GROUP2" ...
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
D=$1; NB=$2; shift 2
mkdir -p $D
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $D/p$i -o run --output-format csv -- python3 tools/kernel_driver.py $NB 1 || exit 1
done
