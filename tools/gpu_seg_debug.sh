#!/bin/bash
# Segment encoder debugging (GPU box): single calls on growing inputs with diagnostic library
# variants (usage: gpu_seg_debug.sh v1 v2 ...), each call under its own time limit; stops at
# the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export APE_LZ4_ENCODER=seg
for V in "$@"; do
  export APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd_$V.so
  [ "$V" = base ] && export APE_LZ4_LIB=$PWD/libapenetwork_amd/libape_lz4_amd.so
  echo "== $V"
  for c in "zeros 1" "comp 1" "rand 1" "comp 64" "runs 8"; do
    timeout -k 10 60 python3 -u tools/seg_debug.py $c || { echo "FAILED: $V $c (rc $?)"; exit 1; }
  done
done
