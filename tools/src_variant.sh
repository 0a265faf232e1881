#!/bin/bash
# Build a diagnostic library variant with one kernel source replaced (e.g. an older
# revision: git show REV:libapenetwork_amd/csrc/lz4_decode.hip > /tmp/old.hip), linked with
# the product's other objects -> libapenetwork_amd/libape_lz4_amd_<name>.so (never the product).
# usage: bash tools/src_variant.sh NAME replacement.hip lz4_decode
set -e
cd "$(dirname "$0")/.."
V=$1; SRC=$2; OBJ=$3
B=libapenetwork_amd/build
make -s -C libapenetwork_amd/csrc >/dev/null
mkdir -p $B/srcvar_$V
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
    -munsafe-fp-atomics -Ilibapenetwork_amd/csrc -Iinclude $([ "$OBJ" = lz4_decode ] && echo -mllvm -amdgpu-sched-strategy=max-ilp) \
    -c $SRC -o $B/srcvar_$V/$OBJ.o
objs=$(ls $B/*.o | grep -v "/$OBJ.o$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o libapenetwork_amd/libape_lz4_amd_$V.so $objs $B/srcvar_$V/$OBJ.o
echo built libapenetwork_amd/libape_lz4_amd_$V.so
