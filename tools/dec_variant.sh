#!/bin/bash
# Build a decoder-only diagnostic variant: lz4_decode.hip with extra -D flags, linked with
# the product's other objects -> libapenetwork_amd/libape_lz4_amd_<name>.so (never the product).
# usage: bash tools/dec_variant.sh NAME "-DAPE_LZ4_DWIN=... -DAPE_LZ4_DSTAGE=..."
set -e
cd "$(dirname "$0")/.."
V=$1; DEFS=$2
B=libapenetwork_amd/build
make -s -C libapenetwork_amd/csrc >/dev/null
mkdir -p $B/decvar_$V
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
    -munsafe-fp-atomics -mllvm -amdgpu-sched-strategy=max-ilp $DEFS -c libapenetwork_amd/csrc/lz4_decode.hip -o $B/decvar_$V/lz4_decode.o
objs=$(ls $B/*.o | grep -v '/lz4_decode.o$')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o libapenetwork_amd/libape_lz4_amd_$V.so $objs $B/decvar_$V/lz4_decode.o
echo built libapenetwork_amd/libape_lz4_amd_$V.so
