#!/bin/bash
# Build an encoder-only diagnostic variant: lz4_encode.hip with extra -D flags, linked with
# the product's other objects -> libapenetwork_amd/libape_lz4_amd_<name>.so (never the product).
# usage: bash tools/enc_variant.sh NAME "-DAPE_LZ4_..." [encoder source]
set -e
cd "$(dirname "$0")/.."
V=$1; DEFS=$2; SRC=${3:-libapenetwork_amd/csrc/lz4_encode.hip}
B=libapenetwork_amd/build
make -s -C libapenetwork_amd/csrc >/dev/null
mkdir -p $B/encvar_$V
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
    -munsafe-fp-atomics -mllvm -amdgpu-sched-strategy=max-ilp -Ilibapenetwork_amd/csrc -Iinclude $DEFS \
    -c $SRC -o $B/encvar_$V/lz4_encode.o
objs=$(ls $B/*.o | grep -v '/lz4_encode.o$')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o libapenetwork_amd/libape_lz4_amd_$V.so $objs $B/encvar_$V/lz4_encode.o
echo built libapenetwork_amd/libape_lz4_amd_$V.so
