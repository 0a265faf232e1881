#!/bin/bash
# TEST INFRASTRUCTURE: build the REFERENCE's socket stack (every /root/reference/src/*.c except
# ape_lz4.c) from its own sources with gcc, and link it with tests/c/ref_socket_lz4.c against the
# product library libape_lz4_amd.so in place of the reference's ape_lz4.o.
# c-ares and OpenSSL come from /opt/conda.  Outputs only under oracle/_ref/net/
# (git-ignored and gpurun-ignored: nothing from the reference is committed or sent to the GPU
# box).  No reference source is copied; nothing stands in for a missing header or library.
#   usage: bash oracle/ref_net.sh   -> oracle/_ref/net/ref_socket_lz4 (exit 2 if unbuildable)
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(dirname "$HERE")
REF=${APE_REF_SRC:-/root/reference/src}
OUT=$HERE/_ref/net
LIBDIR=$ROOT/libapenetwork_amd
CONDA=/opt/conda
[ -d "$REF" ] || { echo "reference sources absent: $REF"; exit 2; }
[ -f "$CONDA/include/ares.h" ] || { echo "c-ares headers absent"; exit 2; }
[ -f "$LIBDIR/libape_lz4_amd.so" ] || make -s -C "$LIBDIR/csrc"
mkdir -p "$OUT"
CFL="-O2 -std=gnu11 -w -D_GNU_SOURCE -DFD_SETSIZE=2048 -DOPENSSL_API_COMPAT=0x10100000L -I$REF -I$CONDA/include"
objs=""
for f in "$REF"/*.c; do
    b=$(basename "$f" .c)
    [ "$b" = ape_lz4 ] && continue          # the codec comes from libape_lz4_amd.so
    o=$OUT/$b.o
    if [ ! -f "$o" ] || [ "$f" -nt "$o" ]; then gcc $CFL -c "$f" -o "$o"; fi
    objs="$objs $o"
done
# the driver, like the socket code, is compiled against the reference's own headers (its
# ape_lz4.h included): the product library must be a binary drop-in for them
gcc -O2 -std=gnu11 -Wall -Werror -Wno-unused-variable -D_GNU_SOURCE -DFD_SETSIZE=2048 -I"$REF" \
    -I$CONDA/include -c "$ROOT/tests/c/ref_socket_lz4.c" -o "$OUT/ref_socket_lz4.o"
# conda's libraries by path (no -L: its older libstdc++ must not resolve the HIP runtime's);
# the executable's RUNPATH finds them at run time, the product's own dependencies resolve as usual
gcc -o "$OUT/ref_socket_lz4" "$OUT/ref_socket_lz4.o" $objs -L"$LIBDIR" -lape_lz4_amd \
    $CONDA/lib/libcares.so.2 $CONDA/lib/libssl.so.1.1 $CONDA/lib/libcrypto.so.1.1 -lz -lm -lpthread \
    -Wl,-rpath-link,/usr/lib/x86_64-linux-gnu -Wl,--enable-new-dtags -Wl,-rpath,"$LIBDIR" -Wl,-rpath,$CONDA/lib
echo "built $OUT/ref_socket_lz4"
