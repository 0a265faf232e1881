/*
 * ape_socket_caller.c -- a C caller of include/ape_lz4.h that uses the codec exactly the way
 * the reference socket does, compiled with -Wall -Werror and linked with -lape_lz4_amd by
 * tests/test_product_abi.py::test_c_caller_links_like_ape_socket.
 *
 *   APE_LZ4_COMPRESSBOUND in a constant expression  (ref src/ape_socket.c:39-41)
 *   createStream / createStreamDecode / free*       (:105-137)
 *   TX: 8 KiB blocks, compress_fast_continue into [int size][block], saveDict (:825-857)
 *   RX: decompress_safe_continue into an 8 KiB tmp, the 64 KiB dictionary ring with its
 *       memmove, setStreamDecode on it                 (:1386-1421)
 *   RX again with a stack APE_LZ4_streamDecode_t (ape_lz4.h's public struct)
 *
 * usage: ape_socket_caller MSG_LEN < messages > out
 * stdin: the messages back to back; stdout: u32 frame bytes, the frames, then the plain
 * bytes of RX pass 1 and of RX pass 2.  Exit status 0, or the failing step.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ape_lz4.h"

#define APE_LZ4_BLOCK_SIZE (1024 * 8)
#define APE_LZ4_BLOCK_COMP_SIZE APE_LZ4_COMPRESSBOUND(APE_LZ4_BLOCK_SIZE)
#define APE_LZ4_DICT_BUFFER_SIZE (1024 * 64)

/* a compile-time use of the macro, as a static buffer size */
static char rx_frame[APE_LZ4_BLOCK_COMP_SIZE + sizeof(int)];

typedef struct {
    char *data;
    int pos;
} dict_ring;

static void ring_push(dict_ring *d, const char *blk, int rc)
{
    if (d->pos + rc > APE_LZ4_DICT_BUFFER_SIZE) {
        const int avail = APE_LZ4_DICT_BUFFER_SIZE - d->pos;
        const int need = rc - avail;
        memmove(d->data, d->data + need, (size_t)(d->pos - need));
        memcpy(d->data + d->pos - need, blk, (size_t)rc);
        d->pos = APE_LZ4_DICT_BUFFER_SIZE;
    } else {
        memcpy(d->data + d->pos, blk, (size_t)rc);
        d->pos += rc;
    }
}

/* one RX pass over the framed stream: returns plain bytes produced, or -1 */
static long rx_pass(APE_LZ4_streamDecode_t *sd, const char *frames, long nframes_bytes,
                    char *plain)
{
    dict_ring ring = {malloc(APE_LZ4_DICT_BUFFER_SIZE), 0};
    char tmp[APE_LZ4_BLOCK_SIZE];
    long p = 0, out = 0;
    if (!ring.data) return -1;
    while (p + (long)sizeof(int) <= nframes_bytes) {
        int sz;
        memcpy(&sz, frames + p, sizeof(int));
        if (sz <= 0 || sz > APE_LZ4_BLOCK_COMP_SIZE || p + 4 + sz > nframes_bytes) break;
        memcpy(rx_frame, frames + p + 4, (size_t)sz);   /* the socket's frame buffer */
        const int rc = APE_LZ4_decompress_safe_continue(sd, rx_frame, tmp, sz, APE_LZ4_BLOCK_SIZE);
        if (rc <= 0) { free(ring.data); return -1; }
        ring_push(&ring, tmp, rc);
        if (!APE_LZ4_setStreamDecode(sd, ring.data, ring.pos)) { free(ring.data); return -1; }
        memcpy(plain + out, tmp, (size_t)rc);
        out += rc;
        p += 4 + sz;
    }
    free(ring.data);
    return p == nframes_bytes ? out : -1;
}

int main(int argc, char **argv)
{
    if (argc != 2) return 2;
    const int msg_len = atoi(argv[1]);
    if (msg_len <= 0) return 2;
    size_t cap = 1 << 20, n = 0;
    char *in = malloc(cap);
    for (size_t r; in && (r = fread(in + n, 1, cap - n, stdin)) > 0;) {
        n += r;
        if (n == cap) in = realloc(in, cap *= 2);
    }
    if (!in || n == 0 || n % (size_t)msg_len) return 3;
    const int nmsg = (int)(n / (size_t)msg_len);
    const int per = (msg_len + APE_LZ4_BLOCK_SIZE - 1) / APE_LZ4_BLOCK_SIZE;

    /* ---- TX (ape_socket_write, :811-871) ---- */
    APE_LZ4_stream_t *tx = APE_LZ4_createStream();
    char *dict_tx = malloc(APE_LZ4_DICT_BUFFER_SIZE);
    char *frames = malloc((size_t)nmsg * per * (APE_LZ4_BLOCK_COMP_SIZE + sizeof(int)));
    if (!tx || !dict_tx || !frames) return 4;
    long fpos = 0;
    for (int m = 0; m < nmsg; m++) {
        const char *data = in + (size_t)m * msg_len;
        for (int cur = 0; cur < per; cur++) {
            const int left = msg_len - APE_LZ4_BLOCK_SIZE * cur;
            const int cmp_len = APE_LZ4_compress_fast_continue(
                tx, data + cur * APE_LZ4_BLOCK_SIZE, frames + fpos + sizeof(int),
                left < APE_LZ4_BLOCK_SIZE ? left : APE_LZ4_BLOCK_SIZE, APE_LZ4_BLOCK_COMP_SIZE, 1);
            if (cmp_len <= 0) return 5;
            memcpy(frames + fpos, &cmp_len, sizeof(int));
            fpos += cmp_len + (long)sizeof(int);
        }
        if (APE_LZ4_saveDict(tx, dict_tx, APE_LZ4_DICT_BUFFER_SIZE) <= 0) return 6;
    }
    if (APE_LZ4_freeStream(tx) != 0) return 7;

    /* ---- RX (ape_socket_read_lz4_stream, :1333-1467), heap stream then stack stream ---- */
    char *plain1 = malloc(n), *plain2 = malloc(n);
    APE_LZ4_streamDecode_t *rx = APE_LZ4_createStreamDecode();
    if (!plain1 || !plain2 || !rx) return 8;
    if (rx_pass(rx, frames, fpos, plain1) != (long)n) return 9;
    if (APE_LZ4_freeStreamDecode(rx) != 0) return 10;
    APE_LZ4_streamDecode_t on_stack;
    memset(&on_stack, 0, sizeof on_stack);
    if (rx_pass(&on_stack, frames, fpos, plain2) != (long)n) return 11;

    const unsigned int fb = (unsigned int)fpos;
    if (fwrite(&fb, 4, 1, stdout) != 1 || fwrite(frames, 1, (size_t)fpos, stdout) != (size_t)fpos ||
        fwrite(plain1, 1, n, stdout) != n || fwrite(plain2, 1, n, stdout) != n)
        return 12;
    free(in); free(dict_tx); free(frames); free(plain1); free(plain2);
    return 0;
}
