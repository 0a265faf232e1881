/*
 * ape_lz4_api.c -- the ape_lz4.h C ABI (all 40 symbols the reference exports,
 * ref src/ape_lz4.h:59-467 plus the 5 undeclared exports) for libape_lz4_amd.so.
 *
 *   one-shot block codec  -> host codec by default; MI355X HIP kernels through
 *                            lz4_runtime.hip when APE_LZ4_ONESHOT_HOST_BELOW selects them
 *     compress_default / compress_fast / compress_fast_extState / compress /
 *     compress_limitedOutput / compress_withState / ..._withState /
 *     compress_fast_force, decompress_safe / decompress_safe_partial /
 *     uncompress_unknownOutputSize, decompress_safe_usingDict(dictSize == 0)
 *   chained streams, dictionaries, decompress_fast, destSize
 *     -> host stream codec (ape_lz4_host.c)
 *
 * One-shot calls run the product's host codec by default (see
 * host_below() below); with the GPU one-shot path selected there is no silent CPU
 * fallback: without a usable gfx950 device the calls report failure (0 from
 * compress, -1 from decompress) and print the runtime error once to stderr.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ape_lz4.h"
#include "../../include/ape_lz4_gpu.h"
#include "ape_lz4_host.h"
#include "lz4_gpu_shim.h"

_Static_assert(sizeof(hst_stream) <= sizeof(APE_LZ4_stream_t), "stream state size");
_Static_assert(sizeof(APE_LZ4_stream_t) == 16416, "APE_LZ4_stream_t ABI size");
_Static_assert(sizeof(hst_stream_dec) == sizeof(APE_LZ4_streamDecode_t), "decode state size");

static void gpu_failed(int rt)
{
    static int reported;
    if (!reported) {
        reported = 1;
        fprintf(stderr, "libape_lz4_amd: GPU codec unavailable (%d): %s\n", rt,
                APE_LZ4_gpu_last_error());
    }
}

/* One-shot compression routing.  The GPU encoder works on
 * independent blocks of at most APE_LZ4_GPU_MAX_BLOCK (= the 64 KiB LZ4 window);
 * a larger one-shot input -- which the reference compresses as one block with its
 * byU32 table (ref src/ape_lz4.c:766-769, :530-755), up to LZ4_MAX_INPUT_SIZE --
 * runs the host codec, whose output is byte-identical to the reference's.  This is
 * a size rule, not a fallback: it applies with or without a GPU. */
static int host_compress(void *state, const char *src, char *dst, int n, int cap, int accel)
{
    hst_stream st;
    return hst_compress_extstate(state ? (hst_stream *)state : &st, src, dst, n, cap, accel);
}

/* One-shot latency routing ("The single-block API stays on the CPU
 * restatement, because a kernel launch costs more than one 8 KiB block").  One call of the
 * GPU one-shot path is a pinned copy, H2D, one workgroup working through the block's 1024
 * chunks, D2H and a stream sync: measured 39 / 126 / 848 us to compress 1 / 8 / 64 KiB
 * (decompress 45 / 112 / 784 us), against 5 / 6 / 47 us (2 / 3 / 15 us) for the reference
 * algorithm on one host core (tests/test_gpu_api.py).  So by default every
 * one-shot call runs the product's host codec (ape_lz4_host.c), byte-identical to the
 * reference; the GPU serves the batch entry points, which fail loudly without a device.
 * A caller can move one-shot calls of blocks >= `bytes` to the GPU with
 * APE_LZ4_gpu_set_oneshot_host_below(bytes) or APE_LZ4_ONESHOT_HOST_BELOW=bytes (0 = every
 * one-shot call on the GPU; compress: input size, decompress: capacity). */
#define ONESHOT_HOST_ALL 0x7FFFFFFF
static int g_host_below = -1;

static int host_below(void)
{
    int v = __atomic_load_n(&g_host_below, __ATOMIC_RELAXED);
    if (v < 0) {
        const char *e = getenv("APE_LZ4_ONESHOT_HOST_BELOW");
        v = (e && *e) ? atoi(e) : ONESHOT_HOST_ALL;
        if (v < 0) v = 0;
        __atomic_store_n(&g_host_below, v, __ATOMIC_RELAXED);
    }
    return v;
}

int APE_LZ4_gpu_set_oneshot_host_below(int bytes)
{
    const int prev = host_below();
    __atomic_store_n(&g_host_below, bytes < 0 ? 0 : bytes, __ATOMIC_RELAXED);
    return prev;
}

static int gpu_compress_st(void *state, const char *src, char *dst, int n, int cap, int accel)
{
    int rt = 0, r;
    if ((unsigned)n > (unsigned)LZ4_MAX_INPUT_SIZE) return 0; /* ref :558 */
    if (n > APE_LZ4_GPU_MAX_BLOCK || n < host_below())
        return host_compress(state, src, dst, n, cap, accel);
    r = ape_lz4_gpu_compress_one(src, dst, n, cap, accel, &rt);
    if (rt) { gpu_failed(rt); return 0; }
    return r == APE_LZ4_GPU_ERANGE ? 0 : r;
}

static int gpu_compress(const char *src, char *dst, int n, int cap, int accel)
{
    return gpu_compress_st(NULL, src, dst, n, cap, accel);
}

static int gpu_decompress(const char *src, char *dst, int csize, int cap, int partial, int target)
{
    int rt = 0, r;
    const int hb = host_below();
    if (hb == ONESHOT_HOST_ALL || (cap >= 0 && cap < hb))
        return hst_decompress_block(src, dst, csize, cap, partial, target);
    r = ape_lz4_gpu_decompress_one(src, dst, csize, cap, partial, target, &rt);
    if (rt) { gpu_failed(rt); return -1; }
    return r;
}

int APE_LZ4_versionNumber(void) { return LZ4_VERSION_NUMBER; }
int APE_LZ4_compressBound(int isize) { return APE_LZ4_COMPRESSBOUND(isize); }
int APE_LZ4_sizeofState(void) { return LZ4_STREAMSIZE; }

/* ---- one-shot compression (ref :758-836, :1679-1699) -> GPU ---- */
int APE_LZ4_compress_default(const char *source, char *dest, int inputSize, int maxOutputSize)
{
    return gpu_compress(source, dest, inputSize, maxOutputSize, 1);
}

int APE_LZ4_compress_fast(const char *source, char *dest, int inputSize, int maxOutputSize,
                          int acceleration)
{
    /* > 1 trades ratio for speed, as in the reference (:789-808); the GPU parse has no
       skip heuristic, so it drops the in-chunk candidate instead */
    return gpu_compress(source, dest, inputSize, maxOutputSize, acceleration);
}

int APE_LZ4_compress_fast_extState(void *state, const char *source, char *dest, int inputSize,
                                   int maxOutputSize, int acceleration)
{
    APE_LZ4_resetStream((APE_LZ4_stream_t *)state); /* ref :762 */
    return gpu_compress_st(state, source, dest, inputSize, maxOutputSize, acceleration);
}

int APE_LZ4_compress_fast_force(const char *source, char *dest, int inputSize,
                                int maxOutputSize, int acceleration)
{
    return APE_LZ4_compress_fast(source, dest, inputSize, maxOutputSize, acceleration);
}

int APE_LZ4_compress_limitedOutput(const char *source, char *dest, int inputSize,
                                   int maxOutputSize)
{
    return APE_LZ4_compress_default(source, dest, inputSize, maxOutputSize);
}

int APE_LZ4_compress(const char *source, char *dest, int inputSize)
{
    return APE_LZ4_compress_default(source, dest, inputSize, APE_LZ4_compressBound(inputSize));
}

int APE_LZ4_compress_limitedOutput_withState(void *state, const char *src, char *dst,
                                             int srcSize, int dstSize)
{
    return APE_LZ4_compress_fast_extState(state, src, dst, srcSize, dstSize, 1);
}

int APE_LZ4_compress_withState(void *state, const char *src, char *dst, int srcSize)
{
    return APE_LZ4_compress_fast_extState(state, src, dst, srcSize,
                                          APE_LZ4_compressBound(srcSize), 1);
}

/* ---- one-shot decompression (ref :1472-1487, :1722-1730) -> GPU ---- */
int APE_LZ4_decompress_safe(const char *source, char *dest, int compressedSize,
                            int maxDecompressedSize)
{
    return gpu_decompress(source, dest, compressedSize, maxDecompressedSize, 0, 0);
}

int APE_LZ4_decompress_safe_partial(const char *source, char *dest, int compressedSize,
                                    int targetOutputSize, int maxDecompressedSize)
{
    return gpu_decompress(source, dest, compressedSize, maxDecompressedSize, 1, targetOutputSize);
}

int APE_LZ4_uncompress_unknownOutputSize(const char *source, char *dest, int isize,
                                         int maxOutputSize)
{
    return APE_LZ4_decompress_safe(source, dest, isize, maxOutputSize);
}

/* ---- destSize and fast decoding (host) ---- */
int APE_LZ4_compress_destSize(const char *src, char *dst, int *srcSizePtr, int targetDstSize)
{
    return hst_compress_destSize(src, dst, srcSizePtr, targetDstSize);
}

int APE_LZ4_decompress_fast(const char *source, char *dest, int originalSize)
{
    return hst_decompress_fast(source, dest, originalSize);
}

int APE_LZ4_uncompress(const char *source, char *dest, int outputSize)
{
    return hst_decompress_fast(source, dest, outputSize);
}

/* ---- streaming compression (ref :1074-1263; socket TX path) ---- */
APE_LZ4_stream_t *APE_LZ4_createStream(void)
{
    APE_LZ4_stream_t *s = (APE_LZ4_stream_t *)calloc(8, LZ4_STREAMSIZE_U64);
    if (s) APE_LZ4_resetStream(s);
    return s;
}

void APE_LZ4_resetStream(APE_LZ4_stream_t *s) { memset(s, 0, sizeof(APE_LZ4_stream_t)); }

int APE_LZ4_freeStream(APE_LZ4_stream_t *s)
{
    free(s);
    return 0;
}

int APE_LZ4_loadDict(APE_LZ4_stream_t *s, const char *dictionary, int dictSize)
{
    return hst_loadDict((hst_stream *)s, dictionary, dictSize);
}

int APE_LZ4_compress_fast_continue(APE_LZ4_stream_t *s, const char *source, char *dest,
                                   int inputSize, int maxOutputSize, int acceleration)
{
    return hst_compress_continue((hst_stream *)s, source, dest, inputSize, maxOutputSize,
                                 acceleration);
}

int APE_LZ4_compress_limitedOutput_continue(APE_LZ4_stream_t *s, const char *src, char *dst,
                                            int srcSize, int maxDstSize)
{
    return APE_LZ4_compress_fast_continue(s, src, dst, srcSize, maxDstSize, 1);
}

int APE_LZ4_compress_continue(APE_LZ4_stream_t *s, const char *source, char *dest,
                              int inputSize)
{
    return APE_LZ4_compress_fast_continue(s, source, dest, inputSize,
                                          APE_LZ4_compressBound(inputSize), 1);
}

int LZ4_compress_forceExtDict(APE_LZ4_stream_t *s, const char *source, char *dest, int inputSize)
{
    return hst_compress_forceExtDict((hst_stream *)s, source, dest, inputSize);
}

int APE_LZ4_saveDict(APE_LZ4_stream_t *s, char *safeBuffer, int dictSize)
{
    return hst_saveDict((hst_stream *)s, safeBuffer, dictSize);
}

/* ---- streaming decompression (ref :1497-1672; socket RX path) ---- */
APE_LZ4_streamDecode_t *APE_LZ4_createStreamDecode(void)
{
    return (APE_LZ4_streamDecode_t *)calloc(1, sizeof(APE_LZ4_streamDecode_t));
}

int APE_LZ4_freeStreamDecode(APE_LZ4_streamDecode_t *s)
{
    free(s);
    return 0;
}

int APE_LZ4_setStreamDecode(APE_LZ4_streamDecode_t *s, const char *dictionary, int dictSize)
{
    return hst_setStreamDecode((hst_stream_dec *)s, dictionary, dictSize);
}

int APE_LZ4_decompress_safe_continue(APE_LZ4_streamDecode_t *s, const char *source, char *dest,
                                     int compressedSize, int maxOutputSize)
{
    return hst_decompress_continue((hst_stream_dec *)s, source, dest, compressedSize,
                                   maxOutputSize, 1);
}

int APE_LZ4_decompress_fast_continue(APE_LZ4_streamDecode_t *s, const char *source, char *dest,
                                     int originalSize)
{
    return hst_decompress_continue((hst_stream_dec *)s, source, dest, 0, originalSize, 0);
}

int APE_LZ4_decompress_safe_usingDict(const char *source, char *dest, int compressedSize,
                                      int maxOutputSize, const char *dictStart, int dictSize)
{
    if (dictSize == 0) /* ref :1630-1633: exactly decompress_safe */
        return APE_LZ4_decompress_safe(source, dest, compressedSize, maxOutputSize);
    return hst_decompress_usingDict(source, dest, compressedSize, maxOutputSize, 1, dictStart,
                                    dictSize);
}

int APE_LZ4_decompress_fast_usingDict(const char *source, char *dest, int originalSize,
                                      const char *dictStart, int dictSize)
{
    return hst_decompress_usingDict(source, dest, 0, originalSize, 0, dictStart, dictSize);
}

int APE_LZ4_decompress_safe_forceExtDict(const char *source, char *dest, int compressedSize,
                                         int maxOutputSize, const char *dictStart, int dictSize)
{
    return hst_decompress_safe_extdict(source, dest, compressedSize, maxOutputSize, dictStart,
                                       dictSize);
}

int APE_LZ4_decompress_safe_withPrefix64k(const char *source, char *dest, int compressedSize,
                                          int maxOutputSize)
{
    return hst_decompress_safe_prefix64k(source, dest, compressedSize, maxOutputSize);
}

int APE_LZ4_decompress_fast_withPrefix64k(const char *source, char *dest, int originalSize)
{
    return hst_decompress_fast(source, dest, originalSize);
}

/* ---- obsolete streaming state API (ref :1735-1767) ---- */
int APE_LZ4_sizeofStreamState(void) { return LZ4_STREAMSIZE; }

int APE_LZ4_resetStreamState(void *state, char *inputBuffer)
{
    if ((((size_t)state) & 3) != 0) return 1;
    memset(state, 0, LZ4_STREAMSIZE);
    ((hst_stream *)state)->bufferStart = (uint8_t *)inputBuffer;
    return 0;
}

void *APE_LZ4_create(char *inputBuffer)
{
    void *s = calloc(8, LZ4_STREAMSIZE_U64);
    if (s) ((hst_stream *)s)->bufferStart = (uint8_t *)inputBuffer;
    return s;
}

char *APE_LZ4_slideInputBuffer(void *state)
{
    hst_stream *s = (hst_stream *)state;
    int d = APE_LZ4_saveDict((APE_LZ4_stream_t *)state, (char *)s->bufferStart, 65536);
    return (char *)(s->bufferStart + d);
}
