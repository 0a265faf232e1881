/*
 * ape_lz4.h -- drop-in replacement header for libapenetwork's LZ4 block codec
 * (reference: src/ape_lz4.h, LZ4 v1.7.1 "r131" with APE_ prefixes).
 *
 * Same 35 declared entry points, same argument meaning, same return
 * conventions, same ABI-visible struct sizes (APE_LZ4_stream_t = 16416 B,
 * APE_LZ4_streamDecode_t = 32 B), so ape_socket.c / ape_buffer.c and any
 * embedder link against libape_lz4_amd.so unchanged (tests/c/ape_socket_caller.c is
 * such a caller, built with -Wall -Werror by the CPU suite).  One-shot calls run the
 * library's host codec by default -- byte-identical to the reference, at its speed on one
 * core -- and move to CDNA4 HIP kernels on an MI355X only when the caller opts in
 * (APE_LZ4_gpu_set_oneshot_host_below / APE_LZ4_ONESHOT_HOST_BELOW; a single block never
 * beats one host core on the GPU).  ape_lz4_gpu.h is the batched
 * device API, the performance path.
 *
 * Reference citations are file:line into the reference tree.
 */
#pragma once

#if defined(__cplusplus)
extern "C" {
#endif

/* ---- version (ref ape_lz4.h:52-59) ---- */
#define LZ4_VERSION_MAJOR 1
#define LZ4_VERSION_MINOR 7
#define LZ4_VERSION_RELEASE 1
#define LZ4_VERSION_NUMBER \
    (LZ4_VERSION_MAJOR * 100 * 100 + LZ4_VERSION_MINOR * 100 + LZ4_VERSION_RELEASE)
int APE_LZ4_versionNumber(void); /* returns 10701 */

/* ---- tuning constant that fixes the state sizes (ref :72) ---- */
#define LZ4_MEMORY_USAGE 14

/* ---- one-shot block API (ref :79-82) ----
 * compress_default: returns bytes written to dest (<= maxDestSize) or 0.
 * decompress_safe : returns bytes decoded (<= maxDecompressedSize) or a
 *                   negative value -(input bytes consumed)-1 on malformed input.
 * Neither ever writes outside dest nor reads outside source. */
int APE_LZ4_compress_default(const char *source, char *dest, int sourceSize,
                             int maxDestSize);
int APE_LZ4_decompress_safe(const char *source, char *dest, int compressedSize,
                            int maxDecompressedSize);

/* ---- sizing (ref :123-143) ---- */
#define LZ4_MAX_INPUT_SIZE 0x7E000000
#define APE_LZ4_COMPRESSBOUND(isize)                                  \
    ((unsigned)(isize) > (unsigned)LZ4_MAX_INPUT_SIZE                 \
         ? 0                                                          \
         : (isize) + ((isize) / 255) + 16)
int APE_LZ4_compressBound(int inputSize);

/* ---- advanced one-shot API (ref :157-234) ---- */
int APE_LZ4_compress_fast(const char *source, char *dest, int sourceSize,
                          int maxDestSize, int acceleration);
int APE_LZ4_sizeofState(void);
int APE_LZ4_compress_fast_extState(void *state, const char *source, char *dest,
                                   int inputSize, int maxDestSize, int acceleration);
int APE_LZ4_compress_destSize(const char *source, char *dest, int *sourceSizePtr,
                              int targetDestSize);
int APE_LZ4_decompress_fast(const char *source, char *dest, int originalSize);
int APE_LZ4_decompress_safe_partial(const char *source, char *dest, int compressedSize,
                                    int targetOutputSize, int maxDecompressedSize);

/* ---- streaming compression (ref :240-310); sizes are ABI ---- */
#define LZ4_STREAMSIZE_U64 ((1 << (LZ4_MEMORY_USAGE - 3)) + 4)
#define LZ4_STREAMSIZE (LZ4_STREAMSIZE_U64 * sizeof(long long))
typedef struct {
    long long table[LZ4_STREAMSIZE_U64];
} APE_LZ4_stream_t;

void APE_LZ4_resetStream(APE_LZ4_stream_t *streamPtr);
APE_LZ4_stream_t *APE_LZ4_createStream(void);
int APE_LZ4_freeStream(APE_LZ4_stream_t *streamPtr);
int APE_LZ4_loadDict(APE_LZ4_stream_t *streamPtr, const char *dictionary, int dictSize);
int APE_LZ4_compress_fast_continue(APE_LZ4_stream_t *streamPtr, const char *src,
                                   char *dst, int srcSize, int maxDstSize,
                                   int acceleration);
int APE_LZ4_saveDict(APE_LZ4_stream_t *streamPtr, char *safeBuffer, int dictSize);

/* ---- streaming decompression (ref :317-400) ---- */
#define LZ4_STREAMDECODESIZE_U64 4
#define LZ4_STREAMDECODESIZE (LZ4_STREAMDECODESIZE_U64 * sizeof(unsigned long long))
typedef struct {
    unsigned long long table[LZ4_STREAMDECODESIZE_U64];
} APE_LZ4_streamDecode_t;

APE_LZ4_streamDecode_t *APE_LZ4_createStreamDecode(void);
int APE_LZ4_freeStreamDecode(APE_LZ4_streamDecode_t *LZ4_stream);
int APE_LZ4_setStreamDecode(APE_LZ4_streamDecode_t *LZ4_streamDecode,
                            const char *dictionary, int dictSize);
int APE_LZ4_decompress_safe_continue(APE_LZ4_streamDecode_t *LZ4_streamDecode,
                                     const char *source, char *dest, int compressedSize,
                                     int maxDecompressedSize);
int APE_LZ4_decompress_fast_continue(APE_LZ4_streamDecode_t *LZ4_streamDecode,
                                     const char *source, char *dest, int originalSize);
int APE_LZ4_decompress_safe_usingDict(const char *source, char *dest, int compressedSize,
                                      int maxDecompressedSize, const char *dictStart,
                                      int dictSize);
int APE_LZ4_decompress_fast_usingDict(const char *source, char *dest, int originalSize,
                                      const char *dictStart, int dictSize);

/* ---- obsolete entry points kept for ABI compatibility (ref :431-467) ---- */
int APE_LZ4_compress(const char *source, char *dest, int sourceSize);
int APE_LZ4_compress_limitedOutput(const char *source, char *dest, int sourceSize,
                                   int maxOutputSize);
int APE_LZ4_compress_withState(void *state, const char *source, char *dest, int inputSize);
int APE_LZ4_compress_limitedOutput_withState(void *state, const char *source, char *dest,
                                             int inputSize, int maxOutputSize);
int APE_LZ4_compress_continue(APE_LZ4_stream_t *LZ4_streamPtr, const char *source,
                              char *dest, int inputSize);
int APE_LZ4_compress_limitedOutput_continue(APE_LZ4_stream_t *LZ4_streamPtr,
                                            const char *source, char *dest, int inputSize,
                                            int maxOutputSize);
void *APE_LZ4_create(char *inputBuffer);
int APE_LZ4_sizeofStreamState(void);
int APE_LZ4_resetStreamState(void *state, char *inputBuffer);
char *APE_LZ4_slideInputBuffer(void *state);
int APE_LZ4_decompress_safe_withPrefix64k(const char *src, char *dst, int compressedSize,
                                          int maxDstSize);
int APE_LZ4_decompress_fast_withPrefix64k(const char *src, char *dst, int originalSize);

/* Exported by the reference although not declared in its header
 * (ape_lz4.c:821, 1224, 1665, 1722, 1726); declared here for completeness. */
int APE_LZ4_compress_fast_force(const char *source, char *dest, int inputSize,
                                int maxOutputSize, int acceleration);
int LZ4_compress_forceExtDict(APE_LZ4_stream_t *LZ4_dict, const char *source, char *dest,
                              int inputSize);
int APE_LZ4_decompress_safe_forceExtDict(const char *source, char *dest,
                                         int compressedSize, int maxOutputSize,
                                         const char *dictStart, int dictSize);
int APE_LZ4_uncompress(const char *source, char *dest, int outputSize);
int APE_LZ4_uncompress_unknownOutputSize(const char *source, char *dest, int isize,
                                         int maxOutputSize);

#if defined(__cplusplus)
}
#endif
