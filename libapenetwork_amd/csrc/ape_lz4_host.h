/* ape_lz4_host.h -- internal interface of the host (CPU) stream codec used for the
 * non-batchable ape_lz4.h entry points (see ape_lz4_host.c). */
#pragma once
#include <stddef.h>
#include <stdint.h>

#define HST_MAX_INPUT 0x7E000000
#define HST_LIMIT64K (65536 + 11)
#define HST_TABLE 4096

/* Layout of APE_LZ4_stream_t's storage (16416 B; ref src/ape_lz4.c:407-414). */
typedef struct {
    uint32_t table[HST_TABLE];
    uint32_t currentOffset;
    uint32_t initCheck;
    const uint8_t *dictionary;
    uint8_t *bufferStart;
    uint32_t dictSize;
} hst_stream;

/* Layout of APE_LZ4_streamDecode_t's storage (32 B; ref :1499-1504). */
typedef struct {
    const uint8_t *externalDict;
    size_t extDictSize;
    const uint8_t *prefixEnd;
    size_t prefixSize;
} hst_stream_dec;

void hst_reset(hst_stream *s);
int hst_compress_extstate(hst_stream *s, const char *src, char *dst, int n, int cap, int accel);
int hst_compress_force(const char *src, char *dst, int n, int cap, int accel);
int hst_compress_destSize(const char *src, char *dst, int *srcSize, int target);
int hst_loadDict(hst_stream *d, const char *dict, int size);
int hst_compress_continue(hst_stream *d, const char *src, char *dst, int n, int cap, int accel);
int hst_compress_forceExtDict(hst_stream *d, const char *src, char *dst, int n);
int hst_saveDict(hst_stream *d, char *safe, int size);
int hst_decompress_fast(const char *s, char *d, int osize);
int hst_decompress_block(const char *s, char *d, int csize, int cap, int partial, int target);
int hst_decompress_safe_prefix64k(const char *s, char *d, int csize, int cap);
int hst_decompress_safe_extdict(const char *s, char *d, int csize, int cap, const char *dict,
                                int dsize);
int hst_decompress_usingDict(const char *s, char *d, int csize, int cap, int safe,
                             const char *dict, int dsize);
int hst_setStreamDecode(hst_stream_dec *sd, const char *dict, int size);
int hst_decompress_continue(hst_stream_dec *sd, const char *src, char *dst, int csize, int cap,
                            int safe);
