/*
 * ape_lz4_gpu.h -- batched MI355X LZ4 block codec: the performance path.
 *
 * Each entry point runs N *independent* LZ4 blocks on the calling thread's
 * current HIP device, one workgroup per block.  Per-block results use exactly
 * the conventions of the single-block calls they batch:
 *
 *   APE_LZ4_compress_batch_dev       == N x APE_LZ4_compress_default
 *                                        (ref src/ape_lz4.c:811-815)
 *   APE_LZ4_decompress_safe_batch_dev == N x APE_LZ4_decompress_safe
 *                                        (ref src/ape_lz4.c:1472-1478)
 *   ..._partial_batch_dev            == N x APE_LZ4_decompress_safe_partial
 *                                        (ref src/ape_lz4.c:1480-1487)
 *
 * Compression emits a valid LZ4 v1.7.1 block (decodable by the reference
 * decompress_safe with cap = srcSize) but not the reference's byte stream:
 * the GPU parse is its own.  Decompression is bit-exact
 * with the reference: same return value, same dst[0:ret].
 *
 * Pointers named d_* are device pointers (hipMalloc / torch CUDA tensors).
 * `stream` is a hipStream_t passed as void* (NULL = default stream).  All
 * launchers are asynchronous and graph-capturable (no allocation, no sync), except
 * APE_LZ4_compress_destSize_batch_dev (stream-ordered scratch; see its _scratch form).
 * Return value of a launcher: 0 on success, otherwise a negative
 * APE_LZ4_GPU_E* code (nothing was launched); per-block status is in d_result.
 *
 * GPU limits: the encoder takes blocks of at most APE_LZ4_GPU_MAX_BLOCK (65536)
 * bytes (the LZ4 window; the benchmark's 64 KiB block); a larger input gets
 * d_result = APE_LZ4_GPU_ERANGE.  The decoder has no block-size limit.
 */
#pragma once
#include <stddef.h>

#if defined(__cplusplus)
extern "C" {
#endif

#define APE_LZ4_GPU_MAX_BLOCK 65536
#define APE_LZ4_GPU_ERANGE (-2147483647 - 1) /* per-block: size outside GPU limits */

enum {
    APE_LZ4_GPU_OK = 0,
    APE_LZ4_GPU_ENODEV = -1,   /* no usable MI355X / HIP runtime          */
    APE_LZ4_GPU_EINVAL = -2,   /* bad argument (N < 0, null pointer ...)  */
    APE_LZ4_GPU_ELAUNCH = -3,  /* kernel launch / HIP runtime error        */
    APE_LZ4_GPU_ENOMEM = -4    /* staging allocation failed                */
};

/* Runtime. */
int APE_LZ4_gpu_init(void);                 /* 0 if a gfx950 device is usable */
int APE_LZ4_gpu_device_count(void);
const char *APE_LZ4_gpu_last_error(void);   /* thread-local message */
const char *APE_LZ4_gpu_arch(void);         /* "gfx950" */

/* ---- batched, device-resident, pointer-array form ----
 * d_src[i]  : block i input (device)     d_srcSize[i] : its size (0..65536)
 * d_dst[i]  : block i output (device)    d_dstCap[i]  : its capacity
 * d_result[i] <- compressed size, or 0 if it does not fit d_dstCap[i]. */
int APE_LZ4_compress_batch_dev(const char *const *d_src, const int *d_srcSize,
                               char *const *d_dst, const int *d_dstCap, int *d_result,
                               int nblocks, void *stream);

/* == N x APE_LZ4_compress_fast (ref src/ape_lz4.c:789-808): acceleration > 1 probes the
 * reference's positions -- the match end, the next two, then steps of acceleration growing
 * by one every 64 misses (:591-600) -- with the reference's unbounded catch-up, so the ratio
 * follows the reference's (within 1 % at 2, 4, 8 on the benchmark data); <= 1 is
 * compress_default. */
int APE_LZ4_compress_fast_batch_dev(const char *const *d_src, const int *d_srcSize,
                                    char *const *d_dst, const int *d_dstCap, int *d_result,
                                    int nblocks, int acceleration, void *stream);

/* Greedy-exact mode (slow, for debugging): == N x APE_LZ4_compress_fast
 * (ref src/ape_lz4.c:789-808 -> LZ4_compress_generic :530-755, byU16), BYTE FOR BYTE -- the
 * reference's sequential parse run by one wave per block, limitedOutput's early exits (0)
 * included; acceleration <= 1 is compress_default.  Deviation: a negative d_dstCap[i] gives 0
 * (the reference treats it as a huge unsigned capacity in its last-literals check). */
int APE_LZ4_compress_exact_batch_dev(const char *const *d_src, const int *d_srcSize,
                                     char *const *d_dst, const int *d_dstCap, int *d_result,
                                     int nblocks, int acceleration, void *stream);

/* d_result[i] <- decoded size, or -(consumed)-1, as APE_LZ4_decompress_safe. */
int APE_LZ4_decompress_safe_batch_dev(const char *const *d_src, const int *d_compressedSize,
                                      char *const *d_dst, const int *d_maxDecompressedSize,
                                      int *d_result, int nblocks, void *stream);

/* As APE_LZ4_decompress_safe_partial with per-block targetOutputSize. */
int APE_LZ4_decompress_safe_partial_batch_dev(const char *const *d_src,
                                              const int *d_compressedSize,
                                              char *const *d_dst, const int *d_targetOutputSize,
                                              const int *d_maxDecompressedSize,
                                              int *d_result, int nblocks, void *stream);

/* ---- chained streams (socket path with the reference wire format) ----
 * The reference socket compresses each chunk with compress_fast_continue against the
 * previous <= 64 KiB of its stream and the receiver decodes it with
 * decompress_safe_continue against its saved dictionary (ref src/ape_lz4.c:1160-1220,
 * :1555-1584; src/ape_socket.c:832-857, :1386-1421).  Batched across connections:
 *
 * compress_withPrefix : d_prefixSize[i] bytes immediately before d_src[i] are the
 *   stream's history; matches may reach into it (the last min(prefix, 65536 - size)
 *   bytes, rounded down to a multiple of 64, are used).  d_result[i] as
 *   APE_LZ4_compress_batch_dev.  The block decodes with decompress_safe_continue /
 *   decompress_safe_usingDict given that history (bytes differ from the reference's,
 *   as for every GPU-compressed block).
 * decompress_safe_usingDict : == N x APE_LZ4_decompress_safe_usingDict(src, dst,
 *   csize, cap, dict, dictSize) (ref src/ape_lz4.c:1625-1655), bit-exact, any
 *   placement of the dictionary (adjacent to dst or not). */
int APE_LZ4_compress_withPrefix_batch_dev(const char *const *d_src, const int *d_srcSize,
                                          const int *d_prefixSize, char *const *d_dst,
                                          const int *d_dstCap, int *d_result, int nblocks,
                                          void *stream);
int APE_LZ4_decompress_safe_usingDict_batch_dev(const char *const *d_src,
                                                const int *d_compressedSize, char *const *d_dst,
                                                const int *d_maxDecompressedSize,
                                                const char *const *d_dict, const int *d_dictSize,
                                                int *d_result, int nblocks, void *stream);

/* == N x APE_LZ4_decompress_fast(src, dst, originalSize) (ref src/ape_lz4.c:1489):
 * d_result[i] <- compressed bytes consumed, or -(consumed)-1.  The reference reads its
 * input without a bound; the batch needs d_srcBound[i] = the readable bytes at d_src[i]
 * (e.g. compressBound(originalSize)), and rejects an offset reaching before d_dst[i]
 * (the reference reads memory before dst there). */
int APE_LZ4_decompress_fast_batch_dev(const char *const *d_src, const int *d_srcBound,
                                      char *const *d_dst, const int *d_originalSize,
                                      int *d_result, int nblocks, void *stream);

/* == N x APE_LZ4_compress_destSize(src, dst, &srcSize, targetDstSize) (ref
 * src/ape_lz4.c:1048-1067, :843-1021): d_srcSize[i] is in/out -- on entry the input size,
 * on return the input bytes the block encodes; d_result[i] <- bytes written to d_dst[i]
 * (<= d_targetDstSize[i]; 0 if the target is < 1 or the size negative).  The output is a
 * valid LZ4 block of src[0, consumed) (decodes with cap = consumed); when the whole block
 * fits the target it is compress_default's output.  Bytes and consumed size differ from
 * the reference's greedy cut (the GPU parse is chunk-parallel; the cut is at a sequence
 * boundary followed by as many literals as fit).  The one launcher that allocates:
 * stream-ordered scratch (hipMallocAsync/hipFreeAsync on `stream`) of ~65.8 KB per
 * block, at most 16384 blocks at a time -- not for graph capture; the _scratch form
 * below takes caller-owned scratch instead and allocates nothing. */
int APE_LZ4_compress_destSize_batch_dev(const char *const *d_src, int *d_srcSize,
                                        char *const *d_dst, const int *d_targetDstSize,
                                        int *d_result, int nblocks, void *stream);
/* Scratch bytes for destSize of nblocks in one pass (a smaller 16-aligned scratch, at
 * least scratch_size(1), makes the call run several passes). */
size_t APE_LZ4_compress_destSize_scratch_size(int nblocks);
int APE_LZ4_compress_destSize_batch_scratch_dev(const char *const *d_src, int *d_srcSize,
                                                char *const *d_dst, const int *d_targetDstSize,
                                                int *d_result, int nblocks, void *d_scratch,
                                                size_t scratch_bytes, void *stream);

/* One-shot routing: ape_lz4.h one-shot calls on blocks smaller than
 * `bytes` (compress: input size; decompress_safe/_partial: capacity) run the host codec,
 * which is byte-identical to the reference; larger ones run on the GPU.  The default is
 * 0x7FFFFFFF -- every one-shot call on the host, because one GPU call costs 40-850 us
 * against 2-47 us on one host core for 1-64 KiB -- or the value of
 * the APE_LZ4_ONESHOT_HOST_BELOW environment variable; 0 puts every one-shot call on the
 * GPU.  The batch entry points below always run on the GPU.  Returns the previous
 * threshold. */
int APE_LZ4_gpu_set_oneshot_host_below(int bytes);

/* ---- batched, device-resident, strided form (block i at base + i*stride) ----
 * The layout the benchmark uses: uncompressed slots of `src_stride` bytes,
 * compressed slots of `dst_stride` bytes; a NULL cap array means
 * "capacity = compressBound(srcSize)" / "= dst_stride". */
int APE_LZ4_compress_batch_strided_dev(const char *d_src, size_t src_stride,
                                       const int *d_srcSize, char *d_dst, size_t dst_stride,
                                       const int *d_dstCap, int *d_result, int nblocks,
                                       void *stream);
int APE_LZ4_decompress_safe_batch_strided_dev(const char *d_src, size_t src_stride,
                                              const int *d_compressedSize, char *d_dst,
                                              size_t dst_stride,
                                              const int *d_maxDecompressedSize,
                                              int *d_result, int nblocks, void *stream);

/* ---- framed stream of independent blocks (socket path) ----
 * The reference socket stream frames each LZ4 block as [int32 size][block]
 * (ref src/ape_socket.c:813-850) with chained blocks; this batched form keeps
 * the frame layout (little-endian size) with independent blocks, back to back.
 *   frame_offsets : d_off[i] = sum_{j<i} (4 + d_compressedSize[j]) for i <= N
 *                   (d_off has N + 1 entries, d_off[N] = stream length);
 *                   d_scratch = APE_LZ4_frame_scratch_size(N) bytes of device memory
 *   frame_pack    : compressed slots (block i at d_comp + i*comp_stride) -> frames
 *   decompress_safe_frames : block i read from d_frames + d_off[i] (size from its
 *                   header), decoded to d_dst + i*dst_stride; results as
 *                   APE_LZ4_decompress_safe. */
size_t APE_LZ4_frame_scratch_size(int nblocks);
int APE_LZ4_frame_offsets_dev(const int *d_compressedSize, long long *d_off, void *d_scratch,
                              int nblocks, void *stream);
int APE_LZ4_frame_pack_strided_dev(const char *d_comp, size_t comp_stride,
                                   const int *d_compressedSize, const long long *d_off,
                                   char *d_frames, int nblocks, void *stream);
int APE_LZ4_decompress_safe_frames_dev(const char *d_frames, const long long *d_off,
                                       char *d_dst, size_t dst_stride,
                                       const int *d_maxDecompressedSize, int *d_result,
                                       int nblocks, void *stream);

/* ---- host-buffer batch (socket / ape_buffer path): pinned staging, H2D,
 * kernel, D2H on an internal stream; synchronous.  h_result as above. */
int APE_LZ4_compress_batch_host(const char *const *h_src, const int *h_srcSize,
                                char *const *h_dst, const int *h_dstCap, int *h_result,
                                int nblocks);
int APE_LZ4_decompress_safe_batch_host(const char *const *h_src, const int *h_compressedSize,
                                       char *const *h_dst, const int *h_maxDecompressedSize,
                                       int *h_result, int nblocks);

/* ---- socket path (BASELINE config 5; lz4_sock.hip) ----
 * APE_LZ4_rxbuf: the receive buffer of ape_socket (`buffer`, ref src/ape_buffer.c:210-228)
 * as a growable host buffer registered with hipHostRegister, plus a frame parser for the
 * [le32 size][block] stream that is correct across any read boundaries (the reference's
 * parser desyncs, src/ape_socket.c:1372-1379).
 *   rxbuf_prepare(b, n) : >= n free bytes after `used` (realloc + re-register); 0 / -1
 *   rxbuf_append        : copy bytes in (what a read() into data + used does)
 *   rxbuf_frames        : off[0..n) = complete frames' header positions, off[n] = their end;
 *                         returns n (<= max_frames), or -1 for a size < 0 or > max_block
 *   rxbuf_consume(b, k) : drop the first k bytes
 * socket_send_blocks : nblocks host blocks -> GPU encode -> frames -> write(fd); returns the
 *                      bytes written or an APE_LZ4_GPU_E* code.
 * socket_recv_blocks : read(fd) -> rxbuf -> GPU decode from the frames -> host blocks;
 *                      h_result[i] as decompress_safe; returns the blocks received, or an
 *                      APE_LZ4_GPU_E* code (EINVAL also for a malformed stream / early EOF).
 * Both are blocking calls for one connection; each overlaps socket I/O with GPU work. */
typedef struct APE_LZ4_rxbuf APE_LZ4_rxbuf;
APE_LZ4_rxbuf *APE_LZ4_rxbuf_new(size_t initial);
int APE_LZ4_rxbuf_prepare(APE_LZ4_rxbuf *b, size_t more);
int APE_LZ4_rxbuf_append(APE_LZ4_rxbuf *b, const char *data, size_t len);
int APE_LZ4_rxbuf_frames(const APE_LZ4_rxbuf *b, long long *off, int max_frames, int max_block);
void APE_LZ4_rxbuf_consume(APE_LZ4_rxbuf *b, size_t n);
char *APE_LZ4_rxbuf_data(APE_LZ4_rxbuf *b);
size_t APE_LZ4_rxbuf_used(const APE_LZ4_rxbuf *b);
size_t APE_LZ4_rxbuf_room(const APE_LZ4_rxbuf *b);
int APE_LZ4_rxbuf_pinned(const APE_LZ4_rxbuf *b);
void APE_LZ4_rxbuf_free(APE_LZ4_rxbuf *b);
long long APE_LZ4_socket_send_blocks(int fd, const char *h_src, size_t src_stride, int block_size,
                                     int nblocks, int batch);
long long APE_LZ4_socket_recv_blocks(int fd, char *h_dst, size_t dst_stride, int block_size,
                                     int nblocks, int batch, int *h_result);

/* ---- chained socket streams: the reference wire format through the GPU (lz4_sock.hip) ----
 * nconn connections, each a stream exactly as the reference socket writes and reads it:
 * every message cut into 8 KiB chunks, each compressed against the previous <= 64 KiB of
 * its stream and framed [int32 size][block] (ref src/ape_socket.c:811-871); the receiver
 * decodes each frame against the previous 64 KiB it decoded (:1333-1467).  An unmodified
 * reference peer reads what chain_send writes and writes what chain_recv reads.
 *   chain_new(nconn, msg_len) : device history windows for nconn send and nconn receive
 *                        streams, msg_len bytes per message (NULL on failure)
 *   chain_send         : nmsg rounds; round m compresses message m of every connection
 *                        (at h_msgs + (m * nconn + i) * msg_stride) in one GPU launch (a
 *                        chunk's history is plaintext the sender has) and writes connection
 *                        i's frames to fds[i].  Returns the bytes written or APE_LZ4_GPU_E*.
 *   chain_recv         : nmsg rounds; reads every fd (poll), parses each connection's frames
 *                        split-safe, decodes round m's message of every connection with one
 *                        usingDict launch per 8 KiB chunk (the connections are the batch) into
 *                        h_out + (m * nconn + i) * out_stride.  h_status[i] = 0 or the first
 *                        bad result of connection i.  Returns the payload bytes or
 *                        APE_LZ4_GPU_E* (EINVAL: malformed frame, early EOF, failed decode).
 * One thread may send while another receives on the same chain.  Errors are sticky per
 * direction: a failed call has consumed frames / advanced the streams it ran, so every later
 * call in that direction returns APE_LZ4_GPU_EINVAL (h_status[i] = -1); free the chain. */
typedef struct APE_LZ4_chain APE_LZ4_chain;
APE_LZ4_chain *APE_LZ4_chain_new(int nconn, int msg_len);
void APE_LZ4_chain_free(APE_LZ4_chain *c);
long long APE_LZ4_chain_send(APE_LZ4_chain *c, const int *fds, const char *h_msgs,
                             size_t msg_stride, int nmsg);
long long APE_LZ4_chain_recv(APE_LZ4_chain *c, const int *fds, char *h_out, size_t out_stride,
                             int nmsg, int *h_status);

/* Time split of the socket calls since the last reset, out[16] in ms: TX [0] H2D, [1] encode
 * + frame offsets + pack (GPU), [2] D2H, [3] write(), [4] host waiting for the GPU, [5]
 * batches (count), [6] the whole send call; RX [7] the whole receive loop, [8] read(), [9]
 * frame parse + leftover copy, [10] H2D, [11] decode (GPU), [12] D2H, [13] host waiting for
 * the GPU, [14] batches (count), [15] receive-buffer growth.  GPU phases are timing events
 * around each batch's stages.  reset != 0 zeroes the counters. */
int APE_LZ4_socket_stats(double *out16, int reset);

/* ---- synthetic benchmark data, device-side ----
 * kind 0 = random bytes, 1 = compressible; block b is seeded with first_block+b. */
int APE_LZ4_synth_blocks_dev(char *d_out, size_t stride, int blockSize,
                             long long first_block, int nblocks, int kind, void *stream);

#if defined(__cplusplus)
}
#endif
