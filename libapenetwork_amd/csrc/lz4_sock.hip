// lz4_sock.hip -- the socket path of the batched codec, host side (BASELINE config 5,
// SURVEY.md 8(f) rows 1-2): ape_buffer's growable receive buffer made pinned, the
// receiver's frame parser rewritten, and TX / RX loops that move framed independent
// blocks between host memory, a socket and the GPU kernels.
//
// Reference: the socket receives into `buffer` (malloc/realloc, src/ape_buffer.c:210-228)
// and parses [int32 size][LZ4 block] frames in ape_socket_read_lz4_stream
// (src/ape_socket.c:1333-1467).  That parser desyncs: it copies header bytes
// to `&current_block_size + decompress_position` -- uint32 pointer arithmetic, so a header
// split across reads lands 4 bytes per byte apart (:1372-1374) -- advances
// `decompress_position` by the whole read instead of the header bytes taken (:1379), and
// memmoves from an already-advanced pointer (:1459).  Here:
//   * APE_LZ4_rxbuf is the `buffer` analogue: APE_LZ4_rxbuf_prepare(b, n) guarantees n
//     free bytes like buffer_prepare (realloc), and re-registers the storage with
//     hipHostRegister, so the frames are DMA'd to the GPU straight from it;
//   * APE_LZ4_rxbuf_frames parses only from a buffer that holds everything received and
//     not yet consumed, header and block bytes alike, so a header or block split over
//     any number of reads is just "not complete yet"; sizes are validated before use;
//   * APE_LZ4_socket_send_blocks / _recv_blocks run the whole path on one connection:
//     TX = H2D blocks -> encode -> frame offsets + pack -> D2H -> write(); RX = read()
//     into the pinned rxbuf -> parse -> H2D frames -> decode from frames -> D2H blocks.
//     Each side double-buffers, so socket I/O of one batch overlaps the GPU work of the
//     next.  The event loop is not rebuilt: these are blocking calls for one connection
//     (a caller runs TX and RX on their own threads, as the loopback benchmark does).
#include <errno.h>
#include <poll.h>
#include <thread>
#include <vector>
#include <time.h>
#include <atomic>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../../include/ape_lz4_gpu.h"
#include "lz4_gpu_internal.h"

using namespace apelz4;

struct APE_LZ4_rxbuf {
    char *data;
    size_t size, used;
    int registered;   // 1 registered for DMA, 0 not (yet), -1 never (a host-only buffer)
};

namespace {

inline size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }
inline int bound_of(int n) { return n + n / 255 + 16; }

void rx_unregister(APE_LZ4_rxbuf *b) {
    if (b->registered == 1) {
        (void)hipHostUnregister(b->data);
        b->registered = 0;
    }
}

int rx_register(APE_LZ4_rxbuf *b) {
    if (!b->data || b->registered) return 0;
    if (hipHostRegister(b->data, b->size, hipHostRegisterDefault) != hipSuccess) return -1;
    b->registered = 1;
    return 0;
}

// write all of buf to fd (blocking), retrying on EINTR / short writes
long long write_all(int fd, const char *buf, size_t len) {
    size_t done = 0;
    while (done < len) {
        const ssize_t w = write(fd, buf + done, len - done);
        if (w < 0) {
            if (errno == EINTR) continue;
            return -1;
        }
        done += (size_t)w;
    }
    return (long long)done;
}

// Time split of the last socket calls (APE_LZ4_socket_stats): GPU phases from timing
// events around each batch's stages, host phases from the monotonic clock.
//   TX: 0 H2D, 1 encode + frame offsets + pack, 2 D2H, 3 write(), 4 waiting for the GPU,
//       5 batches, 6 the whole call;  RX: 7 the whole loop, 8 read(), 9 frame parse +
//       leftover copy, 10 H2D, 11 decode, 12 D2H, 13 waiting for the GPU, 14 batches,
//       15 receive-buffer growth (prepare).   (ns; batches as counts)
std::atomic<long long> g_sock_ns[16];
inline long long now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (long long)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}
inline void sock_add(int i, long long v) { g_sock_ns[i].fetch_add(v, std::memory_order_relaxed); }

struct Dev {   // device buffers of one batch slot
    char *src = nullptr, *comp = nullptr, *frames = nullptr, *out = nullptr;
    int *csz = nullptr, *sizes = nullptr, *res = nullptr;
    long long *off = nullptr;
    int *hres = nullptr;      // RX: pinned landing slot of the batch's results (a D2H into
                              // the caller's pageable array would block the receive loop)
    void *scratch = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;
    hipEvent_t tev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};   // stage timing
};

// elapsed ns between timing events a and b (both complete)
inline long long ev_ns(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? (long long)(ms * 1e6) : 0;
}

int dev_alloc(Dev &d, int batch, int bs, bool tx) {
    const size_t slot = up16((size_t)bound_of(bs));
    bool ok = hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&d.ev, hipEventDisableTiming) == hipSuccess &&
              hipEventCreate(&d.tev[0]) == hipSuccess && hipEventCreate(&d.tev[1]) == hipSuccess &&
              hipEventCreate(&d.tev[2]) == hipSuccess && hipEventCreate(&d.tev[3]) == hipSuccess &&
              hipEventCreate(&d.tev[4]) == hipSuccess &&
              hipMalloc((void **)&d.frames, (size_t)batch * (slot + 4) + 64) == hipSuccess &&
              hipMalloc((void **)&d.off, ((size_t)batch + 1) * sizeof(long long)) == hipSuccess &&
              hipMalloc((void **)&d.sizes, (size_t)batch * sizeof(int)) == hipSuccess;
    if (ok && tx)
        ok = hipMalloc((void **)&d.src, (size_t)batch * bs) == hipSuccess &&
             hipMalloc((void **)&d.comp, (size_t)batch * slot) == hipSuccess &&
             hipMalloc((void **)&d.csz, (size_t)batch * sizeof(int)) == hipSuccess &&
             hipMalloc(&d.scratch, APE_LZ4_frame_scratch_size(batch) + 16) == hipSuccess;
    if (ok && !tx)
        ok = hipMalloc((void **)&d.out, (size_t)batch * bs) == hipSuccess &&
             hipMalloc((void **)&d.res, (size_t)batch * sizeof(int)) == hipSuccess &&
             hipHostMalloc((void **)&d.hres, (size_t)batch * sizeof(int), hipHostMallocDefault) == hipSuccess;
    if (ok) {
        int *h = (int *)malloc((size_t)batch * sizeof(int));
        ok = h != nullptr;
        if (ok) {
            for (int i = 0; i < batch; i++) h[i] = bs;
            ok = hipMemcpy(d.sizes, h, (size_t)batch * sizeof(int), hipMemcpyHostToDevice) == hipSuccess;
            free(h);
        }
    }
    return ok ? 0 : -1;
}

void dev_free(Dev &d) {
    if (d.st) (void)hipStreamSynchronize(d.st);
    for (void *p : {(void *)d.src, (void *)d.comp, (void *)d.frames, (void *)d.out, (void *)d.csz,
                    (void *)d.sizes, (void *)d.res, (void *)d.off, d.scratch})
        if (p) (void)hipFree(p);
    if (d.hres) (void)hipHostFree(d.hres);
    if (d.ev) (void)hipEventDestroy(d.ev);
    for (hipEvent_t e : d.tev)
        if (e) (void)hipEventDestroy(e);
    if (d.st) (void)hipStreamDestroy(d.st);
    d = Dev();
}

}  // namespace

extern "C" {

APE_LZ4_rxbuf *APE_LZ4_rxbuf_new(size_t initial) {
    APE_LZ4_rxbuf *b = (APE_LZ4_rxbuf *)calloc(1, sizeof *b);
    if (!b) return nullptr;
    if (initial && APE_LZ4_rxbuf_prepare(b, initial) != 0) {
        free(b);
        return nullptr;
    }
    return b;
}

// buffer_prepare (ref src/ape_buffer.c:210-228): at least `more` free bytes after `used`;
// growth doubles the storage (realloc) and re-registers it for DMA.
int APE_LZ4_rxbuf_prepare(APE_LZ4_rxbuf *b, size_t more) {
    if (!b) return -1;
    if (b->size - b->used >= more && b->data) return 0;
    size_t ns = b->size ? b->size : 4096;
    while (ns - b->used < more) ns *= 2;
    rx_unregister(b);
    char *p = (char *)realloc(b->data, ns);
    if (!p) {
        (void)rx_register(b);
        return -1;
    }
    b->data = p;
    b->size = ns;
    (void)rx_register(b);   // without a device the storage stays pageable (still correct)
    return 0;
}

char *APE_LZ4_rxbuf_data(APE_LZ4_rxbuf *b) { return b ? b->data : nullptr; }
size_t APE_LZ4_rxbuf_used(const APE_LZ4_rxbuf *b) { return b ? b->used : 0; }
size_t APE_LZ4_rxbuf_room(const APE_LZ4_rxbuf *b) { return b ? b->size - b->used : 0; }
int APE_LZ4_rxbuf_pinned(const APE_LZ4_rxbuf *b) { return b ? b->registered == 1 : 0; }

// append raw bytes (what a read() into the buffer does); returns 0 or -1
int APE_LZ4_rxbuf_append(APE_LZ4_rxbuf *b, const char *data, size_t len) {
    if (APE_LZ4_rxbuf_prepare(b, len) != 0) return -1;
    memcpy(b->data + b->used, data, len);
    b->used += len;
    return 0;
}

// Complete frames [le32 size][block] at the start of the buffer: off[i] = frame i's
// header position (i < n), off[n] = the end of the last complete frame.  At most
// max_frames; a size < 0 or > max_block is malformed: -1 (the stream is unusable, as
// the reference socket's decode error, src/ape_socket.c:1393-1396).
namespace {
// frames_from: APE_LZ4_rxbuf_frames continued after the `n0` frames already found in
// off[0..n0] (off[n0] = where parsing stopped), so a receiver that reads a batch in many
// pieces parses each frame once
int frames_from(const APE_LZ4_rxbuf *b, long long *off, int n0, int max_frames, int max_block) {
    size_t pos = n0 ? (size_t)off[n0] : 0;
    int n = n0;
    while (n < max_frames && b->used - pos >= 4) {
        const unsigned char *h = (const unsigned char *)b->data + pos;
        const uint32_t sz = (uint32_t)h[0] | ((uint32_t)h[1] << 8) | ((uint32_t)h[2] << 16) |
                            ((uint32_t)h[3] << 24);
        if ((int32_t)sz < 0 || (int32_t)sz > max_block) return -1;
        if (b->used - pos - 4 < sz) break;   // the block is not all here yet
        off[n++] = (long long)pos;
        pos += 4 + (size_t)sz;
    }
    off[n] = (long long)pos;
    return n;
}
}  // namespace

int APE_LZ4_rxbuf_frames(const APE_LZ4_rxbuf *b, long long *off, int max_frames, int max_block) {
    if (!b || !off || max_frames < 0) return -1;
    size_t pos = 0;
    int n = 0;
    while (n < max_frames && b->used - pos >= 4) {
        const unsigned char *h = (const unsigned char *)b->data + pos;
        const uint32_t sz = (uint32_t)h[0] | ((uint32_t)h[1] << 8) | ((uint32_t)h[2] << 16) |
                            ((uint32_t)h[3] << 24);
        if ((int32_t)sz < 0 || (int32_t)sz > max_block) return -1;
        if (b->used - pos - 4 < sz) break;   // the block is not all here yet
        off[n++] = (long long)pos;
        pos += 4 + (size_t)sz;
    }
    off[n] = (long long)pos;
    return n;
}

// drop the first n bytes (consumed frames), keeping the rest at the start
void APE_LZ4_rxbuf_consume(APE_LZ4_rxbuf *b, size_t n) {
    if (!b) return;
    if (n >= b->used) {
        b->used = 0;
        return;
    }
    memmove(b->data, b->data + n, b->used - n);
    b->used -= n;
}

void APE_LZ4_rxbuf_free(APE_LZ4_rxbuf *b) {
    if (!b) return;
    rx_unregister(b);
    free(b->data);
    free(b);
}

// TX: compress nblocks blocks of block_size bytes (block i at h_src + i*src_stride) on the
// current device, `batch` at a time, and write the framed stream to fd.  Returns the
// bytes written, or a negative APE_LZ4_GPU_E* code.
long long APE_LZ4_socket_send_blocks(int fd, const char *h_src, size_t src_stride,
                                     int block_size, int nblocks, int batch) {
    if (fd < 0 || !h_src || block_size <= 0 || block_size > kMaxBlock || nblocks < 0 || batch <= 0 ||
        src_stride < (size_t)block_size)
        return APE_LZ4_GPU_EINVAL;
    int rc = APE_LZ4_gpu_init();
    if (rc) return rc;
    const size_t slot = up16((size_t)bound_of(block_size));
    Dev d[2];
    char *hf[2] = {nullptr, nullptr};
    long long *htot[2] = {nullptr, nullptr};
    long long sent = 0;
    int nb[2] = {0, 0};
    const int nbat = (nblocks + batch - 1) / batch;
    for (int i = 0; i < 2 && rc == 0; i++) {
        if (dev_alloc(d[i], batch, block_size, true) != 0 ||
            hipHostMalloc((void **)&hf[i], (size_t)batch * (slot + 4) + 64, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void **)&htot[i], sizeof(long long), hipHostMallocDefault) != hipSuccess)
            rc = APE_LZ4_GPU_ENOMEM;
    }
    auto launch = [&](int c) -> int {
        Dev &D = d[c & 1];
        const int k = nblocks - c * batch < batch ? nblocks - c * batch : batch;
        nb[c & 1] = k;
        const char *src = h_src + (size_t)c * batch * src_stride;
        (void)hipEventRecord(D.tev[0], D.st);
        hipError_t e = hipMemcpy2DAsync(D.src, (size_t)block_size, src, src_stride, (size_t)block_size,
                                        (size_t)k, hipMemcpyHostToDevice, D.st);
        if (e != hipSuccess) return APE_LZ4_GPU_ELAUNCH;
        (void)hipEventRecord(D.tev[1], D.st);
        int r = APE_LZ4_compress_batch_strided_dev(D.src, (size_t)block_size, D.sizes, D.comp, slot,
                                                   nullptr, D.csz, k, D.st);
        if (r == 0) r = APE_LZ4_frame_offsets_dev(D.csz, D.off, D.scratch, k, D.st);
        if (r == 0) r = APE_LZ4_frame_pack_strided_dev(D.comp, slot, D.csz, D.off, D.frames, k, D.st);
        if (r) return r;
        (void)hipEventRecord(D.tev[2], D.st);
        e = hipMemcpyAsync(htot[c & 1], D.off + k, sizeof(long long), hipMemcpyDeviceToHost, D.st);
        if (e == hipSuccess) e = hipEventRecord(D.ev, D.st);
        return e == hipSuccess ? 0 : APE_LZ4_GPU_ELAUNCH;
    };
    const long long ttx = now_ns();
    if (rc == 0 && nbat > 0) rc = launch(0);
    for (int c = 0; c < nbat && rc == 0; c++) {
        Dev &D = d[c & 1];
        long long t0 = now_ns();
        if (hipEventSynchronize(D.ev) != hipSuccess) { rc = APE_LZ4_GPU_ELAUNCH; break; }
        const long long tot = *htot[c & 1];
        (void)hipEventRecord(D.tev[3], D.st);
        if (hipMemcpyAsync(hf[c & 1], D.frames, (size_t)tot, hipMemcpyDeviceToHost, D.st) != hipSuccess ||
            hipEventRecord(D.tev[4], D.st) != hipSuccess || hipStreamSynchronize(D.st) != hipSuccess) {
            rc = APE_LZ4_GPU_ELAUNCH;
            break;
        }
        long long t1 = now_ns();
        sock_add(4, t1 - t0);
        sock_add(0, ev_ns(D.tev[0], D.tev[1]));
        sock_add(1, ev_ns(D.tev[1], D.tev[2]));
        sock_add(2, ev_ns(D.tev[3], D.tev[4]));
        sock_add(5, 1);
        if (c + 1 < nbat) rc = launch(c + 1);   // the next batch's GPU work under this write
        if (rc) break;
        t0 = now_ns();
        const long long w = write_all(fd, hf[c & 1], (size_t)tot);
        sock_add(3, now_ns() - t0);
        if (w < 0) { rc = APE_LZ4_GPU_EINVAL; break; }
        sent += w;
    }
    sock_add(6, now_ns() - ttx);
    for (int i = 0; i < 2; i++) {
        dev_free(d[i]);
        if (hf[i]) (void)hipHostFree(hf[i]);
        if (htot[i]) (void)hipHostFree(htot[i]);
    }
    return rc ? rc : sent;
}

// RX: read the framed stream from fd into pinned rxbufs, decode `batch` frames at a time
// on the current device into block i at h_dst + i*dst_stride (capacity block_size),
// h_result[i] = decompress_safe's result.  Returns the blocks received, or a negative
// APE_LZ4_GPU_E* code (APE_LZ4_GPU_EINVAL also for a malformed frame or early EOF).
long long APE_LZ4_socket_recv_blocks(int fd, char *h_dst, size_t dst_stride, int block_size,
                                     int nblocks, int batch, int *h_result) {
    if (fd < 0 || !h_dst || !h_result || block_size <= 0 || block_size > kMaxBlock ||
        nblocks < 0 || batch <= 0 ||
        dst_stride < (size_t)block_size)
        return APE_LZ4_GPU_EINVAL;
    int rc = APE_LZ4_gpu_init();
    if (rc) return rc;
    const int maxc = bound_of(block_size);
    const size_t chunk = 4u << 20;   // read() granularity
    Dev d[2];
    APE_LZ4_rxbuf *rb[2] = {APE_LZ4_rxbuf_new(4u << 20), APE_LZ4_rxbuf_new(4u << 20)};
    long long *hoff[2] = {nullptr, nullptr};
    bool busy[2] = {false, false};
    long long base[2] = {0, 0};   // first block of the batch in flight on d[i]
    int cnt[2] = {0, 0};          // ... and its block count
    for (int i = 0; i < 2 && rc == 0; i++) {
        if (!rb[i] || dev_alloc(d[i], batch, block_size, false) != 0 ||
            hipHostMalloc((void **)&hoff[i], ((size_t)batch + 1) * sizeof(long long),
                          hipHostMallocDefault) != hipSuccess)
            rc = APE_LZ4_GPU_ENOMEM;
    }
    long long done = 0;       // blocks handed to the GPU
    const long long trx = now_ns();
    int cur = 0;              // rxbuf receiving
    int parsed = 0;           // complete frames already found in rb[cur]
    bool eof = false;
    while (rc == 0 && done < nblocks) {
        APE_LZ4_rxbuf *b = rb[cur];
        const int want = nblocks - done < batch ? (int)(nblocks - done) : batch;
        long long t0 = now_ns();
        const int n = frames_from(b, hoff[cur], parsed, want, maxc);
        sock_add(9, now_ns() - t0);
        if (n < 0) { rc = APE_LZ4_GPU_EINVAL; break; }
        parsed = n;
        if (n < want) {   // read more
            if (eof) { rc = APE_LZ4_GPU_EINVAL; break; }
            t0 = now_ns();
            if (APE_LZ4_rxbuf_prepare(b, chunk) != 0) { rc = APE_LZ4_GPU_ENOMEM; break; }
            sock_add(15, now_ns() - t0);
            t0 = now_ns();
            const ssize_t r = read(fd, b->data + b->used, b->size - b->used);
            sock_add(8, now_ns() - t0);
            if (r < 0) {
                if (errno == EINTR) continue;
                rc = APE_LZ4_GPU_EINVAL;
                break;
            }
            if (r == 0) eof = true;
            b->used += (size_t)r;
            continue;
        }
        // a full batch: hand this buffer to the GPU, continue receiving in the other one
        const int nxt = cur ^ 1;
        if (busy[nxt]) {
            t0 = now_ns();
            if (hipStreamSynchronize(d[nxt].st) != hipSuccess) { rc = APE_LZ4_GPU_ELAUNCH; break; }
            sock_add(13, now_ns() - t0);
            Dev &P = d[nxt];
            sock_add(10, ev_ns(P.tev[0], P.tev[1]));
            sock_add(11, ev_ns(P.tev[1], P.tev[2]));
            sock_add(12, ev_ns(P.tev[2], P.tev[3]));
            sock_add(14, 1);
            memcpy(h_result + base[nxt], P.hres, (size_t)cnt[nxt] * sizeof(int));
            busy[nxt] = false;
        }
        const size_t end = (size_t)hoff[cur][n];
        APE_LZ4_rxbuf *o = rb[nxt];
        o->used = 0;
        t0 = now_ns();
        if (APE_LZ4_rxbuf_append(o, b->data + end, b->used - end) != 0) { rc = APE_LZ4_GPU_ENOMEM; break; }
        sock_add(9, now_ns() - t0);
        b->used = end;
        Dev &D = d[cur];
        (void)hipEventRecord(D.tev[0], D.st);
        hipError_t e = hipMemcpyAsync(D.frames, b->data, end, hipMemcpyHostToDevice, D.st);
        if (e == hipSuccess)
            e = hipMemcpyAsync(D.off, hoff[cur], ((size_t)n + 1) * sizeof(long long),
                               hipMemcpyHostToDevice, D.st);
        if (e != hipSuccess) { rc = APE_LZ4_GPU_ELAUNCH; break; }
        (void)hipEventRecord(D.tev[1], D.st);
        rc = APE_LZ4_decompress_safe_frames_dev(D.frames, D.off, D.out, (size_t)block_size, D.sizes,
                                                D.res, n, D.st);
        if (rc) break;
        (void)hipEventRecord(D.tev[2], D.st);
        e = hipMemcpy2DAsync(h_dst + (size_t)done * dst_stride, dst_stride, D.out, (size_t)block_size,
                             (size_t)block_size, (size_t)n, hipMemcpyDeviceToHost, D.st);
        if (e == hipSuccess)
            e = hipMemcpyAsync(D.hres, D.res, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, D.st);
        if (e == hipSuccess) e = hipEventRecord(D.tev[3], D.st);
        if (e != hipSuccess) { rc = APE_LZ4_GPU_ELAUNCH; break; }
        busy[cur] = true;
        base[cur] = done;
        cnt[cur] = n;
        done += n;
        cur = nxt;
        parsed = 0;
    }
    sock_add(7, now_ns() - trx);
    for (int i = 0; i < 2; i++) {   // drain every batch in flight, whatever rc is
        if (!busy[i]) continue;
        if (hipStreamSynchronize(d[i].st) != hipSuccess) {
            if (rc == 0) rc = APE_LZ4_GPU_ELAUNCH;   // its results never reached h_result
            continue;
        }
        if (rc == 0) {   // the last batches' results and stage times
            sock_add(10, ev_ns(d[i].tev[0], d[i].tev[1]));
            sock_add(11, ev_ns(d[i].tev[1], d[i].tev[2]));
            sock_add(12, ev_ns(d[i].tev[2], d[i].tev[3]));
            sock_add(14, 1);
            memcpy(h_result + base[i], d[i].hres, (size_t)cnt[i] * sizeof(int));
        }
    }
    for (int i = 0; i < 2; i++) {
        dev_free(d[i]);
        APE_LZ4_rxbuf_free(rb[i]);
        if (hoff[i]) (void)hipHostFree(hoff[i]);
    }
    return rc ? rc : done;
}

}  // extern "C"

// ---------------------------------------------------------------------------------
// Chained streams: the reference wire format through the GPU.
//
// The reference socket sends every message cut into 8 KiB chunks (APE_LZ4_BLOCK_SIZE,
// src/ape_socket.c:39), each compressed with compress_fast_continue against the previous
// <= 64 KiB of the connection's stream and framed [int32 size][block] (:811-871; saveDict
// after the message keeps the history, :856); the receiver decodes each frame with
// decompress_safe_continue against its 64 KiB dictionary buffer (:1386-1421).  A server holds
// many connections, so the GPU batches them, K messages per connection per round:
//   TX: a chunk's history is plaintext the sender already has, so every chunk of the round
//       (nconn x K x nch) is compressed in ONE withPrefix launch, each against the bytes
//       before it in its connection's device window; the frames are packed on the GPU and
//       each connection's frames of the round are written to its socket with one write().
//   RX: per connection a receive buffer with the split-safe parser; a round takes K messages
//       (K x nch frames) from every connection and decodes them with K x nch usingDict
//       launches of nconn blocks each (chunk q + 1's dictionary is chunk q's output: the
//       chunks of one stream are sequential, the connections are the batch).
// Both sides keep a window of W bytes per connection on the device; when the next round
// would pass its end, the last 64 KiB move to its start (one 2-D device copy for all).
// Bytes on the wire: exactly the reference's format, so an unmodified reference peer reads
// what chain_send writes and writes what chain_recv reads (tests/test_sock.py).
namespace {

constexpr int kChunk = 8192;                      // APE_LZ4_BLOCK_SIZE (:39)
constexpr int kChunkBound = kChunk + kChunk / 255 + 16;   // APE_LZ4_COMPRESSBOUND(8192)
constexpr size_t kChunkSlot = (kChunkBound + 15) & ~15;
constexpr int kHist = 65536;                      // the dictionary (:43)
constexpr size_t kRoundBytes = 32u << 20;         // payload per round (all connections)

// TX pointer arrays of a round of k messages: chunk t = (connection i, message mm, chunk j),
// t = (i * k + mm) * nch + j -- connection-major, so a connection's frames are contiguous
__global__ void chain_tx_setup(char *win, size_t W, uint32_t pos, int msg, int nch, int k, int n,
                               char *slots, const char **src, int *size, int *pre, char **dst,
                               int *cap) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const int i = t / (k * nch), r = t - i * k * nch, mm = r / nch, j = r - mm * nch;
    const int len = msg - kChunk * j < kChunk ? msg - kChunk * j : kChunk;
    const uint32_t at = pos + (uint32_t)mm * (uint32_t)msg + (uint32_t)(kChunk * j);
    src[t] = win + (size_t)i * W + at;
    size[t] = len;
    pre[t] = (int)at;   // the whole stream so far (the encoder keeps what fits its window)
    dst[t] = slots + (size_t)t * kChunkSlot;
    cap[t] = len + len / 255 + 16;
}

// RX pointer arrays of a round, chunk-major: launch q (= mm * nch + j) decodes entries
// [q * nconn, (q + 1) * nconn); entry q * nconn + i = chunk q of connection i, its payload at
// stage + poff[i * k * nch + q]
__global__ void chain_rx_setup(const char *stage, const long long *poff, char *win, size_t W,
                               uint32_t pos, int msg, int nch, int k, int nconn, const char **src,
                               char **dst, int *cap, const char **dict, int *dsz) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= k * nch * nconn) return;
    const int q = e / nconn, i = e - q * nconn, mm = q / nch, j = q - mm * nch;
    const uint32_t at = pos + (uint32_t)mm * (uint32_t)msg + (uint32_t)(kChunk * j);
    const uint32_t h = at < (uint32_t)kHist ? at : (uint32_t)kHist;
    src[e] = stage + poff[(size_t)i * k * nch + q];
    dst[e] = win + (size_t)i * W + at;
    cap[e] = msg - kChunk * j < kChunk ? msg - kChunk * j : kChunk;
    dict[e] = win + (size_t)i * W + at - h;
    dsz[e] = (int)h;
}

}  // namespace

// One part of a chain: a subset of the connections served by one host thread with its own
// streams and buffers (APE_LZ4_chain below splits the connections over kChainThreads parts).
struct ChainPart {
    int dev = 0, nconn = 0, msg = 0, nch = 0, K = 1, nt = 0;   // nt = chunks of a full round
    bool loop = true;                // RX: one looping launch per round (APE_LZ4_CHAIN_LOOP=0: one
                                     // launch per chunk position)
    size_t W = 0;
    // TX (one thread): device window, compressed slots, frames, pointer arrays
    hipStream_t tst = nullptr;
    hipEvent_t tev[2] = {nullptr, nullptr};
    char *txwin = nullptr, *slots = nullptr;
    int *csz = nullptr, *size = nullptr, *pre = nullptr, *cap = nullptr;
    const char **src = nullptr;
    char **dst = nullptr;
    long long *off = nullptr;
    void *scratch = nullptr;
    char *h_frames[2] = {nullptr, nullptr};   // pinned; the pack kernel writes them (zero-copy)
    char *d_hframes[2] = {nullptr, nullptr};  // their device-mapped addresses
    long long *h_off[2] = {nullptr, nullptr};
    uint32_t txpos = 0;
    // RX (one thread): device window, staged payloads, pointer arrays, results
    hipStream_t rst = nullptr;
    hipEvent_t rev[2] = {nullptr, nullptr};
    char *rxwin = nullptr, *rstage[2] = {nullptr, nullptr};
    long long *rpoff[2] = {nullptr, nullptr};
    int *rcsz[2] = {nullptr, nullptr}, *rcap = nullptr, *rdsz = nullptr, *rres[2] = {nullptr, nullptr};
    const char **rsrc = nullptr, **rdict = nullptr;
    char **rdst = nullptr;
    char *h_stage[2] = {nullptr, nullptr};
    long long *h_poff[2] = {nullptr, nullptr};
    int *h_csz[2] = {nullptr, nullptr}, *h_res[2] = {nullptr, nullptr};
    uint32_t rxpos = 0;
    // per-connection receive buffers, kept across recv calls: a read may take in frames beyond
    // the messages one call needs, and the next call on the chain resumes with those bytes
    std::vector<APE_LZ4_rxbuf *> rb;
    std::vector<char> eof;
    // sticky failure: a failed call has consumed frames and advanced the stream
    // position / history of its direction for the rounds it ran, so no later call in that
    // direction can be correct -- each returns APE_LZ4_GPU_EINVAL until the chain is freed
    bool tx_failed = false, rx_failed = false;
};

namespace {

void chain_release(ChainPart *c) {
    if (c->tst) (void)hipStreamSynchronize(c->tst);
    if (c->rst) (void)hipStreamSynchronize(c->rst);
    for (void *p : {(void *)c->txwin, (void *)c->slots, (void *)c->csz,
                    (void *)c->size, (void *)c->pre, (void *)c->cap, (void *)c->src, (void *)c->dst,
                    (void *)c->off, c->scratch, (void *)c->rxwin, (void *)c->rstage[0],
                    (void *)c->rstage[1], (void *)c->rpoff[0], (void *)c->rpoff[1],
                    (void *)c->rcsz[0], (void *)c->rcsz[1], (void *)c->rcap, (void *)c->rdsz,
                    (void *)c->rres[0], (void *)c->rres[1], (void *)c->rsrc, (void *)c->rdict,
                    (void *)c->rdst})
        if (p) (void)hipFree(p);
    for (void *p : {(void *)c->h_frames[0], (void *)c->h_frames[1], (void *)c->h_off[0], (void *)c->h_off[1],
                    (void *)c->h_stage[0], (void *)c->h_stage[1], (void *)c->h_poff[0],
                    (void *)c->h_poff[1], (void *)c->h_csz[0], (void *)c->h_csz[1],
                    (void *)c->h_res[0], (void *)c->h_res[1]})
        if (p) (void)hipHostFree(p);
    for (APE_LZ4_rxbuf *b : c->rb) APE_LZ4_rxbuf_free(b);
    for (hipEvent_t e : {c->tev[0], c->tev[1], c->rev[0], c->rev[1]})
        if (e) (void)hipEventDestroy(e);
    if (c->tst) (void)hipStreamDestroy(c->tst);
    if (c->rst) (void)hipStreamDestroy(c->rst);
    delete c;
}

template <typename T>
bool dalloc(T *&p, size_t n) { return hipMalloc((void **)&p, n * sizeof(T)) == hipSuccess; }
template <typename T>
bool halloc(T *&p, size_t n) {
    return hipHostMalloc((void **)&p, n * sizeof(T), hipHostMallocDefault) == hipSuccess;
}

// the window slides when the next round (`need` bytes) would pass its end: the last <= 64 KiB
// of every connection's stream move to the start of its row (a 2-D device copy; a row never
// overlaps its source since W >= 2 x 64 KiB + a round)
hipError_t chain_slide(char *win, size_t W, int nconn, uint32_t &pos, size_t need, hipStream_t st) {
    if ((size_t)pos + need <= W) return hipSuccess;
    const uint32_t keep = pos < (uint32_t)kHist ? pos : (uint32_t)kHist;
    const hipError_t e = hipMemcpy2DAsync(win, W, win + (pos - keep), W, keep, (size_t)nconn,
                                          hipMemcpyDeviceToDevice, st);
    pos = keep;
    return e;
}

inline int chunk_len(int msg, int j) { return msg - kChunk * j < kChunk ? msg - kChunk * j : kChunk; }

ChainPart *part_new(int nconn, int msg_len, int dev) {
    ChainPart *c = new ChainPart();
    c->dev = dev;
    c->nconn = nconn;
    c->msg = msg_len;
    c->nch = (msg_len + kChunk - 1) / kChunk;
    const size_t per = (size_t)nconn * (size_t)msg_len;
    c->K = (int)(per >= kRoundBytes ? 1 : (kRoundBytes / per < 16 ? kRoundBytes / per : 16));
    if (const char *ev = getenv("APE_LZ4_CHAIN_ROUND")) {   // messages per round (tests: many rounds)
        const int k = atoi(ev);
        if (k >= 1 && k <= 64) c->K = k;
    }
    if (const char *ev = getenv("APE_LZ4_CHAIN_LOOP")) c->loop = atoi(ev) != 0;
    c->nt = nconn * c->K * c->nch;
    c->W = ((size_t)2 * kHist + (size_t)c->K * msg_len + 255) & ~(size_t)255;
    const size_t nt = (size_t)c->nt, fr = nt * (kChunkSlot + 4) + 64;
    // RX at the highest stream priority, TX at the lowest: the receive side is a chain of small
    // dependent launches (one per chunk position, each one chunk per connection) whose latency
    // bounds the connection's rate, while the TX launch of a round is one large batch; the
    // parts' streams share the device's hardware queues (APE_LZ4_CHAIN_PRIO=0: default priority)
    int lo = 0, hi = 0;   // numerically: lo = least, hi = greatest priority
    const char *pe = getenv("APE_LZ4_CHAIN_PRIO");
    if (!(pe && atoi(pe) == 0) && hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
    if (pe && atoi(pe) == 0) lo = hi = 0;
    bool ok = hipStreamCreateWithPriority(&c->tst, hipStreamNonBlocking, lo) == hipSuccess &&
              hipStreamCreateWithPriority(&c->rst, hipStreamNonBlocking, hi) == hipSuccess;
    for (int b = 0; b < 2 && ok; b++)
        ok = hipEventCreateWithFlags(&c->tev[b], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&c->rev[b], hipEventDisableTiming) == hipSuccess &&
             halloc(c->h_off[b], nt + 1) && halloc(c->h_frames[b], fr) &&
             hipHostGetDevicePointer((void **)&c->d_hframes[b], c->h_frames[b], 0) == hipSuccess &&
             dalloc(c->rstage[b], fr) && dalloc(c->rpoff[b], nt) &&
             dalloc(c->rcsz[b], nt) && dalloc(c->rres[b], nt) && halloc(c->h_stage[b], fr) &&
             halloc(c->h_poff[b], nt) && halloc(c->h_csz[b], nt) && halloc(c->h_res[b], nt);
    ok = ok && dalloc(c->txwin, (size_t)nconn * c->W) && dalloc(c->slots, nt * kChunkSlot) &&
         dalloc(c->csz, nt) && dalloc(c->size, nt) && dalloc(c->pre, nt) &&
         dalloc(c->cap, nt) && dalloc(c->src, nt) && dalloc(c->dst, nt) && dalloc(c->off, nt + 1) &&
         hipMalloc(&c->scratch, APE_LZ4_frame_scratch_size(c->nt) + 16) == hipSuccess &&
         dalloc(c->rxwin, (size_t)nconn * c->W) && dalloc(c->rcap, nt) &&
         dalloc(c->rdsz, nt) && dalloc(c->rsrc, nt) && dalloc(c->rdict, nt) && dalloc(c->rdst, nt);
    if (!ok) {
        chain_release(c);
        return nullptr;
    }
    return c;
}

// TX of one part: nmsg messages per connection (message m of local connection i at h_msgs +
// m * row_pitch + i * msg_stride) as the reference's frames on fds[i], in rounds of K messages.
// Returns the bytes written or an error code.
long long part_send(ChainPart *c, const int *fds, const char *h_msgs, size_t msg_stride,
                    size_t row_pitch, int nmsg) {
    if (c->tx_failed) return APE_LZ4_GPU_EINVAL;
    if (hipSetDevice(c->dev) != hipSuccess) return APE_LZ4_GPU_ENODEV;
    const int M = c->nconn, nch = c->nch, nr = (nmsg + c->K - 1) / c->K;
    long long sent = 0;
    int rc = 0;
    auto round_k = [&](int r) { return nmsg - r * c->K < c->K ? nmsg - r * c->K : c->K; };
    auto launch = [&](int r) -> int {
        const int b = r & 1, k = round_k(r), nt = M * k * nch;
        if (chain_slide(c->txwin, c->W, M, c->txpos, (size_t)k * c->msg, c->tst) != hipSuccess)
            return APE_LZ4_GPU_ELAUNCH;
        for (int mm = 0; mm < k; mm++) {
            const char *h = h_msgs + (size_t)(r * c->K + mm) * row_pitch;
            if (hipMemcpy2DAsync(c->txwin + c->txpos + (size_t)mm * c->msg, c->W, h, msg_stride,
                                 (size_t)c->msg, (size_t)M, hipMemcpyHostToDevice, c->tst) != hipSuccess)
                return APE_LZ4_GPU_ELAUNCH;
        }
        hipLaunchKernelGGL(chain_tx_setup, dim3((nt + 255) / 256), dim3(256), 0, c->tst, c->txwin,
                           c->W, c->txpos, c->msg, nch, k, nt, c->slots, c->src, c->size, c->pre,
                           c->dst, c->cap);
        if (hipGetLastError() != hipSuccess) return APE_LZ4_GPU_ELAUNCH;
        int e = APE_LZ4_compress_withPrefix_batch_dev(c->src, c->size, c->pre, c->dst, c->cap,
                                                      c->csz, nt, c->tst);
        if (e == 0) e = APE_LZ4_frame_offsets_dev(c->csz, c->off, c->scratch, nt, c->tst);
        // frames straight into the pinned send buffer of this round (zero-copy)
        if (e == 0) e = APE_LZ4_frame_pack_strided_dev(c->slots, kChunkSlot, c->csz, c->off, c->d_hframes[b], nt, c->tst);
        if (e) return e;
        if (hipMemcpyAsync(c->h_off[b], c->off, ((size_t)nt + 1) * sizeof(long long),
                           hipMemcpyDeviceToHost, c->tst) != hipSuccess ||
            hipEventRecord(c->tev[b], c->tst) != hipSuccess)
            return APE_LZ4_GPU_ELAUNCH;
        c->txpos += (uint32_t)(k * c->msg);
        return 0;
    };
    const long long t_all = now_ns();
    if (nr > 0) rc = launch(0);
    for (int r = 0; r < nr && rc == 0; r++) {
        const int b = r & 1, k = round_k(r), nt = M * k * nch;
        long long t0 = now_ns();
        if (hipEventSynchronize(c->tev[b]) != hipSuccess) { rc = APE_LZ4_GPU_ELAUNCH; break; }
        const long long *off = c->h_off[b];
        // a chunk that did not fit its bound is a codec failure (never for valid sizes): its
        // csz <= 0 would go out as a frame the reference receiver rejects, so any one fails
        // the round (frame j spans off[j+1] - off[j] = 4 + csz bytes)
        for (int j = 0; j < nt && rc == 0; j++)
            if (off[j + 1] - off[j] <= 4) rc = APE_LZ4_GPU_ELAUNCH;
        if (rc) break;
        sock_add(4, now_ns() - t0);
        sock_add(5, 1);
        if (r + 1 < nr) rc = launch(r + 1);   // the next round's GPU work under these writes
        if (rc) break;
        t0 = now_ns();
        for (int i = 0; i < M && rc == 0; i++) {   // connection i's frames of the round
            const long long a = off[(size_t)i * k * nch], e = off[(size_t)(i + 1) * k * nch];
            const long long w = write_all(fds[i], c->h_frames[b] + a, (size_t)(e - a));
            if (w < 0) rc = APE_LZ4_GPU_EINVAL;
            else sent += w;
        }
        sock_add(3, now_ns() - t0);
    }
    if (hipStreamSynchronize(c->tst) != hipSuccess && rc == 0) rc = APE_LZ4_GPU_ELAUNCH;
    sock_add(6, now_ns() - t_all);
    if (rc) c->tx_failed = true;
    return rc ? rc : sent;
}

// RX of one part: nmsg messages per connection, in rounds of K; message m of local connection i
// is decoded into h_out + m * row_pitch + i * out_stride.  h_status[i] = 0, or the first failing
// chunk's result (decompress_safe_continue's value, or the wrong size it produced); a failing
// connection makes the call return APE_LZ4_GPU_EINVAL.  Returns the payload bytes delivered or
// an error code (EINVAL also for a malformed frame or an early EOF).
long long part_recv(ChainPart *c, const int *fds, char *h_out, size_t out_stride, size_t row_pitch,
                    int nmsg, int *h_status) {
    if (c->rx_failed) {
        for (int i = 0; i < c->nconn; i++) h_status[i] = -1;
        return APE_LZ4_GPU_EINVAL;
    }
    if (hipSetDevice(c->dev) != hipSuccess) return APE_LZ4_GPU_ENODEV;
    const int M = c->nconn, nch = c->nch, nr = (nmsg + c->K - 1) / c->K;
    const int maxf = c->K * nch;   // frames of a full round per connection
    std::vector<long long> offs((size_t)M * (maxf + 1), 0);
    std::vector<int> parsed((size_t)M, 0);
    std::vector<pollfd> pf((size_t)M);
    std::vector<int> pmap((size_t)M);
    int rc = 0;
    if (c->rb.empty()) {
        c->rb.assign((size_t)M, nullptr);
        c->eof.assign((size_t)M, 0);
    }
    std::vector<APE_LZ4_rxbuf *> &rb = c->rb;
    std::vector<char> &eof = c->eof;
    for (int i = 0; i < M; i++) {   // host-only buffers: the payloads go to the GPU through
        h_status[i] = 0;            // the pinned staging area, so no per-connection registration
        if (!rb[i]) {
            rb[i] = (APE_LZ4_rxbuf *)calloc(1, sizeof(APE_LZ4_rxbuf));
            if (rb[i]) rb[i]->registered = -1;
        }
        if (!rb[i] || APE_LZ4_rxbuf_prepare(rb[i], 1u << 16) != 0) rc = APE_LZ4_GPU_ENOMEM;
    }
    auto round_k = [&](int r) { return nmsg - r * c->K < c->K ? nmsg - r * c->K : c->K; };
    long long got = 0;
    bool busy[2] = {false, false};
    int bk[2] = {0, 0};   // messages of the round in flight on slot b
    auto check = [&](int b) {   // results of the round on slot b (its event has completed)
        const int *res = c->h_res[b];
        bool bad = false;
        for (int q = 0; q < bk[b] * nch; q++) {
            const int want = chunk_len(c->msg, q % nch);
            for (int i = 0; i < M; i++) {
                const int v = res[(size_t)q * M + i];
                if (v != want && h_status[i] == 0) {
                    h_status[i] = v != 0 ? v : -1;
                    bad = true;
                }
            }
        }
        if (!bad) got += (long long)M * bk[b] * c->msg;
        busy[b] = false;
        return bad ? APE_LZ4_GPU_EINVAL : 0;
    };
    const long long t_all = now_ns();
    for (int r = 0; r < nr && rc == 0; r++) {
        const int k = round_k(r), nf = k * nch, ne = M * nf;
        // ---- receive until every connection holds the round's k x nch frames (split-safe) ----
        long long t0 = now_ns();
        for (;;) {
            int np = 0;
            for (int i = 0; i < M; i++) {
                long long *o = &offs[(size_t)i * (maxf + 1)];
                if (parsed[i] < nf) {
                    const int n = frames_from(rb[i], o, parsed[i], nf, kChunkBound);
                    if (n < 0) { rc = APE_LZ4_GPU_EINVAL; break; }
                    parsed[i] = n;
                }
                if (parsed[i] < nf) {
                    if (eof[i]) { rc = APE_LZ4_GPU_EINVAL; break; }
                    pf[np].fd = fds[i];
                    pf[np].events = POLLIN;
                    pf[np].revents = 0;
                    pmap[np++] = i;
                }
            }
            if (rc || np == 0) break;
            if (poll(pf.data(), (nfds_t)np, -1) < 0) {
                if (errno == EINTR) continue;
                rc = APE_LZ4_GPU_EINVAL;
                break;
            }
            for (int q = 0; q < np && rc == 0; q++) {
                if (!(pf[q].revents & (POLLIN | POLLHUP | POLLERR))) continue;
                const int i = pmap[q];
                APE_LZ4_rxbuf *bf = rb[i];
                if (APE_LZ4_rxbuf_prepare(bf, 1u << 18) != 0) { rc = APE_LZ4_GPU_ENOMEM; break; }
                const ssize_t n = read(fds[i], bf->data + bf->used, bf->size - bf->used);
                if (n < 0) {
                    if (errno == EINTR || errno == EAGAIN) continue;
                    rc = APE_LZ4_GPU_EINVAL;
                    break;
                }
                if (n == 0) eof[i] = 1;
                bf->used += (size_t)n;
            }
        }
        sock_add(8, now_ns() - t0);
        if (rc) break;
        const int b = r & 1;
        t0 = now_ns();
        if (busy[b]) {   // round r - 2 used these buffers
            if (hipEventSynchronize(c->rev[b]) != hipSuccess) { rc = APE_LZ4_GPU_ELAUNCH; break; }
            rc = check(b);
            if (rc) break;
        }
        sock_add(13, now_ns() - t0);
        // ---- stage the round's payloads (packed, 16-byte aligned starts) ----
        t0 = now_ns();
        size_t at = 0;
        for (int i = 0; i < M; i++) {
            const long long *o = &offs[(size_t)i * (maxf + 1)];
            for (int q = 0; q < nf; q++) {
                const unsigned char *hp = (const unsigned char *)rb[i]->data + o[q];
                const int sz = (int)((uint32_t)hp[0] | ((uint32_t)hp[1] << 8) | ((uint32_t)hp[2] << 16) |
                                     ((uint32_t)hp[3] << 24));
                memcpy(c->h_stage[b] + at, hp + 4, (size_t)sz);
                c->h_poff[b][(size_t)i * nf + q] = (long long)at;
                c->h_csz[b][(size_t)q * M + i] = sz;
                at = (at + (size_t)sz + 15) & ~(size_t)15;
            }
            APE_LZ4_rxbuf_consume(rb[i], (size_t)o[nf]);
            parsed[i] = 0;
        }
        sock_add(9, now_ns() - t0);
        // ---- H2D, k x nch usingDict launches of M blocks, D2H into the caller's rows ----
        if (chain_slide(c->rxwin, c->W, M, c->rxpos, (size_t)k * c->msg, c->rst) != hipSuccess) {
            rc = APE_LZ4_GPU_ELAUNCH;
            break;
        }
        hipError_t e = hipMemcpyAsync(c->rstage[b], c->h_stage[b], at + 16, hipMemcpyHostToDevice, c->rst);
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->rpoff[b], c->h_poff[b], (size_t)ne * sizeof(long long), hipMemcpyHostToDevice, c->rst);
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->rcsz[b], c->h_csz[b], (size_t)ne * sizeof(int), hipMemcpyHostToDevice, c->rst);
        if (e != hipSuccess) { rc = APE_LZ4_GPU_ELAUNCH; break; }
        hipLaunchKernelGGL(chain_rx_setup, dim3((ne + 255) / 256), dim3(256), 0, c->rst, c->rstage[b],
                           c->rpoff[b], c->rxwin, c->W, c->rxpos, c->msg, nch, k, M, c->rsrc, c->rdst,
                           c->rcap, c->rdict, c->rdsz);
        if (hipGetLastError() != hipSuccess) { rc = APE_LZ4_GPU_ELAUNCH; break; }
        if (c->loop) {   // one launch: workgroup i decodes connection i's nf chunks in order
            BlockArgs a{};
            a.src = c->rsrc;
            a.src_size = c->rcsz[b];
            a.dst = c->rdst;
            a.dst_cap = c->rcap;
            a.dict = c->rdict;
            a.dict_size = c->rdsz;
            a.result = c->rres[b];
            a.nblocks = ne;
            if (apelz4::launch_decode_chain(a, M, nf, c->rst) != hipSuccess) rc = APE_LZ4_GPU_ELAUNCH;
        } else {         // a usingDict launch per chunk position
            for (int q = 0; q < nf && rc == 0; q++) {
                const size_t e0 = (size_t)q * M;
                rc = APE_LZ4_decompress_safe_usingDict_batch_dev(c->rsrc + e0, c->rcsz[b] + e0,
                                                                 c->rdst + e0, c->rcap + e0,
                                                                 c->rdict + e0, c->rdsz + e0,
                                                                 c->rres[b] + e0, M, c->rst);
            }
        }
        if (rc) break;
        for (int mm = 0; mm < k && e == hipSuccess; mm++)
            e = hipMemcpy2DAsync(h_out + (size_t)(r * c->K + mm) * row_pitch, out_stride,
                                 c->rxwin + c->rxpos + (size_t)mm * c->msg, c->W, (size_t)c->msg,
                                 (size_t)M, hipMemcpyDeviceToHost, c->rst);
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->h_res[b], c->rres[b], (size_t)ne * sizeof(int), hipMemcpyDeviceToHost, c->rst);
        if (e == hipSuccess) e = hipEventRecord(c->rev[b], c->rst);
        if (e != hipSuccess) { rc = APE_LZ4_GPU_ELAUNCH; break; }
        busy[b] = true;
        bk[b] = k;
        sock_add(14, 1);
        c->rxpos += (uint32_t)(k * c->msg);
    }
    // drain every round in flight, whatever rc is, before the buffers are reused
    for (int b2 = 0; b2 < 2; b2++) {
        const int b = (nr + b2) & 1;   // the older round first
        if (!busy[b]) continue;
        if (hipEventSynchronize(c->rev[b]) != hipSuccess) {
            if (rc == 0) rc = APE_LZ4_GPU_ELAUNCH;
            busy[b] = false;
            continue;
        }
        const int r2 = check(b);
        if (rc == 0) rc = r2;
    }
    // an error path may leave copies into h_out / out of h_stage queued for a round that never
    // became busy: nothing of this call is in flight when it returns
    if (hipStreamSynchronize(c->rst) != hipSuccess && rc == 0) rc = APE_LZ4_GPU_ELAUNCH;
    sock_add(7, now_ns() - t_all);
    if (rc) c->rx_failed = true;
    return rc ? rc : got;
}

// parts per chain: each part's socket I/O, staging and launches run on a host thread of its
// own (the syscalls of many small frames are what one thread cannot keep up with)
constexpr int kChainThreads = 8;

}  // namespace

struct APE_LZ4_chain {
    int nconn = 0, msg = 0, nparts = 0;
    // sticky per direction over the whole chain: the parts that did not fail advanced their
    // streams in the failed call, so no connection of it can resume either
    bool tx_failed = false, rx_failed = false;
    int first[kChainThreads + 1] = {};
    ChainPart *part[kChainThreads] = {};
};

namespace {

// run f(p) for every part, parts 1.. on threads of their own, part 0 on the caller's; the
// first error (in part order) or the sum of the results
template <typename F>
long long chain_parallel(APE_LZ4_chain *c, F f) {
    long long res[kChainThreads] = {};
    std::vector<std::thread> th;
    for (int p = 1; p < c->nparts; p++) th.emplace_back([&, p] { res[p] = f(p); });
    res[0] = f(0);
    for (auto &t : th) t.join();
    long long sum = 0;
    for (int p = 0; p < c->nparts; p++) {
        if (res[p] < 0) return res[p];
        sum += res[p];
    }
    return sum;
}

}  // namespace

extern "C" {

APE_LZ4_chain *APE_LZ4_chain_new(int nconn, int msg_len) {
    if (nconn <= 0 || msg_len <= 0 || msg_len > (1 << 24) || APE_LZ4_gpu_init() != 0) return nullptr;
    int dev = 0;
    (void)hipGetDevice(&dev);
    APE_LZ4_chain *c = new APE_LZ4_chain();
    c->nconn = nconn;
    c->msg = msg_len;
    int np = 4;
    if (const char *ev = getenv("APE_LZ4_CHAIN_THREADS")) np = atoi(ev);
    np = np < 1 ? 1 : (np > kChainThreads ? kChainThreads : np);
    c->nparts = np < nconn ? np : nconn;
    for (int p = 0; p <= c->nparts; p++) c->first[p] = (int)((long long)p * nconn / c->nparts);
    for (int p = 0; p < c->nparts; p++) {
        c->part[p] = part_new(c->first[p + 1] - c->first[p], msg_len, dev);
        if (!c->part[p]) {
            APE_LZ4_chain_free(c);
            return nullptr;
        }
    }
    return c;
}

void APE_LZ4_chain_free(APE_LZ4_chain *c) {
    if (!c) return;
    for (int p = 0; p < c->nparts; p++)
        if (c->part[p]) chain_release(c->part[p]);
    delete c;
}

// TX: nmsg messages per connection (message m of connection i at h_msgs + (m * nconn + i) *
// msg_stride) as the reference's frames on fds[i].  Returns the bytes written or an error code.
long long APE_LZ4_chain_send(APE_LZ4_chain *c, const int *fds, const char *h_msgs,
                             size_t msg_stride, int nmsg) {
    if (!c || !fds || !h_msgs || nmsg < 0 || msg_stride < (size_t)c->msg) return APE_LZ4_GPU_EINVAL;
    if (c->tx_failed) return APE_LZ4_GPU_EINVAL;
    const long long r = chain_parallel(c, [&](int p) {
        const int i0 = c->first[p];
        return part_send(c->part[p], fds + i0, h_msgs + (size_t)i0 * msg_stride, msg_stride,
                         (size_t)c->nconn * msg_stride, nmsg);
    });
    if (r < 0) c->tx_failed = true;
    return r;
}

// RX: nmsg messages per connection; message m of connection i is decoded into h_out + (m *
// nconn + i) * out_stride; h_status[i] as part_recv.  Returns the payload bytes or an error code.
long long APE_LZ4_chain_recv(APE_LZ4_chain *c, const int *fds, char *h_out, size_t out_stride,
                             int nmsg, int *h_status) {
    if (!c || !fds || !h_out || !h_status || nmsg < 0 || out_stride < (size_t)c->msg)
        return APE_LZ4_GPU_EINVAL;
    if (c->rx_failed) {
        for (int i = 0; i < c->nconn; i++) h_status[i] = -1;
        return APE_LZ4_GPU_EINVAL;
    }
    const long long r = chain_parallel(c, [&](int p) {
        const int i0 = c->first[p];
        return part_recv(c->part[p], fds + i0, h_out + (size_t)i0 * out_stride, out_stride,
                         (size_t)c->nconn * out_stride, nmsg, h_status + i0);
    });
    if (r < 0) c->rx_failed = true;
    return r;
}

}  // extern "C"

extern "C" {

// Time split of the socket calls since the last reset (see g_sock_ns): out[16] in ms
// (the two batch counts as counts).  reset != 0 zeroes the accumulators afterwards.
int APE_LZ4_socket_stats(double *out, int reset) {
    if (!out) return APE_LZ4_GPU_EINVAL;
    for (int i = 0; i < 16; i++) {
        const long long v = reset ? g_sock_ns[i].exchange(0) : g_sock_ns[i].load();
        out[i] = (i == 5 || i == 14) ? (double)v : (double)v * 1e-6;
    }
    return 0;
}

}  // extern "C"
