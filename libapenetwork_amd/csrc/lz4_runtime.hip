// lz4_runtime.hip -- the thin C-ABI shim between the C host code and the HIP
// kernels: device checks, the batched launchers of include/ape_lz4_gpu.h, and
// the pinned-staging host path used by the one-shot ape_lz4.h calls.
//
// No CPU fallback anywhere: without a usable gfx950 device every entry point
// returns APE_LZ4_GPU_ENODEV (and the one-shot API reports failure).
#include <mutex>
#include <stdio.h>
#include <string.h>
#include <vector>

#include "../../include/ape_lz4_gpu.h"
#include "lz4_gpu_internal.h"
#include "lz4_gpu_shim.h"

using namespace apelz4;

namespace {

thread_local char g_err[256] = "";

void set_err(const char *what, hipError_t e) {
    snprintf(g_err, sizeof g_err, "%s: %s", what, e == hipSuccess ? "ok" : hipGetErrorString(e));
}

int g_ndev = -1;
std::vector<int> g_dev_ok;  // per device: 1 = gfx950
std::once_flag g_once;

void probe() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    g_ndev = n;
    g_dev_ok.assign(n > 0 ? n : 0, 0);
    for (int d = 0; d < n; d++) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, d) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0)
            g_dev_ok[d] = 1;
    }
}

int check_device() {
    std::call_once(g_once, probe);
    if (g_ndev <= 0) {
        snprintf(g_err, sizeof g_err, "no HIP device visible (libape_lz4_amd needs an MI355X)");
        return APE_LZ4_GPU_ENODEV;
    }
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= g_ndev || !g_dev_ok[d]) {
        snprintf(g_err, sizeof g_err, "current HIP device %d is not gfx950 (MI355X)", d);
        return APE_LZ4_GPU_ENODEV;
    }
    return APE_LZ4_GPU_OK;
}

int finish_launch(hipError_t e, const char *what) {
    if (e != hipSuccess) {
        set_err(what, e);
        return APE_LZ4_GPU_ELAUNCH;
    }
    return APE_LZ4_GPU_OK;
}

// ---- pinned staging for the host-buffer path: a process-wide pool ----
// A call borrows one context (stream + pinned + device staging) for its duration and
// returns it, so concurrent callers never share staging, and a thread that exits holds
// nothing (no thread-local HIP resources to leak).  Contexts whose staging grew past
// kKeepBytes are freed on return instead of pooled.
struct HostCtx {
    int dev = -1;
    hipStream_t stream = nullptr;
    char *h = nullptr;  // pinned
    size_t hcap = 0;
    char *d = nullptr;  // device
    size_t dcap = 0;
    void release() {
        if (h) (void)hipHostFree(h);
        if (d) (void)hipFree(d);
        if (stream) (void)hipStreamDestroy(stream);
        *this = HostCtx();
    }
};
constexpr size_t kKeepBytes = 64u << 20;
std::mutex g_pool_mu;
std::vector<HostCtx *> g_pool;   // idle contexts (any device)

HostCtx *ctx_acquire() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); i++) {
            if (g_pool[i]->dev == dev) {
                HostCtx *c = g_pool[i];
                g_pool.erase(g_pool.begin() + (long)i);
                return c;
            }
        }
    }
    HostCtx *c = new HostCtx();
    c->dev = dev;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        set_err("hipStreamCreate", e);
        delete c;
        return nullptr;
    }
    return c;
}

void ctx_return(HostCtx *c) {
    if (!c) return;
    if (c->hcap > kKeepBytes || c->dcap > kKeepBytes) {
        c->release();
        delete c;
        return;
    }
    std::lock_guard<std::mutex> g(g_pool_mu);
    g_pool.push_back(c);
}

int host_reserve(HostCtx &c, size_t bytes) {
    if (c.hcap < bytes) {
        if (c.h) (void)hipHostFree(c.h);
        c.h = nullptr;
        size_t cap = bytes < (1u << 20) ? (1u << 20) : bytes;
        hipError_t e = hipHostMalloc((void **)&c.h, cap, hipHostMallocDefault);
        if (e != hipSuccess) { c.hcap = 0; set_err("hipHostMalloc", e); return APE_LZ4_GPU_ENOMEM; }
        c.hcap = cap;
    }
    if (c.dcap < bytes) {
        if (c.d) (void)hipFree(c.d);
        c.d = nullptr;
        size_t cap = bytes < (1u << 20) ? (1u << 20) : bytes;
        hipError_t e = hipMalloc((void **)&c.d, cap);
        if (e != hipSuccess) { c.dcap = 0; set_err("hipMalloc", e); return APE_LZ4_GPU_ENOMEM; }
        c.dcap = cap;
    }
    return APE_LZ4_GPU_OK;
}

inline size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }

// Staging layout (same offsets on host and device):
//   [ptr arrays: src, dst][int arrays: in_size, cap, target, result][inputs][outputs]
// mode: 0 = compress, 1 = decompress_safe, 2 = decompress_safe_partial
int host_batch_run(HostCtx &ctx, int mode, int accel, const char *const *h_src, const int *h_in,
                   char *const *h_dst, const int *h_cap, const int *h_target, int *h_res, int nb,
                   const std::vector<size_t> &in_off, const std::vector<size_t> &out_off,
                   const std::vector<size_t> &out_len, size_t total);

int host_batch(int mode, int accel, const char *const *h_src, const int *h_in, char *const *h_dst,
               const int *h_cap, const int *h_target, int *h_res, int nb) {
    if (nb < 0 || (nb > 0 && (!h_src || !h_in || !h_dst || !h_cap || !h_res))) {
        snprintf(g_err, sizeof g_err, "invalid argument");
        return APE_LZ4_GPU_EINVAL;
    }
    int rc = check_device();
    if (rc) return rc;
    if (nb == 0) return APE_LZ4_GPU_OK;
    std::vector<size_t> in_off(nb), out_off(nb), out_len(nb);
    size_t meta = up16((size_t)nb * 2 * sizeof(void *)) + up16((size_t)nb * 4 * sizeof(int));
    size_t pos = meta;
    for (int i = 0; i < nb; i++) {
        in_off[i] = pos;
        size_t len = h_in[i] > 0 ? (size_t)h_in[i] : 1;  // size <= 0 still reads src[0]
        pos += up16(len);
    }
    for (int i = 0; i < nb; i++) {
        out_off[i] = pos;
        size_t lim;
        if (mode == 0) {
            int n = h_in[i] > 0 ? h_in[i] : 0;
            size_t bound = (size_t)n + n / 255 + 16;
            lim = h_cap[i] <= 0 ? 0 : ((size_t)h_cap[i] < bound ? (size_t)h_cap[i] : bound);
        } else {
            // the decoder writes only decoded bytes, and LZ4 expands at most 255x (a
            // 255 length byte per 255 output bytes): a huge cap needs no huge staging
            const size_t cs = h_in[i] > 0 ? (size_t)h_in[i] : 0;
            const size_t most = 255 * cs + 64;
            lim = h_cap[i] <= 0 ? 0 : ((size_t)h_cap[i] < most ? (size_t)h_cap[i] : most);
        }
        out_len[i] = lim;
        pos += up16(lim ? lim : 1);
    }
    const size_t total = pos;
    HostCtx *ctx = ctx_acquire();
    if (!ctx) return APE_LZ4_GPU_ENOMEM;
    rc = host_reserve(*ctx, total);
    if (rc) { ctx_return(ctx); return rc; }
    rc = host_batch_run(*ctx, mode, accel, h_src, h_in, h_dst, h_cap, h_target, h_res, nb,
                        in_off, out_off, out_len, total);
    // a failed run may have left copies or the kernel queued on the context's stream:
    // drain them before another caller can borrow its pinned buffer
    if (rc) (void)hipStreamSynchronize(ctx->stream);
    ctx_return(ctx);
    return rc;
}

int host_batch_run(HostCtx &ctx, int mode, int accel, const char *const *h_src, const int *h_in,
                   char *const *h_dst, const int *h_cap, const int *h_target, int *h_res, int nb,
                   const std::vector<size_t> &in_off, const std::vector<size_t> &out_off,
                   const std::vector<size_t> &out_len, size_t total) {
    char *H = ctx.h, *D = ctx.d;
    const char **hp_src = (const char **)H;
    char **hp_dst = (char **)(H + (size_t)nb * sizeof(void *));
    int *hi = (int *)(H + up16((size_t)nb * 2 * sizeof(void *)));
    int *h_size = hi, *h_capd = hi + nb, *h_tgt = hi + 2 * nb;
    const size_t ioff = up16((size_t)nb * 2 * sizeof(void *));
    for (int i = 0; i < nb; i++) {
        hp_src[i] = D + in_off[i];
        hp_dst[i] = D + out_off[i];
        h_size[i] = h_in[i];
        h_capd[i] = h_cap[i];
        h_tgt[i] = h_target ? h_target[i] : 0;
        if (h_in[i] > 0) memcpy(H + in_off[i], h_src[i], (size_t)h_in[i]);
        else H[in_off[i]] = h_src[i] ? h_src[i][0] : 0;
    }
    hipStream_t s = ctx.stream;
    hipError_t e = hipMemcpyAsync(D, H, out_off[0], hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return finish_launch(e, "hipMemcpyAsync H2D");
    BlockArgs a{};
    a.accel = accel;
    a.src = (const char *const *)D;
    a.dst = (char *const *)(D + (size_t)nb * sizeof(void *));
    a.src_size = (const int *)(D + ioff);
    a.dst_cap = (const int *)(D + ioff) + nb;
    a.target = (const int *)(D + ioff) + 2 * nb;
    a.result = (int *)(D + ioff) + 3 * nb;
    a.nblocks = nb;
    e = (mode == 0) ? launch_encode(a, s) : launch_decode(a, mode == 2, s);
    if (e != hipSuccess) return finish_launch(e, "kernel launch");
    e = hipMemcpyAsync(H + ioff + 3 * nb * sizeof(int), (const char *)a.result, nb * sizeof(int),
                       hipMemcpyDeviceToHost, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(H + out_off[0], D + out_off[0], total - out_off[0],
                           hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return finish_launch(e, "D2H / synchronize");
    const int *hres = (const int *)(H + ioff) + 3 * nb;
    for (int i = 0; i < nb; i++) {
        h_res[i] = hres[i];
        if (hres[i] > 0 && (size_t)hres[i] <= out_len[i]) memcpy(h_dst[i], H + out_off[i], hres[i]);
    }
    return APE_LZ4_GPU_OK;
}

BlockArgs ptr_args(const char *const *src, const int *in, char *const *dst, const int *cap,
                   const int *tgt, int *res, int nb) {
    BlockArgs a{};
    a.src = src;
    a.dst = dst;
    a.src_size = in;
    a.dst_cap = cap;
    a.target = tgt;
    a.result = res;
    a.nblocks = nb;
    return a;
}

}  // namespace

extern "C" {

int APE_LZ4_gpu_init(void) { return check_device(); }

int APE_LZ4_gpu_device_count(void) {
    std::call_once(g_once, probe);
    return g_ndev < 0 ? 0 : g_ndev;
}

const char *APE_LZ4_gpu_last_error(void) { return g_err; }
const char *APE_LZ4_gpu_arch(void) { return "gfx950"; }

int APE_LZ4_compress_batch_dev(const char *const *d_src, const int *d_srcSize,
                               char *const *d_dst, const int *d_dstCap, int *d_result,
                               int nblocks, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_srcSize || !d_dst || !d_dstCap || !d_result)))
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    return finish_launch(launch_encode(ptr_args(d_src, d_srcSize, d_dst, d_dstCap, nullptr,
                                                d_result, nblocks),
                                       (hipStream_t)stream),
                         "lz4_encode_kernel");
}

int APE_LZ4_compress_fast_batch_dev(const char *const *d_src, const int *d_srcSize,
                                    char *const *d_dst, const int *d_dstCap, int *d_result,
                                    int nblocks, int acceleration, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_srcSize || !d_dst || !d_dstCap || !d_result)))
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    BlockArgs a = ptr_args(d_src, d_srcSize, d_dst, d_dstCap, nullptr, d_result, nblocks);
    a.accel = acceleration;
    return finish_launch(launch_encode(a, (hipStream_t)stream), "lz4_encode_kernel");
}

int APE_LZ4_compress_exact_batch_dev(const char *const *d_src, const int *d_srcSize,
                                     char *const *d_dst, const int *d_dstCap, int *d_result,
                                     int nblocks, int acceleration, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_srcSize || !d_dst || !d_dstCap || !d_result)))
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    BlockArgs a = ptr_args(d_src, d_srcSize, d_dst, d_dstCap, nullptr, d_result, nblocks);
    a.accel = acceleration;
    return finish_launch(launch_encode_exact(a, (hipStream_t)stream), "lz4_encode_exact_kernel");
}

int APE_LZ4_decompress_safe_batch_dev(const char *const *d_src, const int *d_compressedSize,
                                      char *const *d_dst, const int *d_maxDecompressedSize,
                                      int *d_result, int nblocks, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_compressedSize || !d_dst ||
                                         !d_maxDecompressedSize || !d_result)))
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    return finish_launch(launch_decode(ptr_args(d_src, d_compressedSize, d_dst,
                                                d_maxDecompressedSize, nullptr, d_result, nblocks),
                                       false, (hipStream_t)stream),
                         "lz4_decode_kernel");
}

int APE_LZ4_decompress_safe_partial_batch_dev(const char *const *d_src,
                                              const int *d_compressedSize, char *const *d_dst,
                                              const int *d_targetOutputSize,
                                              const int *d_maxDecompressedSize, int *d_result,
                                              int nblocks, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_compressedSize || !d_dst ||
                                         !d_targetOutputSize || !d_maxDecompressedSize ||
                                         !d_result)))
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    return finish_launch(launch_decode(ptr_args(d_src, d_compressedSize, d_dst,
                                                d_maxDecompressedSize, d_targetOutputSize,
                                                d_result, nblocks),
                                       true, (hipStream_t)stream),
                         "lz4_decode_kernel<partial>");
}

int APE_LZ4_decompress_safe_usingDict_batch_dev(const char *const *d_src,
                                                const int *d_compressedSize, char *const *d_dst,
                                                const int *d_maxDecompressedSize,
                                                const char *const *d_dict, const int *d_dictSize,
                                                int *d_result, int nblocks, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_compressedSize || !d_dst ||
                                         !d_maxDecompressedSize || !d_dict || !d_dictSize ||
                                         !d_result)))
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    BlockArgs a = ptr_args(d_src, d_compressedSize, d_dst, d_maxDecompressedSize, nullptr,
                           d_result, nblocks);
    a.dict = d_dict;
    a.dict_size = d_dictSize;
    return finish_launch(launch_decode(a, false, (hipStream_t)stream),
                         "lz4_decode_kernel<usingDict>");
}

int APE_LZ4_decompress_fast_batch_dev(const char *const *d_src, const int *d_srcBound,
                                      char *const *d_dst, const int *d_originalSize,
                                      int *d_result, int nblocks, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_srcBound || !d_dst || !d_originalSize ||
                                         !d_result)))
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    BlockArgs a = ptr_args(d_src, d_srcBound, d_dst, d_originalSize, nullptr, d_result, nblocks);
    a.fast = 1;
    return finish_launch(launch_decode(a, false, (hipStream_t)stream), "lz4_decode_kernel<fast>");
}

int APE_LZ4_compress_withPrefix_batch_dev(const char *const *d_src, const int *d_srcSize,
                                          const int *d_prefixSize, char *const *d_dst,
                                          const int *d_dstCap, int *d_result, int nblocks,
                                          void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_srcSize || !d_prefixSize || !d_dst ||
                                         !d_dstCap || !d_result)))
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    BlockArgs a = ptr_args(d_src, d_srcSize, d_dst, d_dstCap, nullptr, d_result, nblocks);
    a.dict_size = d_prefixSize;
    return finish_launch(launch_encode(a, (hipStream_t)stream), "lz4_encode_kernel<prefix>");
}

namespace {

constexpr int kDsSub = 16384;   // destSize: blocks per scratch pass
inline size_t ds_stride() { return up16((size_t)kMaxBlock + kMaxBlock / 255 + 16); }
inline size_t ds_scratch(int sub) { return (size_t)sub * ds_stride() + (size_t)sub * sizeof(int); }

// encode into the scratch (full-size output, every block fits), then cut each block to
// its target; `sub` blocks per pass (the scratch holds ds_scratch(sub) bytes)
hipError_t destsize_passes(const char *const *d_src, int *d_srcSize, char *const *d_dst,
                           const int *d_targetDstSize, int *d_result, int nblocks, char *scr,
                           int sub, hipStream_t s) {
    const size_t stride = ds_stride();
    int *sres = (int *)(scr + (size_t)sub * stride);
    hipError_t e = hipSuccess;
    for (int off = 0; off < nblocks && e == hipSuccess; off += sub) {
        const int m = nblocks - off < sub ? nblocks - off : sub;
        BlockArgs a{};
        a.src = d_src + off;
        a.dst_base = scr;
        a.dst_stride = stride;  // cap = stride >= compressBound: every block fits
        a.src_size = d_srcSize + off;
        a.result = sres;
        a.nblocks = m;
        e = launch_encode(a, s);
        if (e == hipSuccess)
            e = launch_destsize(d_src + off, d_srcSize + off, d_dst + off, d_targetDstSize + off,
                                d_result + off, scr, stride, sres, m, s);
    }
    return e;
}

}  // namespace

size_t APE_LZ4_compress_destSize_scratch_size(int nblocks) {
    const int sub = nblocks < 1 ? 1 : (nblocks < kDsSub ? nblocks : kDsSub);
    return ds_scratch(sub);
}

int APE_LZ4_compress_destSize_batch_scratch_dev(const char *const *d_src, int *d_srcSize,
                                                char *const *d_dst, const int *d_targetDstSize,
                                                int *d_result, int nblocks, void *d_scratch,
                                                size_t scratch_bytes, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_srcSize || !d_dst || !d_targetDstSize ||
                                         !d_result || !d_scratch)))
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    if (nblocks == 0) return APE_LZ4_GPU_OK;
    // as many blocks per pass as the caller's scratch holds (at least one)
    int sub = (int)(scratch_bytes / (ds_stride() + sizeof(int)));
    if (sub < 1) {
        snprintf(g_err, sizeof g_err, "destSize scratch of %zu bytes < %zu (one block)",
                 scratch_bytes, ds_scratch(1));
        return APE_LZ4_GPU_EINVAL;
    }
    if (sub > nblocks) sub = nblocks;
    if ((uintptr_t)d_scratch & 15u) return APE_LZ4_GPU_EINVAL;
    return finish_launch(destsize_passes(d_src, d_srcSize, d_dst, d_targetDstSize, d_result,
                                         nblocks, (char *)d_scratch, sub, (hipStream_t)stream),
                         "lz4_encode_kernel + lz4_destsize_kernel");
}

int APE_LZ4_compress_destSize_batch_dev(const char *const *d_src, int *d_srcSize,
                                        char *const *d_dst, const int *d_targetDstSize,
                                        int *d_result, int nblocks, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_srcSize || !d_dst || !d_targetDstSize ||
                                         !d_result)))
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    if (nblocks == 0) return APE_LZ4_GPU_OK;
    // The one launcher that allocates: stream-ordered scratch (hipMallocAsync / hipFreeAsync
    // on the caller's stream, so concurrent calls never share it).  Under graph capture
    // use APE_LZ4_compress_destSize_batch_scratch_dev with caller-owned scratch.
    const int sub = nblocks < kDsSub ? nblocks : kDsSub;
    hipStream_t s = (hipStream_t)stream;
    char *scr = nullptr;
    hipError_t e = hipMallocAsync((void **)&scr, ds_scratch(sub), s);
    if (e != hipSuccess) {
        set_err("hipMallocAsync (destSize scratch)", e);
        return APE_LZ4_GPU_ENOMEM;
    }
    e = destsize_passes(d_src, d_srcSize, d_dst, d_targetDstSize, d_result, nblocks, scr, sub, s);
    hipError_t ef = hipFreeAsync(scr, s);
    if (e == hipSuccess) e = ef;
    return finish_launch(e, "lz4_encode_kernel + lz4_destsize_kernel");
}

int APE_LZ4_compress_batch_strided_dev(const char *d_src, size_t src_stride, const int *d_srcSize,
                                       char *d_dst, size_t dst_stride, const int *d_dstCap,
                                       int *d_result, int nblocks, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_srcSize || !d_dst || !d_result)))
        return APE_LZ4_GPU_EINVAL;
    if (!d_dstCap && dst_stride > 0x7FFFFFFF) return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    BlockArgs a{};
    a.src_base = d_src;
    a.dst_base = d_dst;
    a.src_stride = src_stride;
    a.dst_stride = dst_stride;
    a.src_size = d_srcSize;
    a.dst_cap = d_dstCap;
    a.result = d_result;
    a.nblocks = nblocks;
    return finish_launch(launch_encode(a, (hipStream_t)stream), "lz4_encode_kernel");
}

int APE_LZ4_decompress_safe_batch_strided_dev(const char *d_src, size_t src_stride,
                                              const int *d_compressedSize, char *d_dst,
                                              size_t dst_stride, const int *d_maxDecompressedSize,
                                              int *d_result, int nblocks, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_src || !d_compressedSize || !d_dst || !d_result)))
        return APE_LZ4_GPU_EINVAL;
    if (!d_maxDecompressedSize && dst_stride > 0x7FFFFFFF) return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    BlockArgs a{};
    a.src_base = d_src;
    a.dst_base = d_dst;
    a.src_stride = src_stride;
    a.dst_stride = dst_stride;
    a.src_size = d_compressedSize;
    a.dst_cap = d_maxDecompressedSize;
    a.result = d_result;
    a.nblocks = nblocks;
    return finish_launch(launch_decode(a, false, (hipStream_t)stream), "lz4_decode_kernel");
}

// ---- framed stream of independent blocks (lz4_frame.hip) ----
size_t APE_LZ4_frame_scratch_size(int nblocks) {
    return nblocks < 0 ? 0 : (size_t)frame_scratch_elems(nblocks) * sizeof(long long);
}

int APE_LZ4_frame_offsets_dev(const int *d_compressedSize, long long *d_off,
                              void *d_scratch, int nblocks, void *stream) {
    if (nblocks < 0 || !d_compressedSize || !d_off || !d_scratch) return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    return finish_launch(launch_frame_offsets(d_compressedSize, d_off, (long long *)d_scratch,
                                              nblocks, (hipStream_t)stream),
                         "frame offsets");
}

int APE_LZ4_frame_pack_strided_dev(const char *d_comp, size_t comp_stride,
                                   const int *d_compressedSize, const long long *d_off,
                                   char *d_frames, int nblocks, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_comp || !d_compressedSize || !d_off || !d_frames)))
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    return finish_launch(launch_frame_pack(d_comp, comp_stride, d_compressedSize, d_off,
                                           d_frames, nblocks, (hipStream_t)stream),
                         "frame pack");
}

int APE_LZ4_decompress_safe_frames_dev(const char *d_frames, const long long *d_off,
                                       char *d_dst, size_t dst_stride,
                                       const int *d_maxDecompressedSize, int *d_result,
                                       int nblocks, void *stream) {
    if (nblocks < 0 || (nblocks > 0 && (!d_frames || !d_off || !d_dst || !d_result)))
        return APE_LZ4_GPU_EINVAL;
    if (!d_maxDecompressedSize && dst_stride > 0x7FFFFFFF) return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    BlockArgs a{};
    a.src_base = d_frames;
    a.frame_off = d_off;
    a.dst_base = d_dst;
    a.dst_stride = dst_stride;
    a.dst_cap = d_maxDecompressedSize;
    a.result = d_result;
    a.nblocks = nblocks;
    return finish_launch(launch_decode(a, false, (hipStream_t)stream), "lz4_decode_kernel");
}

int APE_LZ4_compress_batch_host(const char *const *h_src, const int *h_srcSize,
                                char *const *h_dst, const int *h_dstCap, int *h_result,
                                int nblocks) {
    return host_batch(0, 1, h_src, h_srcSize, h_dst, h_dstCap, nullptr, h_result, nblocks);
}

int APE_LZ4_decompress_safe_batch_host(const char *const *h_src, const int *h_compressedSize,
                                       char *const *h_dst, const int *h_maxDecompressedSize,
                                       int *h_result, int nblocks) {
    return host_batch(1, 1, h_src, h_compressedSize, h_dst, h_maxDecompressedSize, nullptr,
                      h_result, nblocks);
}

int APE_LZ4_synth_blocks_dev(char *d_out, size_t stride, int blockSize, long long first_block,
                             int nblocks, int kind, void *stream) {
    if (nblocks < 0 || blockSize < 0 || blockSize > kMaxBlock || (nblocks > 0 && !d_out) ||
        stride < (size_t)blockSize)
        return APE_LZ4_GPU_EINVAL;
    int rc = check_device();
    if (rc) return rc;
    return finish_launch(launch_synth(d_out, stride, blockSize, first_block, nblocks, kind,
                                      (hipStream_t)stream),
                         "lz4_synth_kernel");
}

#ifdef APE_LZ4_STATS
}  // extern "C"
namespace apelz4 {
hipError_t dec_stats_read(unsigned long long *out, int reset);
hipError_t enc_stats_read(unsigned long long *out, int reset);
}
extern "C" {
// Diagnostic build only: per-phase cycle sums (which: 0 = decode, 1 = encode).
int APE_LZ4_debug_stats(int which, unsigned long long *out16, int reset) {
    hipError_t e = which ? apelz4::enc_stats_read(out16, reset) : apelz4::dec_stats_read(out16, reset);
    return e == hipSuccess ? 0 : -1;
}
#endif

// ---- internal shim for the one-shot C API (ape_lz4_api.c) ----
int ape_lz4_gpu_compress_one(const char *src, char *dst, int n, int cap, int accel, int *rt) {
    int res = 0;
    *rt = host_batch(0, accel, &src, &n, &dst, &cap, nullptr, &res, 1);
    return res;
}

int ape_lz4_gpu_decompress_one(const char *src, char *dst, int csize, int cap, int partial,
                               int target, int *rt) {
    int res = 0;
    *rt = host_batch(partial ? 2 : 1, 1, &src, &csize, &dst, &cap, partial ? &target : nullptr,
                     &res, 1);
    return res;
}

}  // extern "C"
