// lz4_gpu_internal.h -- shared device helpers and launcher prototypes for the
// MI355X LZ4 kernels (gfx950 / CDNA4, wave64).  Internal to libape_lz4_amd.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace apelz4 {

// Format constants of LZ4 v1.7.1 (ref src/ape_lz4.c:237-254).
constexpr int kMinMatch = 4;
constexpr int kLastLiterals = 5;
constexpr int kMFLimit = 12;
constexpr int kMinLength = 13;
constexpr int kMaxBlock = 65536;  // GPU block limit (LZ4 window, benchmark block)
constexpr int kErange = -2147483647 - 1;

// ---- wave64 helpers ----
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

// Exclusive prefix sum over the 64 lanes of a wave.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v) {
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane_id() >= d) x += y;
    }
    return x - v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// ---- diagnostic phase timers (built only into libape_lz4_amd_stats.so) ----
// Thread 0 of every workgroup accumulates s_memtime cycles per phase and adds them
// to a per-kernel __device__ array at exit.  Never compiled into the product.
#ifdef APE_LZ4_STATS
#define STATS_DECL uint64_t st_t_ = clock64(); uint64_t st_acc_[16] = {0};
#define STAT(i) do { uint64_t t_ = clock64(); st_acc_[i] += t_ - st_t_; st_t_ = t_; } while (0)
#define STAT_ADD(i, v) (st_acc_[i] += (uint64_t)(v))
#define STATS_FLUSH(arr) do { if (threadIdx.x == 0) { _Pragma("unroll") for (int i_ = 0; i_ < 16; i_++) atomicAdd(&(arr)[i_], (unsigned long long)st_acc_[i_]); } } while (0)
#else
#define STATS_DECL
#define STAT(i) do {} while (0)
#define STAT_ADD(i, v) do {} while (0)
#define STATS_FLUSH(arr) do {} while (0)
#endif
hipError_t stats_read(int which, unsigned long long *out, int reset);

// Launchers (lz4_decode.hip / lz4_encode.hip / lz4_synth.hip).
struct BlockArgs {
    const char *const *src;   // pointer-array form (nullptr when strided)
    char *const *dst;
    const char *src_base;     // strided form
    char *dst_base;
    size_t src_stride, dst_stride;
    const int *src_size;      // per-block input size
    const int *dst_cap;       // per-block capacity (nullable -> default)
    const int *target;        // partial decode target (nullable)
    int *result;
    int nblocks;
};

hipError_t launch_decode(const BlockArgs &a, bool partial, hipStream_t s);
hipError_t launch_encode(const BlockArgs &a, hipStream_t s);
hipError_t launch_synth(char *out, size_t stride, int n, long long first, int nblocks,
                        int kind, hipStream_t s);

}  // namespace apelz4
