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

// Global-address-space byte pointers: global_load/store with an SGPR base and a
// 32-bit offset instead of flat accesses (which also tie up lgkmcnt).
typedef __attribute__((address_space(1))) const uint8_t gcu8;
typedef __attribute__((address_space(1))) uint8_t gu8;
typedef uint32_t u32x4_u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32x2_u __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));

// unaligned 16 / 8 / 4-byte global accesses (the hardware handles any alignment)
__device__ __forceinline__ uint4 gload16(gcu8 *p) {
    const u32x4_u v = *(__attribute__((address_space(1))) const u32x4_u *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
typedef uint32_t u32x3_u __attribute__((ext_vector_type(3), aligned(1)));
__device__ __forceinline__ uint3 gload12(gcu8 *p) {
    const u32x3_u v = *(__attribute__((address_space(1))) const u32x3_u *)p;
    return make_uint3(v.x, v.y, v.z);
}
__device__ __forceinline__ uint2 gload8(gcu8 *p) {
    const u32x2_u v = *(__attribute__((address_space(1))) const u32x2_u *)p;
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint32_t gload4(gcu8 *p) {
    return *(__attribute__((address_space(1))) const u32_u *)p;
}
__device__ __forceinline__ void gstore16(gu8 *p, uint4 v) {
    u32x4_u w;
    w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
    *(__attribute__((address_space(1))) u32x4_u *)p = w;
}
__device__ __forceinline__ void gstore4(gu8 *p, uint32_t v) {
    *(__attribute__((address_space(1))) u32_u *)p = v;
}

// ---- wave64 helpers ----
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

// Wave votes on a bool: HIP's __ballot / __any take an int, and the int round trip
// costs a v_cndmask + v_cmp per vote where the condition already is a lane mask.
__device__ __forceinline__ uint64_t wave_ballot(bool c) { return __builtin_amdgcn_ballot_w64(c); }
__device__ __forceinline__ bool wave_any(bool c) { return __builtin_amdgcn_ballot_w64(c) != 0; }
// This lane's bit of a wave-uniform mask as a lane predicate: the mask itself becomes the
// condition register (no shift / and / 64-bit compare per lane).
__device__ __forceinline__ bool lane_in(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

// DPP lane moves (GFX9-family controls, available on gfx950): lanes whose
// source is outside the row / masked off keep `old`.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROW_MASK, 0xF, false);
}
// ... with every row and bank enabled and bound_ctrl set: a lane whose source is outside
// reads 0, and no `old` register is needed (no v_mov 0 before the move)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_z(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
constexpr int kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114,
              kDppRowShr8 = 0x118, kDppBcast15 = 0x142, kDppBcast31 = 0x143,
              kDppWaveShr1 = 0x138, kDppWaveShl1 = 0x130;

// Inclusive scans over the 64 lanes (Hillis-Steele inside 16-lane rows, then
// row broadcasts) -- VALU latency instead of LDS-crossbar shuffles.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += dpp<kDppRowShr1>(0u, x);
    x += dpp<kDppRowShr2>(0u, x);
    x += dpp<kDppRowShr4>(0u, x);
    x += dpp<kDppRowShr8>(0u, x);
    x += dpp<kDppBcast15, 0xA>(0u, x);
    x += dpp<kDppBcast31, 0xC>(0u, x);
    return x;
}

__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    x = umax(x, dpp<kDppRowShr1>(0u, x));
    x = umax(x, dpp<kDppRowShr2>(0u, x));
    x = umax(x, dpp<kDppRowShr4>(0u, x));
    x = umax(x, dpp<kDppRowShr8>(0u, x));
    x = umax(x, dpp<kDppBcast15, 0xA>(0u, x));
    x = umax(x, dpp<kDppBcast31, 0xC>(0u, x));
    return x;
}

// value of the previous lane (lane 0 gets `first`)
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x, uint32_t first) {
    return dpp<kDppWaveShr1>(first, x);
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v) {
    return wave_shr1(wave_incl_sum(v), 0u);
}

__device__ __forceinline__ uint32_t lane_val(uint32_t v, int l) {  // l wave-uniform
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// ---- diagnostic phase timers (built only into libape_lz4_amd_stats.so) ----
// Thread 0 of every workgroup accumulates s_memtime cycles per phase and adds them
// to a per-kernel __device__ array at exit.  Never compiled into the product.
#ifdef APE_LZ4_STATS
#define STATS_DECL uint64_t st_t_ = clock64(); uint64_t st_acc_[16] = {0};
#define STAT(i) do { uint64_t t_ = clock64(); st_acc_[i] += t_ - st_t_; st_t_ = t_; } while (0)
#define STAT_ADD(i, v) (st_acc_[i] += (uint64_t)(v))
#define STATS_FLUSH(arr) STATS_FLUSH_TID(arr, 0)
#define STATS_FLUSH_TID(arr, t) do { if (threadIdx.x == (t)) { _Pragma("unroll") for (int i_ = 0; i_ < 16; i_++) if (st_acc_[i_]) atomicAdd(&(arr)[i_], (unsigned long long)st_acc_[i_]); } } while (0)
#else
#define STATS_DECL
#define STAT(i) do {} while (0)
#define STAT_ADD(i, v) do {} while (0)
#define STATS_FLUSH(arr) do {} while (0)
#define STATS_FLUSH_TID(arr, t) do {} while (0)
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
    const long long *frame_off;  // decoder: blocks read from a framed stream at src_base
                                 // (frame i = [le32 size][block] at src_base + frame_off[i])
    const char *const *dict;  // decoder: per-block external dictionary (nullable) ...
    const int *dict_size;     // ... and its size (usingDict, ref src/ape_lz4.c:1625-1647)
    int fast;                 // decoder: decompress_fast (src_size = readable bound of src)
    int accel;                // encoder: acceleration (compress_fast, :789); > 1 drops the
                              // in-chunk candidate (faster, lower ratio)
    int *result;
    int nblocks;
};

hipError_t launch_decode(const BlockArgs &a, bool partial, hipStream_t s);
// usingDict decodes of nq chunk positions x nconn connections (block q * nconn + i), one
// workgroup per connection looping over its chunks in order (lz4_decode.hip)
hipError_t launch_decode_chain(const BlockArgs &a, int nconn, int nq, hipStream_t s);
hipError_t launch_encode(const BlockArgs &a, hipStream_t s);
// the greedy-exact mode (lz4_encode_exact.hip): the reference's sequential parse, byte for byte
hipError_t launch_encode_exact(const BlockArgs &a, hipStream_t s);
// compress_destSize pass 2 (lz4_destsize.hip): scratch slot i (at scratch + i*stride, encoder
// result sres[i]) -> dst[i] cut to target[i]; src_size[i] <- consumed input
hipError_t launch_destsize(const char *const *src, int *src_size, char *const *dst,
                           const int *target, int *result, const char *scratch, size_t stride,
                           const int *sres, int n, hipStream_t s);
hipError_t launch_frame_offsets(const int *csize, long long *off, long long *scratch, int n,
                                hipStream_t s);
int frame_scratch_elems(int n);
hipError_t launch_frame_pack(const char *comp, size_t stride, const int *csize,
                             const long long *off, char *frames, int n, hipStream_t s);
hipError_t launch_synth(char *out, size_t stride, int n, long long first, int nblocks,
                        int kind, hipStream_t s);

}  // namespace apelz4
