// lz4_destsize.hip -- N x APE_LZ4_compress_destSize (ref src/ape_lz4.c:843-1067) on the GPU.
//
// The reference runs a greedy parse that stops when the output reaches targetDstSize and
// reports how much input it consumed (*srcSizePtr).  Here a batch is encoded in two
// stream-ordered passes:
//   1. the regular encoder (lz4_encode.hip) compresses every block in full into a scratch
//      slot of compressBound bytes;
//   2. lz4_destsize_kernel (one wave per block) keeps the block whole when it fits the
//      target; otherwise it walks the scratch block's sequences and picks the cut that
//      consumes the most input: the first k whole sequences, then a final literal run
//      from the end of match k, as long as the target allows (`:1000-1021`).  A cut is
//      only legal when the block stays decodable with cap = consumed size: the last
//      match must end >= 5 bytes before the end (LASTLITERALS, `:1444-1447`) and start
//      >= 12 bytes before it (MFLIMIT, `:1346-1350`).
// The output is a valid LZ4 block of src[0, consumed) that fits the target (as the
// reference's); its bytes and the consumed size differ from the reference's, as for
// every GPU-compressed block (the parse is chunk-parallel).
#include "lz4_gpu_internal.h"

namespace apelz4 {
namespace {

constexpr uint32_t kWin = 2048;  // LDS window over the scratch block (bytes)

__device__ __forceinline__ uint32_t ext_len(uint32_t L) { return L >= 15u ? (L - 15u) / 255u + 1u : 0u; }

// Longest final literal run whose token + length bytes + literals fit `room` (>= 1) bytes,
// capped at `rem` (the input left).  The reference's fill rule (`:1002-1006`), exact.
__device__ __forceinline__ uint32_t max_lastrun(uint32_t room, uint32_t rem) {
    const uint32_t b = room - 1u;
    uint32_t L = b - (b + 240u) / 255u;
    while (L && L + ext_len(L) > b) L--;
    while (L + 1u + ext_len(L + 1u) <= b) L++;
    return L < rem ? L : rem;
}

__global__ void __launch_bounds__(64)
lz4_destsize_kernel(const char *const *src, int *src_size, char *const *dst, const int *target,
                    int *result, const char *scratch, size_t stride, const int *sres) {
    __shared__ uint4 win4[kWin / 16];
    const uint8_t *win = (const uint8_t *)win4;
    const int b = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    const int n = src_size[b];
    const int T = target[b];
    const uint8_t *in = (const uint8_t *)src[b];
    uint8_t *out = (uint8_t *)dst[b];
    const uint8_t *blk = (const uint8_t *)scratch + (size_t)b * stride;
    // the reference's early exits (`:866-872`, and compress_fast for large targets)
    if (T < 1 || n < 0) {
        if (lane == 0) result[b] = 0;
        return;
    }
    if (n > kMaxBlock) {
        if (lane == 0) result[b] = kErange;
        return;
    }
    const int c = sres[b];
    if (c > 0 && c <= T) {  // the whole block fits: keep it (as compress_fast at `:1034`)
        for (int i = (int)lane; i < c; i += 64) out[i] = blk[i];
        if (lane == 0) result[b] = c;
        return;
    }
    // Walk the sequences (every lane runs the same scalar walk; bytes come from an LDS
    // window over the scratch block, refilled by the whole wave).
    uint32_t w = 0x80000000u;  // window start (none yet: i - w >= kWin for every i)
    auto byte_at = [&](uint32_t i) -> uint32_t {
        if (i - w >= kWin) {  // wave-uniform: i and w are uniform
            w = i & ~15u;
            __syncthreads();
            for (uint32_t j = lane; j < kWin / 16; j += 64) {
                const size_t o = (size_t)w + 16u * j;
                win4[j] = o + 16u <= stride ? *(const uint4 *)(blk + o) : make_uint4(0, 0, 0, 0);
            }
            __syncthreads();
        }
        return (uint32_t)__builtin_amdgcn_readfirstlane(win[i - w]);
    };
    const uint32_t un = (uint32_t)n, uT = (uint32_t)T, uc = (uint32_t)(c > 0 ? c : 0);
    // k = 0: literals only
    uint32_t best_n = max_lastrun(uT, un), best_o = 0, best_a = 0;
    uint32_t op = 0, pos = 0;
    while (op < uc) {
        const uint32_t tok = byte_at(op++);
        uint32_t lit = tok >> 4;
        if (lit == 15u) {
            uint32_t s;
            do { s = byte_at(op++); lit += s; } while (s == 255u);
        }
        op += lit;
        pos += lit;
        if (op + 2u > uc) break;  // the final (literal-only) sequence
        op += 2u;                 // offset
        uint32_t ml = tok & 15u;
        if (ml == 15u) {
            uint32_t s;
            do { s = byte_at(op++); ml += s; } while (s == 255u);
        }
        ml += 4u;
        pos += ml;
        if (op + 1u > uT) break;  // no room left for the final token
        const uint32_t need = ml >= 7u ? 5u : 12u - ml;
        const uint32_t L = max_lastrun(uT - op, un - pos);
        if (L >= need && pos + L > best_n) {
            best_n = pos + L;
            best_o = op;
            best_a = pos;
        }
    }
    const uint32_t L = best_n - best_a;
    const uint32_t hdr = 1u + ext_len(L);
    for (uint32_t i = lane; i < best_o; i += 64) out[i] = blk[i];
    for (uint32_t i = lane; i < hdr; i += 64) {
        uint32_t v;
        if (i == 0) v = (L < 15u ? L : 15u) << 4;
        else if (i + 1 < hdr) v = 255u;
        else v = (L - 15u) % 255u;
        out[best_o + i] = (uint8_t)v;
    }
    for (uint32_t i = lane; i < L; i += 64) out[best_o + hdr + i] = in[best_a + i];
    if (lane == 0) {
        result[b] = (int)(best_o + hdr + L);
        src_size[b] = (int)best_n;
    }
}

}  // namespace

hipError_t launch_destsize(const char *const *src, int *src_size, char *const *dst,
                           const int *target, int *result, const char *scratch, size_t stride,
                           const int *sres, int n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(lz4_destsize_kernel, dim3(n), dim3(64), 0, s, src, src_size, dst, target,
                       result, scratch, stride, sres);
    return hipGetLastError();
}

}  // namespace apelz4
