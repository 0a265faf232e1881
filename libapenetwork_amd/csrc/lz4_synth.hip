// lz4_synth.hip -- device generator for the benchmark blocks of SURVEY.md
// Appendix C (identical bytes to oracle/synth.c; tests check that).
// One 64-thread workgroup per block: lane 0 runs the sequential generator into
// LDS (copies may overlap, so it is inherently serial within a block), then
// the wave writes the block to HBM with 16-byte stores.  Untimed setup only.
#include "lz4_gpu_internal.h"

namespace apelz4 {

namespace {
__device__ __forceinline__ uint64_t xs(uint64_t &s) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}
}  // namespace

__global__ void __launch_bounds__(64)
lz4_synth_kernel(char *out, size_t stride, int n, long long first, int kind) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[kMaxBlock + 16];
    const long long blk = first + blockIdx.x;
    uint8_t *dst = (uint8_t *)out + (size_t)blockIdx.x * stride;
    if (threadIdx.x == 0) {
        uint64_t s = (uint64_t)blk * 0x9E3779B97F4A7C15ULL + 1ULL;
        int i = 0;
        if (kind == 0) {
            while (i < n) {
                uint64_t w = xs(s);
                for (int k = 0; k < 8 && i < n; k++, i++) buf[i] = (uint8_t)(w >> (8 * k));
            }
        } else {
            while (i < n) {
                uint64_t r = xs(s);
                if (i >= 64 && (r & 3) != 0) {
                    int len = 4 + (int)((r >> 32) % 60);
                    int win = i < 65535 ? i : 65535;
                    int off = 1 + (int)((r >> 8) % (uint64_t)win);
                    int e = i + len < n ? i + len : n;
                    for (; i < e; i++) buf[i] = buf[i - off];
                } else {
                    int len = 1 + (int)((r >> 8) % 16);
                    int e = i + len < n ? i + len : n;
                    for (; i < e; i++) buf[i] = (uint8_t)('a' + (xs(s) & 15));
                }
            }
        }
    }
    __syncthreads();
    if ((((uintptr_t)dst) & 15) == 0) {
        int n16 = n & ~15;
        for (int k = 16 * threadIdx.x; k < n16; k += 16 * 64)
            *(uint4 *)(dst + k) = *(const uint4 *)(buf + k);
        for (int k = n16 + threadIdx.x; k < n; k += 64) dst[k] = buf[k];
    } else {
        for (int k = threadIdx.x; k < n; k += 64) dst[k] = buf[k];
    }
}

hipError_t launch_synth(char *out, size_t stride, int n, long long first, int nblocks, int kind,
                        hipStream_t s) {
    if (nblocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(lz4_synth_kernel, dim3(nblocks), dim3(64), 0, s, out, stride, n, first,
                       kind);
    return hipGetLastError();
}

}  // namespace apelz4
