// fetch_calib.hip -- DIAGNOSTIC microbenchmark (not product): what rocprofv3's FETCH_SIZE
// reports for access shapes of known byte counts on gfx950.
//
// MI355X_MICROARCH.md calibrates FETCH_SIZE for one shape only (16 B/lane coalesced streaming
// reads: it reports half the bytes).  The encoder's fetch is dominated by scattered per-lane
// gathers of 16-20 bytes (candidate bytes in[T-4, T+12) and stage-2 windows), so the factor
// is measured here for that shape.  Every kernel reads a 4 GiB buffer (far beyond the 256 MiB
// Infinity Cache and the L2s) and touches every line it reads exactly once, so the bytes that
// must cross the L2's memory side are known from the access list alone:
//   stream16   16 B per lane, coalesced, the whole buffer          -> bytes = buffer
//   gather16   16 B per lane in a distinct 128-B line (16-B aligned inside it)
//                                                                  -> 128 B lines: nlines
//   gather20   16 + 4 B per lane at an unaligned offset in a distinct 128-B line, as the
//              encoder's candidate load (a dwordx4 + a dword)      -> same lines
//   gather16h  16 B per lane in a distinct 64-B half line (both halves of every line read,
//              by lanes of different waves far apart in time)     -> 64 B halves: 2 nlines
// The line order is a bijective scramble, so consecutive lanes hit lines far apart (no
// coalescing, as the encoder's random candidates).
//   hipcc -O3 --offload-arch=gfx950 -o fetch_calib fetch_calib.hip
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -d out -o run --output-format csv -- ./fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32;
typedef unsigned long long u64;

__device__ __forceinline__ u64 scramble(u64 i, u64 mask) {   // bijection on [0, mask]
    i = (i * 0x9E3779B97F4A7C15ull) & mask;
    i ^= i >> 7;
    i = (i * 0xC2B2AE3D27D4EB4Full) & mask;
    return i;
}

__global__ void __launch_bounds__(256) stream16(const uint4 *in, u64 n16, u32 *sink) {
    u32 acc = 0;
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (u64)gridDim.x * 256ull) {
        const uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;   // keeps the loads alive
}

template <int KIND>
__global__ void __launch_bounds__(256) gather(const unsigned char *in, u64 nacc, u64 mask,
                                              u32 *sink) {
    const u64 i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= nacc) return;
    const u64 slot = scramble(i, mask);
    u32 acc;
    if (KIND == 0) {   // 16 B at a 16-B offset of a distinct 128-B line
        const u64 a = slot * 128ull + ((i * 5ull) & 7ull) * 16ull;
        const uint4 v = *(const uint4 *)(in + a);
        acc = v.x ^ v.y ^ v.z ^ v.w;
    } else if (KIND == 1) {   // 16 + 4 B at an unaligned offset inside a distinct 128-B line
        const u64 a = slot * 128ull + ((i * 37ull) % 108ull);
        typedef u32 u32x4u __attribute__((ext_vector_type(4), aligned(1)));
        typedef u32 u32u __attribute__((aligned(1)));
        const u32x4u v = *(const u32x4u *)(in + a);
        const u32 w = *(const u32u *)(in + a + 16);
        acc = v.x ^ v.y ^ v.z ^ v.w ^ w;
    } else {   // 16 B in a distinct 64-B half line
        const u64 a = slot * 64ull + ((i * 3ull) & 3ull) * 16ull;
        const uint4 v = *(const uint4 *)(in + a);
        acc = v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[1] = acc;
}

int main() {
    const u64 bytes = 4ull << 30;
    unsigned char *buf = nullptr;
    u32 *sink = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    if (hipMemset(buf, 0x5A, bytes) != hipSuccess) return 1;
    // stream16 first (the guide's calibrated shape), then the gathers in scrambled line order:
    // at most the last 256 MiB streamed can still sit in the Infinity Cache (~6 % of the lines)
    const u64 nl = bytes / 128ull, nh = bytes / 64ull;
    hipLaunchKernelGGL(stream16, dim3(4096), dim3(256), 0, 0, (const uint4 *)buf, bytes / 16ull, sink);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    hipLaunchKernelGGL(gather<0>, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, 0, buf, nl, nl - 1, sink);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    hipLaunchKernelGGL(gather<1>, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, 0, buf, nl, nl - 1, sink);
    if (hipDeviceSynchronize() != hipSuccess) return 4;
    hipLaunchKernelGGL(gather<2>, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, 0, buf, nh, nh - 1, sink);
    if (hipDeviceSynchronize() != hipSuccess) return 5;
    // the known byte counts, one JSON line (the profile's FETCH_SIZE rows are in launch order)
    printf("{\"buffer_bytes\": %llu, \"stream16\": {\"accesses\": %llu, \"bytes\": %llu}, "
           "\"gather16\": {\"accesses\": %llu, \"lines128\": %llu, \"useful_bytes\": %llu}, "
           "\"gather20\": {\"accesses\": %llu, \"lines128\": %llu, \"useful_bytes\": %llu}, "
           "\"gather16h\": {\"accesses\": %llu, \"halves64\": %llu, \"useful_bytes\": %llu}}\n",
           bytes, bytes / 16ull, bytes, nl, nl, nl * 16ull, nl, nl, nl * 20ull, nh, nh, nh * 16ull);
    (void)hipFree(buf);
    (void)hipFree(sink);
    return 0;
}
