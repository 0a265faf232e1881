// gather_rate.hip -- DIAGNOSTIC microbenchmark (not product): throughput of per-lane
// gathers on gfx950 by access shape, from an L2-resident buffer, to price the encoder's
// candidate loads (each lane reads 16 bytes at its own position).  Every wave issues
// `iters` independent loads of one shape (8 in flight), 32 waves per CU on every CU; prints
// CU cycles per wave-instruction for each shape:
//   coal16   16 B per lane, the wave's 1 KiB contiguous
//   quad16   16 B per lane, 16 groups of 4 lanes, each group 64 contiguous bytes (stage 2)
//   scat16   16 B per lane, 64 different 128-B lines (the T-candidate gather)
//   scat8    8 B per lane, 64 different lines
//   scat4    4 B per lane, 64 different lines
//   half16   16 B per lane, 32 lines (lanes in pairs)
//   scat16u  as scat16 at a random byte offset (unaligned, may cross a line): the T candidate
//   quad16u  as quad16 from an unaligned group base: the stage-2 windows
//   byte8u   8 B per lane at base + lane (byte stride, overlapping): the own-bytes load
//   coal16u  as coal16 shifted by one byte
//   hipcc -O3 --offload-arch=gfx950 -o gather_rate gather_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32;

template <int KIND>
__global__ void __launch_bounds__(256) gath(const unsigned char *buf, u32 mask, int iters, u32 *sink) {
    const u32 lane = threadIdx.x & 63u, w = (blockIdx.x * 4u + (threadIdx.x >> 6));
    u32 acc = 0, s = w * 0x9E3779B9u + lane * 0x85EBCA6Bu;
    for (int it = 0; it < iters; it += 8) {
        u32 a[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            s = s * 1664525u + 1013904223u;
            const u32 wb = (w * 977u + (u32)(it + u) * 4099u) * 1024u;   // per-wave base
            u32 off;
            if (KIND == 0) off = wb + lane * 16u;
            else if (KIND == 1) off = (s & ~63u) + (lane & 3u) * 16u;   // lane groups of 4
            else if (KIND == 5) off = (s & ~127u) * 1u + (lane & 1u) * 16u;
            else if (KIND == 6) off = s & ~0u;                           // any byte
            else if (KIND == 7) off = s;                                 // group base below
            else if (KIND == 8) off = wb + 3u + lane;                    // byte stride
            else if (KIND == 9) off = wb + 1u + lane * 16u;
            else off = (s & ~127u) + (lane * 36u & 112u);
            a[u] = off & mask;
        }
        if (KIND == 1) {   // groups of 4 share the base of their first lane
#pragma unroll
            for (int u = 0; u < 8; u++) a[u] = __shfl(a[u], lane & ~3u) + (lane & 3u) * 16u;
        }
        if (KIND == 5) {
#pragma unroll
            for (int u = 0; u < 8; u++) a[u] = __shfl(a[u], lane & ~1u) + (lane & 1u) * 16u;
        }
        if (KIND == 7) {
#pragma unroll
            for (int u = 0; u < 8; u++) a[u] = __shfl(a[u], lane & ~3u) + (lane & 3u) * 16u;
        }
        typedef u32 u32x4u __attribute__((ext_vector_type(4), aligned(1)));
        typedef u32 u32x2u __attribute__((ext_vector_type(2), aligned(1)));
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if (KIND == 3) acc ^= ((const uint2 *)(buf + (a[u] & ~7u)))->x;
            else if (KIND == 4) acc ^= *(const u32 *)(buf + (a[u] & ~3u));
            else if (KIND == 8) {
                const u32x2u v = *(const u32x2u *)(buf + (a[u] & (mask >> 1)));
                acc ^= v.x ^ v.y;
            } else if (KIND >= 6) {
                const u32x4u v = *(const u32x4u *)(buf + (a[u] & (mask >> 1)));
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            } else {
                const uint4 v = *(const uint4 *)(buf + (a[u] & ~15u));
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int KIND>
float run(const unsigned char *buf, u32 mask, int iters, u32 *sink, int blocks) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(gath<KIND>, dim3(blocks), dim3(256), 0, 0, buf, mask, iters, sink);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(gath<KIND>, dim3(blocks), dim3(256), 0, 0, buf, mask, iters, sink);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    unsigned char *buf;
    u32 *sink;
    const size_t bytes = 4u << 20;   // L2-resident (each XCD caches what it reads)
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount, blocks = cus * 8;   // 8 x 4 waves = 32 waves per CU
    const int iters = 2048;
    const double clk = 2.4e9;   // nominal; the ratios between shapes are what matter
    const char *names[10] = {"coal16", "quad16", "scat16", "scat8", "scat4", "half16", "scat16u",
                             "quad16u", "byte8u", "coal16u"};
    float ms[10];
    ms[0] = run<0>(buf, bytes - 1, iters, sink, blocks);
    ms[1] = run<1>(buf, bytes - 1, iters, sink, blocks);
    ms[2] = run<2>(buf, bytes - 1, iters, sink, blocks);
    ms[3] = run<3>(buf, bytes - 1, iters, sink, blocks);
    ms[4] = run<4>(buf, bytes - 1, iters, sink, blocks);
    ms[5] = run<5>(buf, bytes - 1, iters, sink, blocks);
    ms[6] = run<6>(buf, bytes - 1, iters, sink, blocks);
    ms[7] = run<7>(buf, bytes - 1, iters, sink, blocks);
    ms[8] = run<8>(buf, bytes - 1, iters, sink, blocks);
    ms[9] = run<9>(buf, bytes - 1, iters, sink, blocks);
    printf("{\"cus\": %d, \"waves_per_cu\": 32, \"loads_per_wave\": %d", cus, iters);
    for (int k = 0; k < 10; k++) {
        const double per_cu = (double)iters * 32.0;   // wave-instructions per CU
        printf(", \"%s\": {\"ms\": %.3f, \"cu_cycles_per_wave_instr\": %.2f}", names[k], ms[k],
               ms[k] * 1e-3 * clk / per_cu);
    }
    printf("}\n");
    return 0;
}
