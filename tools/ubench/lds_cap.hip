// lds_cap.hip -- DIAGNOSTIC: the device's LDS limits, and whether a 1024-thread workgroup
// with ~156 KiB of static LDS keeps every byte (plain writes/reads, u16 writes, and
// ds_add_rtn atomics on packed u16 counters above and below 64 KiB).
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int kWords = 159940 / 4;
__global__ void __launch_bounds__(1024) ldsk(unsigned *bad) {
    __shared__ unsigned L[kWords];
    for (int i = threadIdx.x; i < kWords; i += 1024) L[i] = i * 2654435761u + blockIdx.x;
    __syncthreads();
    unsigned b = 0;
    for (int i = threadIdx.x; i < kWords; i += 1024) b += L[(i * 7 + 13) % kWords] != ((i * 7 + 13) % kWords) * 2654435761u + blockIdx.x;
    if (b) atomicAdd(&bad[0], b);
    __syncthreads();
    // atomics: counters at word offsets 1000 (below 64 KiB) and 30000 (above), packed halves
    const int base[2] = {1000, 30000};
    for (int k = 0; k < 2; k++) {
        for (int i = threadIdx.x; i < 512; i += 1024) L[base[k] + i] = 0;
        __syncthreads();
        const unsigned h = (threadIdx.x * 37u) & 1023u;
        const unsigned old = atomicAdd(&L[base[k] + (h >> 1)], (h & 1) ? 0x10000u : 1u);
        (void)old;
        __syncthreads();
        // every counter half must now equal the number of threads with that h (= 1 each)
        if (threadIdx.x < 1024) {
            const unsigned v = (L[base[k] + (threadIdx.x >> 1)] >> ((threadIdx.x & 1) * 16)) & 0xFFFFu;
            if (v != 1u) atomicAdd(&bad[1 + k], 1u);
        }
        __syncthreads();
        // u16 stores
        ((unsigned short *)&L[base[k]])[threadIdx.x] = (unsigned short)(threadIdx.x * 3);
        __syncthreads();
        if (((unsigned short *)&L[base[k]])[threadIdx.x ^ 5] != (unsigned short)((threadIdx.x ^ 5) * 3)) atomicAdd(&bad[3 + k], 1u);
        __syncthreads();
    }
}
int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("sharedMemPerBlock %zu maxSharedMemoryPerMultiProcessor %zu\n", p.sharedMemPerBlock,
           p.maxSharedMemoryPerMultiProcessor);
    unsigned *d; hipMalloc(&d, 64); hipMemset(d, 0, 64);
    hipLaunchKernelGGL(ldsk, dim3(4096), dim3(1024), 0, 0, d);
    hipError_t e = hipDeviceSynchronize();
    unsigned h[5] = {0}; hipMemcpy(h, d, 20, hipMemcpyDeviceToHost);
    printf("launch %s, mismatches plain %u, atomics <64K %u >64K %u, u16 <64K %u >64K %u\n", hipGetErrorString(e), h[0], h[1], h[2], h[3], h[4]);
    return 0;
}
