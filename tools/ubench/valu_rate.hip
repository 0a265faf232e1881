// valu_rate.hip -- DIAGNOSTIC microbenchmark (not product): wave64 integer VALU issue
// rate per SIMD on gfx950 as a function of waves per SIMD, to tell whether a kernel
// at "1 VALU per quad-cycle per SIMD" is issue-bound.
//   hipcc -O3 --offload-arch=gfx950 -o valu_rate valu_rate.hip && ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ void __launch_bounds__(256) kern(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 11, a5 = a0 + 13,
             a6 = a0 ^ 17, a7 = a0 ^ 19;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if (KIND == 0) {   // v_xor_b32 / v_add_u32 (8 independent chains)
                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a0) : "v"(a1));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a1) : "v"(a2));
                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a2) : "v"(a3));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a3) : "v"(a4));
                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a4) : "v"(a5));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a5) : "v"(a6));
                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a6) : "v"(a7));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a7) : "v"(a0));
            } else if (KIND == 1) {   // v_alignbyte_b32 (3-operand)
                asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(a0) : "v"(a1));
                asm volatile("v_alignbyte_b32 %0, %0, %1, 2" : "+v"(a1) : "v"(a2));
                asm volatile("v_alignbyte_b32 %0, %0, %1, 3" : "+v"(a2) : "v"(a3));
                asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(a3) : "v"(a4));
                asm volatile("v_alignbyte_b32 %0, %0, %1, 2" : "+v"(a4) : "v"(a5));
                asm volatile("v_alignbyte_b32 %0, %0, %1, 3" : "+v"(a5) : "v"(a6));
                asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(a6) : "v"(a7));
                asm volatile("v_alignbyte_b32 %0, %0, %1, 2" : "+v"(a7) : "v"(a0));
            } else if (KIND == 2) {   // v_mul_u32_u24
                asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a0) : "v"(a1));
                asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a1) : "v"(a2));
                asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a2) : "v"(a3));
                asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a3) : "v"(a4));
                asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a4) : "v"(a5));
                asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a5) : "v"(a6));
                asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a6) : "v"(a7));
                asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a7) : "v"(a0));
            } else if (KIND == 3) {   // v_cndmask with a VCC compare in between (select pattern)
                asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a0) : "v"(a1) : "vcc");
                asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a2) : "v"(a3) : "vcc");
                asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a4) : "v"(a5) : "vcc");
                asm volatile("v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a6) : "v"(a7) : "vcc");
            } else if (KIND == 4) {   // s_add_u32 (SALU) chains
                unsigned s0 = 1, s1 = 2, s2 = 3, s3 = 4;
                asm volatile("s_add_u32 %0, %0, %1\n\ts_add_u32 %1, %1, %2\n\ts_add_u32 %2, %2, %3\n\ts_add_u32 %3, %3, %0\n\t"
                             "s_add_u32 %0, %0, %1\n\ts_add_u32 %1, %1, %2\n\ts_add_u32 %2, %2, %3\n\ts_add_u32 %3, %3, %0"
                             : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3));
                a0 += s0 + s1 + s2 + s3;
            } else if (KIND == 5) {   // DPP row_shr:1 moves
                asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(a0) : "v"(a1));
                asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(a2) : "v"(a3));
                asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(a4) : "v"(a5));
                asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(a6) : "v"(a7));
                asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(a1) : "v"(a0));
                asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(a3) : "v"(a2));
                asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(a5) : "v"(a4));
                asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(a7) : "v"(a6));
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int KIND>
void run(const char *name, int per_instr, unsigned *d) {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int iters = 4096;
    for (int wps = 1; wps <= 8; wps *= 2) {   // waves per SIMD = blocks (of 4 waves) per CU
        const int grid = cus * wps;
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        kern<KIND><<<grid, 256>>>(d, 16);
        hipEventRecord(e0);
        kern<KIND><<<grid, 256>>>(d, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        // wave-instructions per SIMD
        const double winst = (double)iters * 8 * per_instr * wps;
        const double cyc = ms * 1e-3 * 2.4e9;
        printf("%-22s waves/SIMD %d: %.3f ms, %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n",
               name, wps, ms, cyc / winst);
    }
}

int main() {
    unsigned *d;
    hipMalloc(&d, 256 * 256 * 64 * 4);
    run<0>("v_xor/v_add", 8, d);
    run<1>("v_alignbyte", 8, d);
    run<2>("v_mul_u32_u24", 8, d);
    run<3>("v_cmp+v_cndmask", 8, d);
    run<4>("s_add_u32 (SALU)", 8, d);
    run<5>("v_mov_dpp row_shr", 8, d);
    hipFree(d);
    return 0;
}
