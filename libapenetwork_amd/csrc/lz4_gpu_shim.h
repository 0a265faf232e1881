/* lz4_gpu_shim.h -- C-callable one-shot entry points into the HIP runtime
 * (lz4_runtime.hip), used by the C host implementation of ape_lz4.h.
 * `*rt` receives APE_LZ4_GPU_OK or a negative APE_LZ4_GPU_E* runtime error;
 * the return value is the codec result (only meaningful when *rt == 0). */
#pragma once
#if defined(__cplusplus)
extern "C" {
#endif
int ape_lz4_gpu_compress_one(const char *src, char *dst, int n, int cap, int accel, int *rt);
int ape_lz4_gpu_decompress_one(const char *src, char *dst, int csize, int cap, int partial,
                               int target, int *rt);
#if defined(__cplusplus)
}
#endif
