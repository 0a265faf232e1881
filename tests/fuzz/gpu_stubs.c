/* gpu_stubs.c -- TEST INFRASTRUCTURE for fuzz_host_codec: the harness links the product's
 * host ABI (ape_lz4_api.c + ape_lz4_host.c) without the HIP runtime.  With the default
 * routing no one-shot call reaches these; if one did, it fails loudly as on a box without
 * a device (APE_LZ4_GPU_ENODEV semantics), never silently. */
#include <stdlib.h>
int ape_lz4_gpu_compress_one(const char *s, char *d, int n, int cap, int accel, int *rt)
{
    (void)s; (void)d; (void)n; (void)cap; (void)accel; *rt = -1; abort();
}
int ape_lz4_gpu_decompress_one(const char *s, char *d, int c, int cap, int p, int t, int *rt)
{
    (void)s; (void)d; (void)c; (void)cap; (void)p; (void)t; *rt = -1; abort();
}
const char *APE_LZ4_gpu_last_error(void) { return "fuzz harness: no GPU runtime linked"; }
