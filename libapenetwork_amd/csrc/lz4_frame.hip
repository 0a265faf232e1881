// lz4_frame.hip -- framed stream of independent blocks for the socket path.
//
// The reference's LZ4 socket stream sends every 8 KiB chunk as
// [int32 host-endian compressed size][LZ4 block] (ref src/ape_socket.c:813-850),
// but its blocks are chained (each uses the previous 64 KiB as dictionary,
// compress_fast_continue :832), which serialises them.  The batched GPU path keeps
// the same frame layout with *independent* blocks (an
// opt-in wire change): frame i = [le32 c_i][c_i bytes], frames back to back.
//
//   frame_offsets: off[i] = sum_{j<i} (4 + c_j), off[N] = total (exclusive scan)
//   frame_pack   : compressed slots (strided) -> framed stream
// and the decoder reads blocks straight out of a framed stream (BlockArgs.frame_off).
//
// All of it is byte moving: HBM-bound, coalesced 16-byte accesses where the
// frame alignment allows, one wave per block for the pack.
#include "lz4_gpu_internal.h"

namespace apelz4 {

namespace {

constexpr int kScanTile = 1024;   // elements per workgroup tile (256 threads x 4)

__device__ __forceinline__ long long frame_len(const int *csize, int i, int n) {
    if (i >= n) return 0;
    const int c = csize[i];
    return 4 + (c > 0 ? c : 0);
}

// tile sums of (4 + c_i)
__global__ void __launch_bounds__(256) frame_tile_sum(const int *csize, int n, long long *tsum) {
    __shared__ long long red[256];
    const int base = blockIdx.x * kScanTile + threadIdx.x * 4;
    long long s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) s += frame_len(csize, base + k, n);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) tsum[blockIdx.x] = red[0];
}

// exclusive scan of the tile sums in place (one workgroup, any tile count)
__global__ void __launch_bounds__(256) frame_tile_scan(long long *tsum, int ntiles) {
    __shared__ long long buf[256];
    long long carry = 0;
    for (int t0 = 0; t0 < ntiles; t0 += 256) {
        const int t = t0 + threadIdx.x;
        const long long v = t < ntiles ? tsum[t] : 0;
        buf[threadIdx.x] = v;
        __syncthreads();
        for (int d = 1; d < 256; d <<= 1) {   // Hillis-Steele inclusive
            const long long x = threadIdx.x >= d ? buf[threadIdx.x - d] : 0;
            __syncthreads();
            buf[threadIdx.x] += x;
            __syncthreads();
        }
        if (t < ntiles) tsum[t] = carry + buf[threadIdx.x] - v;
        carry += buf[255];
        __syncthreads();
    }
}

// per-tile exclusive scan + tile offset -> off[i]; off[n] = total
__global__ void __launch_bounds__(256) frame_tile_apply(const int *csize, int n,
                                                        const long long *tsum, long long *off) {
    __shared__ long long buf[256];
    const int base = blockIdx.x * kScanTile + threadIdx.x * 4;
    long long v[4], s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) { v[k] = frame_len(csize, base + k, n); s += v[k]; }
    buf[threadIdx.x] = s;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
        const long long x = threadIdx.x >= d ? buf[threadIdx.x - d] : 0;
        __syncthreads();
        buf[threadIdx.x] += x;
        __syncthreads();
    }
    long long o = tsum[blockIdx.x] + buf[threadIdx.x] - s;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = base + k;
        if (i <= n) off[i] = o;   // i == n: the total
        o += v[k];
    }
}

// frame i = [le32 c][c bytes] at frames + off[i]; one wave per block
__global__ void __launch_bounds__(64) frame_pack_kernel(const char *comp, size_t stride,
                                                        const int *csize, const long long *off,
                                                        char *frames) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const int c = csize[b] > 0 ? csize[b] : 0;
    gcu8 *s = (gcu8 *)(comp + (size_t)b * stride);
    gu8 *d = (gu8 *)(frames + off[b]);
    if (lane < 4) d[lane] = (uint8_t)((uint32_t)c >> (8 * lane));
    d += 4;
    // 16 bytes per lane per step (unaligned 16-byte global accesses), byte tail
    const int c16 = c & ~15;
    for (int k = 16 * lane; k < c16; k += 1024) gstore16(d + k, gload16(s + k));
    for (int k = c16 + lane; k < c; k += 64) d[k] = s[k];
}

}  // namespace

hipError_t launch_frame_offsets(const int *csize, long long *off, long long *scratch, int n,
                                hipStream_t s) {
    const int ntiles = (n + 1 + kScanTile - 1) / kScanTile;   // covers index n (the total)
    hipLaunchKernelGGL(frame_tile_sum, dim3(ntiles), dim3(256), 0, s, csize, n, scratch);
    hipLaunchKernelGGL(frame_tile_scan, dim3(1), dim3(256), 0, s, scratch, ntiles);
    hipLaunchKernelGGL(frame_tile_apply, dim3(ntiles), dim3(256), 0, s, csize, n,
                       (const long long *)scratch, off);
    return hipGetLastError();
}

int frame_scratch_elems(int n) { return (n + 1 + kScanTile - 1) / kScanTile; }

hipError_t launch_frame_pack(const char *comp, size_t stride, const int *csize,
                             const long long *off, char *frames, int n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(frame_pack_kernel, dim3(n), dim3(64), 0, s, comp, stride, csize, off,
                       frames);
    return hipGetLastError();
}

}  // namespace apelz4
