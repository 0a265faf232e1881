// lz4_encode_seg.hip -- MI355X (gfx950) batched LZ4 block encoder, segment-parallel form.
//
// Replaces the per-block work of APE_LZ4_compress_default (ref src/ape_lz4.c:811-815 ->
// LZ4_compress_generic :530-755, byU16 / noDict, acceleration 1).  Like the reference it is
// a greedy LZ77 parse over a hash of 5 bytes; unlike it, the parse of one 64 KiB block is
// cut into 1024 independent 64-byte segments that 1024 lanes parse at once, against an
// index of the whole block that is built before any parsing.  The output is a valid LZ4
// v1.7.1 block (every rule decompress_safe enforces, :1346-1366, :1375, :1444-1447: matches
// start at <= n-12 and end at <= n-5, the last >= 5 bytes are literals), decoded by the
// reference itself in the tests; the bytes differ from the reference's.
//
// One 1024-thread workgroup (16 waves) per block, the whole block in LDS (64 KiB) next to
// its index, so that no parse step touches global memory:
//
//   LOAD   the block into LDS with 16-byte coalesced loads (its 16-byte-aligned chunks).
//   INDEX  every 4th position p (p <= n-13) hashed (5 bytes, 10 bits) and bucket-sorted by
//          a stable counting sort: per-wave bucket counts (wave w holds positions
//          [4096w, 4096w+4096)), a block-wide scan, then each wave scatters its own
//          positions in order -> pos[] holds each bucket's positions in ascending order.
//          Deterministic: no two waves ever update the same counter.
//   PARSE  lane k parses segment [64k, 64k+64) greedily, as the reference's search loop
//          (:591-619): at position q the bucket of hash(q) is binary-searched for the
//          four latest indexed positions < q; each is measured against q over 16 bytes
//          (LDS reads + v_alignbyte, xor, v_ffbl) and the longest wins (ties: the most
//          recent); a 16-byte match is extended 16 bytes at a time; catch-up backwards
//          into the segment's pending literals (:623-627).  A match may run up to 64
//          bytes past the segment end.  Records {start, length, offset} go to LDS.
//   SPLICE the end of each segment's last match, prefix-maxed over segments, is where the
//          next segment's kept sequences start: matches inside it are dropped, one that
//          straddles it is cut (kept if >= 4 bytes); literal runs join across segments.
//          Per-segment output sizes are prefix-summed into output offsets.
//   EMIT   each lane writes its sequences (token, length bytes, literals, offset) into an
//          LDS staging window (runs longer than 64 literals are copied by the whole wave),
//          and the window is stored to dst with coalesced stores; >36 KiB outputs take
//          more than one window.  A block the parse cannot shrink is stored as one literal
//          run, as the reference stores incompressible input (:732-751).
//
// Searching the latest four candidates instead of one gives a better ratio than the
// reference's single-candidate table (tools/seg_model.c: 3.30 vs 3.157 on SURVEY App. C
// data); the index of every 4th position and the segment cut cost little (catch-up finds
// the true match start; a segment's last match may overrun into the next segment).
#include "lz4_gpu_internal.h"

namespace apelz4 {

#ifdef APE_LZ4_STATS
__device__ unsigned long long g_seg_stats[16];
// per-phase cycle sums of the segment encoder (workgroup thread 0, barrier to barrier)
hipError_t seg_stats_read(unsigned long long *out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_seg_stats), sizeof(g_seg_stats));
    if (e == hipSuccess && reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_seg_stats), z, sizeof(z));
    }
    return e;
}
#endif

namespace {

constexpr int kSThreads = 1024, kSWaves = kSThreads / 64, kSHalf = kSWaves / 2;
constexpr int kSSeg = 16;                         // bytes per segment (a lane's unit of work)
constexpr int kSSegs = kMaxBlock / kSSeg;         // 4096 segments
constexpr int kSRecS = 3;                         // record slots per segment
constexpr int kSStride = 4;                       // indexed positions: multiples of 4
constexpr int kSHLog = 11, kSBuckets = 1 << kSHLog;
constexpr int kSIdx = kMaxBlock / kSStride;       // 16384 index entries
constexpr int kSCapX = 64;                        // a match may end this far past its segment
#ifndef APE_SEG_DEPTH
#define APE_SEG_DEPTH 4
#endif
constexpr int kSDepth = APE_SEG_DEPTH;            // candidates measured per position
constexpr int kSLongRun = 64;                     // longer literal runs: copied by the wave
constexpr int kSFront = 16;                       // zero bytes before the block (backward reads)
constexpr int kSBlkW = (kSFront + kMaxBlock + 64) / 4;   // block bytes at kSFront + a (a < 16) + padding

struct SegLds {
    uint32_t blk[kSBlkW];
    union {
        struct {
            uint16_t pos[kSIdx];
            uint32_t offs[kSBuckets + 1];
        } ix;
        uint8_t stage[kSIdx * 2 + (kSBuckets + 1) * 4];
    } u;
    union {
        struct {                                  // index build, one half of the waves at a time:
            uint32_t cnt[kSHalf * kSBuckets / 2]; // per-wave u16 bucket counters, packed in pairs
            uint32_t tot[kSBuckets];              // bucket totals, then the second half's starts
        } ib;
        uint32_t rec[kSRecS * kSSegs];            // parse: slot r of segment g at [r*4096 + g]
    } r;
    uint32_t wsum[kSWaves];
    uint32_t wmax[kSWaves];
    uint32_t segnext;                             // parse: next segment to hand out
};
constexpr int kSStage = (int)sizeof(((SegLds *)0)->u.stage) & ~15;
static_assert(sizeof(SegLds) <= 160 * 1024, "LDS");
static_assert(kSSeg == 16 && kSThreads * 4 == kSSegs, "a thread's 64-byte region = 4 segments (start field: 4 bits)");

__device__ __forceinline__ uint32_t sffbl(uint32_t d) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(d));
    return r;
}

// hash of the 5 bytes x (little-endian dword) + b4 onto kSHLog bits: two full-rate 24-bit
// multiplies (v_mul_u32_u24 / v_mad_u32_u24)
__device__ __forceinline__ uint32_t shash(uint32_t x, uint32_t b4) {
    const uint32_t lo = x & 0xFFFFFFu, hi = (x >> 24) | ((b4 & 0xFFu) << 8);
    // (__umul24 returns int: the sum is shifted as unsigned)
    return ((uint32_t)__umul24(lo, 0x9E3779u) + (uint32_t)__umul24(hi, 0xC2B2AEu)) >> (32 - kSHLog);
}

// 16 / 4 bytes at byte address x of the block buffer.  Default: single unaligned LDS reads
// (gfx950 serves any alignment; aligned dword reads + v_alignbyte were measured no faster,
// and an 8-byte prefilter choosing one of the four candidates -3.5 % time for ratio 3.39 -> 3.19).
typedef uint32_t l32x4 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t l32x4a2 __attribute__((ext_vector_type(4), aligned(2)));
typedef uint32_t l32 __attribute__((aligned(1)));
typedef uint32_t l32x2 __attribute__((ext_vector_type(2), aligned(1)));
__device__ __forceinline__ uint4 lds16(const SegLds &S, uint32_t x) {
    const l32x4 v = *(const l32x4 *)((const uint8_t *)S.blk + x);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t lds4(const SegLds &S, uint32_t x) {
    return *(const l32 *)((const uint8_t *)S.blk + x);
}
__device__ __forceinline__ uint32_t ldsb(const SegLds &S, uint32_t x) {
    return ((const uint8_t *)S.blk)[x];
}

// common prefix of A and B in bytes (0..16): first differing bit by ffbl + saturating add + min
__device__ __forceinline__ uint32_t prefix16(uint4 A, uint4 B) {
    uint32_t m = sffbl(A.x ^ B.x);
    m = umin(m, __builtin_elementwise_add_sat(sffbl(A.y ^ B.y), 32u));
    m = umin(m, __builtin_elementwise_add_sat(sffbl(A.z ^ B.z), 64u));
    m = umin(m, __builtin_elementwise_add_sat(sffbl(A.w ^ B.w), 96u));
    return umin(m, 128u) >> 3;
}

__device__ __forceinline__ int extlen(int v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }

// Diagnostic build (-DAPE_SEG_GUARD, never the product): every data-dependent loop gets an
// iteration bound; a tripped bound ends the loop and marks the block's result.
#ifdef APE_SEG_GUARD
#define SGUARD(cnt, lim, code) if (++(cnt) > (lim)) { g_trip = (code); break; }
#define SGUARD_DECL(cnt) int cnt = 0;
#else
#define SGUARD(cnt, lim, code)
#define SGUARD_DECL(cnt)
#endif

// block-wide exclusive sum over the 1024 threads; *total = the sum of all
__device__ __forceinline__ uint32_t block_excl_sum(SegLds &S, uint32_t v, int wave, int lane,
                                                   uint32_t *total) {
    const uint32_t inc = wave_incl_sum(v);
    if (lane == 63) S.wsum[wave] = inc;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kSWaves; w++) {
        const uint32_t t = S.wsum[w];
        before += w < wave ? t : 0u;
        all += t;
    }
    __syncthreads();
    *total = all;
    return before + inc - v;
}

// block-wide exclusive max (0 for thread 0); *total = the max of all
__device__ __forceinline__ uint32_t block_excl_max(SegLds &S, uint32_t v, int wave, int lane,
                                                   uint32_t *total) {
    const uint32_t inc = wave_incl_max(v);
    if (lane == 63) S.wmax[wave] = inc;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kSWaves; w++) {
        const uint32_t t = S.wmax[w];
        before = w < wave ? umax(before, t) : before;
        all = umax(all, t);
    }
    __syncthreads();
    *total = all;
    return umax(before, wave_shr1(inc, 0u));
}

// one output byte at absolute position o, if it falls into the staging window [w0, w0+kSStage)
__device__ __forceinline__ void put(SegLds &S, uint32_t o, uint32_t w0, uint32_t v) {
    const uint32_t i = o - w0;
    if (i < (uint32_t)kSStage) S.u.stage[i] = (uint8_t)v;
}

// the length bytes after a token nibble of 15: (v - 15) / 255 bytes of 255 and the rest
__device__ __forceinline__ uint32_t put_len(SegLds &S, uint32_t o, uint32_t w0, int v) {
    v -= 15;
#pragma unroll 1
    for (; v >= 255; v -= 255) put(S, o++, w0, 255u);
    put(S, o++, w0, (uint32_t)v);
    return o;
}

}  // namespace

__global__ void __launch_bounds__(kSThreads) lz4_encode_seg_kernel(BlockArgs a) {
    __shared__ SegLds S;
    STATS_DECL
#ifdef APE_SEG_GUARD
    int g_trip = 0;
    if (threadIdx.x == 0) S.wmax[15] = 0u;
#endif
    const int b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const char *srcp = a.src ? a.src[b] : a.src_base + (size_t)b * a.src_stride;
    char *dstp = a.dst ? a.dst[b] : a.dst_base + (size_t)b * a.dst_stride;
    const int n = a.src_size[b];
    const int cap = a.dst_cap ? a.dst_cap[b] : (int)a.dst_stride;
    if (n < 0 || n > kMaxBlock || cap < 0) {
        if (tid == 0) a.result[b] = (n > kMaxBlock) ? kErange : 0;
        return;
    }

    // ---- LOAD: the 16-byte-aligned chunks that hold the block's bytes; byte i of the
    // block lands at blk byte a0 = 16 + a + i.  Chunks outside the block are never read (a chunk
    // with one valid byte lies in the same page as that byte); the padding is zeroed.
    const uint32_t amis = (uint32_t)((uintptr_t)srcp & 15u);
    const uint32_t a0 = (uint32_t)kSFront + amis;   // blk byte of block byte 0
    {
        const u32x4_u *g = (const u32x4_u *)(srcp - amis);
        const int nch = n > 0 ? (int)((amis + (uint32_t)n + 15u) >> 4) : 0;
        uint4 *L = (uint4 *)S.blk;
        for (int c = tid; c < kSBlkW / 4; c += kSThreads) {
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            const int gc = c - kSFront / 16;
            if (gc >= 0 && gc < nch) {
                const u32x4_u t = __builtin_nontemporal_load(g + gc);
                v = make_uint4(t.x, t.y, t.z, t.w);
            }
            L[c] = v;
        }
        for (int i = tid; i < kSHalf * kSBuckets / 2 + kSBuckets; i += kSThreads) S.r.ib.cnt[i] = 0u;
    }
    __syncthreads();

    STAT(0);
    // ---- INDEX: stable counting sort of positions 4i (4i <= n-13) by hash ----
    // Wave w holds index entries [1024w, 1024w + 1024).  Bucket totals first; then, one half
    // of the waves at a time (the per-wave counters of all 16 waves do not fit beside the
    // rest), per-wave counts -> per-wave starts -> each wave scatters its own entries in
    // order.  No two waves update one counter, and a wave's atomics on one counter return in
    // lane order, so every bucket lists its positions in ascending order, deterministically.
    const int nidx = n >= 13 ? (n - 13) / kSStride + 1 : 0;
    uint16_t *c16 = (uint16_t *)S.r.ib.cnt;
    const bool first_half = wave < kSHalf;
    const int hw = wave & (kSHalf - 1);
#pragma unroll 4
    for (int r = 0; r < 16; r++) {
        const int i = wave * 1024 + r * 64 + lane;
        if (i < nidx) {
            const uint32_t x = a0 + (uint32_t)(i * kSStride);
            const uint32_t h = shash(lds4(S, x), ldsb(S, x + 4));
            atomicAdd(&S.r.ib.tot[h], 1u);
            if (first_half) atomicAdd(&S.r.ib.cnt[hw * (kSBuckets / 2) + (h >> 1)], (h & 1u) ? 0x10000u : 1u);
        }
    }
    __syncthreads();
    {   // bucket starts (two buckets per thread), then the first half's per-wave starts
        const int h0 = 2 * tid;
        const uint32_t t0 = S.r.ib.tot[h0], t1 = S.r.ib.tot[h0 + 1];
        uint32_t all;
        const uint32_t base = block_excl_sum(S, t0 + t1, wave, lane, &all);
        S.u.ix.offs[h0] = base;
        S.u.ix.offs[h0 + 1] = base + t0;
        if (tid == kSThreads - 1) S.u.ix.offs[kSBuckets] = all;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int h = h0 + k;
            uint32_t at = base + (k ? t0 : 0u);
#pragma unroll
            for (int w = 0; w < kSHalf; w++) {
                const uint32_t c = c16[w * kSBuckets + h];
                c16[w * kSBuckets + h] = (uint16_t)at;
                at += c;
            }
            S.r.ib.tot[h] = at;   // where the second half's entries of bucket h begin
        }
    }
    __syncthreads();
#pragma unroll 1
    for (int half = 0; half < 2; half++) {
        if (half == 1) {   // per-wave counts of the second half
            for (int i = tid; i < kSHalf * kSBuckets / 2; i += kSThreads) S.r.ib.cnt[i] = 0u;
            __syncthreads();
            if (!first_half) {
#pragma unroll 4
                for (int r = 0; r < 16; r++) {
                    const int i = wave * 1024 + r * 64 + lane;
                    if (i < nidx) {
                        const uint32_t x = a0 + (uint32_t)(i * kSStride);
                        const uint32_t h = shash(lds4(S, x), ldsb(S, x + 4));
                        atomicAdd(&S.r.ib.cnt[hw * (kSBuckets / 2) + (h >> 1)], (h & 1u) ? 0x10000u : 1u);
                    }
                }
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const int h = 2 * tid + k;
                uint32_t at = S.r.ib.tot[h];
#pragma unroll
                for (int w = 0; w < kSHalf; w++) {
                    const uint32_t c = c16[w * kSBuckets + h];
                    c16[w * kSBuckets + h] = (uint16_t)at;
                    at += c;
                }
            }
            __syncthreads();
        }
        if (first_half == (half == 0)) {
#pragma unroll 1
            for (int r = 0; r < 16; r++) {   // in order: a wave's entries enter each bucket ascending
                const int i = wave * 1024 + r * 64 + lane;
                if (i < nidx) {
                    const uint32_t x = a0 + (uint32_t)(i * kSStride);
                    const uint32_t h = shash(lds4(S, x), ldsb(S, x + 4));
                    const uint32_t old = atomicAdd(&S.r.ib.cnt[hw * (kSBuckets / 2) + (h >> 1)],
                                                   (h & 1u) ? 0x10000u : 1u);
                    const uint32_t slot = (old >> ((h & 1u) * 16)) & 0xFFFFu;
#ifdef APE_SEG_GUARD
                    if (slot >= (uint32_t)nidx) atomicOr(&S.wmax[15], 1u << 5);
#endif
                    S.u.ix.pos[slot] = (uint16_t)(i * kSStride);
                }
            }
        }
        __syncthreads();
    }

#ifdef APE_SEG_GUARD
    {   // diagnostic: index consistency (bits of the block's result)
        int bad = 0;
        if (tid == 0 && S.u.ix.offs[kSBuckets] != (uint32_t)nidx) atomicOr(&S.wmax[15], 1u << 2);
        for (int hh = tid; hh < kSBuckets; hh += kSThreads) {
            const uint32_t o0 = S.u.ix.offs[hh], o1 = S.u.ix.offs[hh + 1];
            if (o1 < o0) atomicOr(&S.wmax[15], 1u << 1);
            for (uint32_t k = o0 + 1; k < o1 && k < (uint32_t)kSIdx; k++)
                bad += S.u.ix.pos[k] <= S.u.ix.pos[k - 1];
            for (uint32_t k = o0; k < o1 && k < (uint32_t)kSIdx; k++)
                if (shash(lds4(S, a0 + S.u.ix.pos[k]), ldsb(S, a0 + S.u.ix.pos[k] + 4)) != (uint32_t)hh) { atomicOr(&S.wmax[15], 1u << 4); break; }
        }
        if (bad) atomicOr(&S.wmax[15], 1u << 3);
        __syncthreads();
        if (S.wmax[15]) g_trip = 100 + (int)S.wmax[15];
        __syncthreads();
    }
#endif
    STAT(1);
#ifdef APE_SEG_INDEXONLY   // diagnostic: load + index alone
    if (tid == 0) a.result[b] = 1;
    return;
#endif
    // ---- PARSE: 16-byte segments, handed out to the lanes as they finish ----
    // Thread t starts with segment t; a lane whose segment is done takes the next one from a
    // block-wide counter (one LDS atomic per wave and round), so the waves finish together
    // instead of waiting for the wave with the slowest 4 KiB.  A segment's records depend only
    // on its bytes and the index, not on the lane that parses it: the output is deterministic.
    const int mfl = n - 12;                  // matches start at <= n-12 (:585)
    for (int i = tid; i < kSRecS * kSSegs; i += kSThreads) S.r.rec[i] = 0u;   // empty slots
    if (tid == 0) S.segnext = (uint32_t)kSThreads;
    __syncthreads();
#ifdef APE_LZ4_STATS
    uint32_t c_probe = 0, c_bs = 0, c_ext = 0, c_cu = 0;
#define SCOUNT(v) (v)++
#else
#define SCOUNT(v)
#endif
    {
        const float inv_span = 1.0f / (float)(nidx * kSStride > 0 ? nidx * kSStride : 1);
        int seg = tid;                       // block segment
        int gs = 0, s1 = 0, capE = 0, q = 0, anchor = 0, nrec = 0;
        auto start_seg = [&]() {
            gs = seg;
            const int s0 = gs * kSSeg;
            if (seg >= kSSegs || s0 >= n || s0 > mfl) {
                seg = kSSegs;   // nothing left for this lane
                return;
            }
            s1 = s0 + kSSeg < n ? s0 + kSSeg : n;
            // matches end at <= n-12 (not n-5): a match cut to start where the coverage of
            // the segments before ends then still starts at <= n-12
            capE = s1 + kSCapX < mfl ? s1 + kSCapX : mfl;
            q = s0 > 1 ? s0 : 1;
            anchor = s0;
            nrec = 0;
        };
        start_seg();
        SGUARD_DECL(gp)
        for (;;) {
            const bool act = seg < kSSegs;
            if (!wave_any(act)) break;
            if (act) {
                SGUARD(gp, 4096, 1)
                SCOUNT(c_probe);
                const uint4 own = lds16(S, a0 + (uint32_t)q);
                const uint32_t h = shash(own.x, own.y);
                const int blo = (int)S.u.ix.offs[h], bhi = (int)S.u.ix.offs[h + 1];
                // The bucket lists its positions in ascending order, spread about evenly over
                // the block: read the 8 entries around where q falls (one LDS read) and find
                // the first >= q among them.  When they do not bracket q: binary search (rare).
                const int est = blo + (int)((float)(bhi - blo) * ((float)q * inv_span));
                int w0 = est - 5 < bhi - 8 ? est - 5 : bhi - 8;
                w0 = w0 > blo ? w0 : blo;
                const l32x4a2 Wv = *(const l32x4a2 *)&S.u.ix.pos[w0];
                const int nv = bhi - w0;   // window entries inside the bucket
                uint32_t e8[8];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const uint32_t dw = i < 2 ? Wv.x : i < 4 ? Wv.y : i < 6 ? Wv.z : Wv.w;
                    e8[i] = i < nv ? ((dw >> ((i & 1) * 16)) & 0xFFFFu) : 0x10000u;
                }
                // ascending: k = entries < q by three compares
                int k = e8[3] < (uint32_t)q ? 4 : 0;
                {
                    const uint32_t v1 = k ? e8[5] : e8[1];
                    k += v1 < (uint32_t)q ? 2 : 0;
                    const uint32_t v0 = k == 0 ? e8[0] : k == 2 ? e8[2] : k == 4 ? e8[4] : e8[6];
                    k += v0 < (uint32_t)q ? 1 : 0;
                    if (k == 7 && e8[7] < (uint32_t)q) k = 8;
                }
                uint64_t r4;   // entries lb-4 .. lb-1 (lb = w0 + k), 16 bits each, lb-1 on top
                int lb = w0 + k, wlo = w0;   // entries below wlo are not in r4
                if ((k == 0 && w0 > blo) || (k == 8 && w0 + 8 < bhi)) {
                    int lo = blo, hi = bhi;
                    SGUARD_DECL(gb)
                    while (lo < hi) {   // first entry >= q
                        SGUARD(gb, 40, 2)
                        SCOUNT(c_bs);
                        const int mid = (lo + hi) >> 1;
                        if ((int)S.u.ix.pos[mid] < q) lo = mid + 1;
                        else hi = mid;
                    }
                    lb = lo;
                    wlo = blo;
                    r4 = 0;
#pragma unroll
                    for (int d = 0; d < 4; d++)
                        if (lb - 4 + d >= blo) r4 |= (uint64_t)S.u.ix.pos[lb - 4 + d] << (16 * d);
                } else {
                    const uint64_t lo64 = ((uint64_t)Wv.y << 32) | Wv.x, hi64 = ((uint64_t)Wv.w << 32) | Wv.z;
                    const int sh = (k - 4) * 16;
                    r4 = sh >= 64 ? hi64 : sh > 0 ? (lo64 >> sh) | (hi64 << (64 - sh)) : sh == 0 ? lo64 : lo64 << (-sh);
                }
                const int room = capE - q;
                int best = 0, bestc = 0;
                // the four latest candidates; those whose first 4 bytes match are measured,
                // one at a time per lane (a loop as long as the lane with the most of them)
                int cd[kSDepth];
                uint32_t okm = 0;
#pragma unroll
                for (int d = 0; d < kSDepth; d++) {
                    const int j = lb - 1 - d;
                    cd[d] = (int)((r4 >> (48 - 16 * d)) & 0xFFFFu);
                    if (j >= wlo && cd[d] < q && lds4(S, a0 + (uint32_t)cd[d]) == own.x) okm |= 1u << d;
                }
                if (room < kMinMatch) okm = 0;
                while (okm) {
                    const uint32_t d = (uint32_t)__builtin_ctz(okm);
                    okm &= okm - 1u;
                    const int c = d == 0 ? cd[0] : d == 1 ? cd[1] : d == 2 ? cd[2] : cd[3];
                    int l = (int)prefix16(own, lds16(S, a0 + (uint32_t)c));
                    l = l < room ? l : room;
                    if (l > best) { best = l; bestc = c; }
                }
                if (best < kMinMatch) {
                    q++;
                } else {
                    int len = best;
                    if (best == 16) {
                        SGUARD_DECL(ge)
                        while (len < room) {
                            SGUARD(ge, 40, 3)
                            SCOUNT(c_ext);
                            const int l = (int)prefix16(lds16(S, a0 + (uint32_t)(q + len)),
                                                        lds16(S, a0 + (uint32_t)(bestc + len)));
                            len += l;
                            if (l < 16) break;
                        }
                        len = len < room ? len : room;
                    }
                    int m = q, c = bestc;   // catch-up (:623-627): up to 4 bytes, one compare
                    {
                        SCOUNT(c_cu);
                        const int room_b = (m - anchor) < c ? (m - anchor) : c;
                        const uint32_t x = lds4(S, a0 + (uint32_t)(m - 4)) ^ lds4(S, a0 + (uint32_t)(c - 4));
                        const int eq = x ? (int)(__builtin_clz(x) >> 3) : 4;   // equal bytes just before
                        const int t = room_b <= 0 ? 0 : (eq < room_b ? eq : room_b);
                        m -= t;
                        c -= t;
                        len += t;
                    }
                    S.r.rec[nrec * kSSegs + gs] = (uint32_t)(m - gs * kSSeg) | ((uint32_t)len << 4) | ((uint32_t)(m - c) << 16);
                    nrec++;
                    anchor = m + len;
                    q = anchor;
                }
            }
            const bool done = act && (q >= s1 || q > mfl || nrec >= kSRecS);
            const uint64_t D = wave_ballot(done);
            if (D) {
                const int f = __builtin_ctzll(D);
                uint32_t nb0 = 0;
                if (lane == f) nb0 = atomicAdd(&S.segnext, (uint32_t)__popcll(D));
                nb0 = lane_val(nb0, f);
                if (done) {
                    seg = (int)nb0 + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(D >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)D, 0u));
                    start_seg();
                }
            }
        }
    }
    STAT(2);
#ifdef APE_LZ4_STATS
    {   // wave-max and lane-sum of the loop counts, for wave 0
        const uint32_t mp = lane_val(wave_incl_max(c_probe), 63), mb = lane_val(wave_incl_max(c_bs), 63);
        const uint32_t me = lane_val(wave_incl_max(c_ext), 63), mc = lane_val(wave_incl_max(c_cu), 63);
        const uint32_t sp = lane_val(wave_incl_sum(c_probe), 63);
        STAT_ADD(11, mp);
        STAT_ADD(12, mb);
        STAT_ADD(13, me);
        STAT_ADD(14, mc);
        STAT_ADD(15, sp);
    }
#endif

#ifdef APE_SEG_PARSEONLY   // diagnostic: instruction counts of load + index + parse alone
    if (tid == 0) a.result[b] = 1;
    return;
#endif
    // ---- SPLICE: thread t owns the 64-byte region of segments 4t .. 4t+3 ----
    // Its records, in order, are walked against the coverage C that the regions before it
    // leave: a match ending inside C is dropped, one that straddles it is cut (kept if >= 4
    // bytes), and a kept match that starts exactly where the previous one ends, at its offset,
    // continues it (one match re-found by the next 16-byte segment).  The region's walk is a
    // function f_t(C) of the incoming coverage; C_t = f_t(C_{t-1}) is scanned as keys
    // C << 10 | t of the regions that produce coverage (0 for the others), so that the
    // exclusive prefix max also names the producer: the fixed point of
    // key = excl-prefix-max(f(key)), reached from the plain prefix max of the regions' last
    // match ends in one or two rounds (a cut < 4 bytes is rare); a sequential pass settles
    // the rest.
    const int s0 = tid * 64;   // this thread's region
    auto rec_at = [&](int i) -> uint32_t {   // i-th slot of the region: segment i / 3, slot i % 3
        return S.r.rec[(i % kSRecS) * kSSegs + tid * 4 + i / kSRecS];
    };
    auto region_f = [&](uint32_t c) -> uint32_t {   // coverage after the region, entering with c
        uint32_t pe = c;
#pragma unroll 1
        for (int i = 0; i < 4 * kSRecS; i++) {
            const uint32_t w = rec_at(i);
            if (!w) continue;
            const uint32_t m = (uint32_t)s0 + (uint32_t)(i / kSRecS) * kSSeg + (w & 15u), e = m + ((w >> 4) & 4095u);
            if (e <= pe) continue;
            if (m < pe && e - pe < (uint32_t)kMinMatch) continue;
            pe = e;
        }
        return pe;
    };
    uint32_t elast = 0;
#pragma unroll 1
    for (int i = 0; i < 4 * kSRecS; i++) {
        const uint32_t w = rec_at(i);
        if (w) {
            const uint32_t e = (uint32_t)s0 + (uint32_t)(i / kSRecS) * kSSeg + (w & 15u) + ((w >> 4) & 4095u);
            elast = e > elast ? e : elast;
        }
    }
    const uint32_t key0 = elast ? (elast << 10) | (uint32_t)tid : 0u;
    uint32_t allk;
    uint32_t ck = block_excl_max(S, key0, wave, lane, &allk);
    STAT(3);
    for (int it = 0;; it++) {
        const uint32_t cin = ck >> 10, cout = region_f(cin);
        const uint32_t E = cout > cin ? (cout << 10) | (uint32_t)tid : 0u;
        uint32_t all2;
        const uint32_t c2 = block_excl_max(S, E, wave, lane, &all2);
        const bool moved = c2 != ck;
        ck = c2;
        allk = all2;
        if (!__syncthreads_or(moved)) break;
        if (it == 3) {   // sequential: thread 0 walks the regions (their outgoing coverage
                         // depends on the incoming one: each thread tabulates nothing; so
                         // thread 0 asks each region in turn through LDS)
            uint32_t *cv = (uint32_t *)S.u.stage;   // cv[t] = incoming key of region t
            if (tid == 0) cv[0] = 0u;
            for (int t2 = 0; t2 < kSThreads; t2++) {
                __syncthreads();
                if (tid == t2) {
                    const uint32_t ci = cv[t2] >> 10, co = region_f(ci);
                    if (t2 + 1 < kSThreads) cv[t2 + 1] = co > ci ? (co << 10) | (uint32_t)t2 : cv[t2];
                    else S.wmax[0] = co > ci ? (co << 10) | (uint32_t)t2 : cv[t2];
                }
            }
            __syncthreads();
            ck = cv[tid];
            allk = S.wmax[0];
            __syncthreads();
            break;
        }
    }
    const uint32_t cover = ck >> 10, cover_all = allk >> 10;

    // The region's kept sequences, local continuations folded: fn(lit_start, m, len, off, k)
    // for the k-th sequence (k = 1, 2, ...); returns the count.
    auto walk = [&](auto fn) -> uint32_t {
        uint32_t pe = cover, cnt = 0, pm = 0, plen = 0, poff = 0, plit = 0;
        bool have = false;
#pragma unroll 1
        for (int i = 0; i < 4 * kSRecS; i++) {
            const uint32_t w = rec_at(i);
            if (!w) continue;
            uint32_t m = (uint32_t)s0 + (uint32_t)(i / kSRecS) * kSSeg + (w & 15u), len = (w >> 4) & 4095u;
            const uint32_t off = w >> 16, e = m + len;
            if (e <= pe) continue;
            if (m < pe) {
                if (e - pe < (uint32_t)kMinMatch) continue;
                len = e - pe;
                m = pe;
            }
            if (have && m == pm + plen && off == poff) {
                plen += len;   // the same match, re-found by the next segment
            } else {
                if (have) fn(plit, pm, plen, poff, ++cnt);
                plit = pe;
                pm = m;
                plen = len;
                poff = off;
                have = true;
            }
            pe = e;
        }
        if (have) fn(plit, pm, plen, poff, ++cnt);
        return cnt;
    };

    // Runs longer than a region: a region's first kept sequence that starts exactly where the
    // coverage ends, at the offset of the sequence that ends there, continues that sequence.
    // It is folded into its head: T_t = val_t + (pass_t ? T_{t+1} : 0) sums the continuations
    // after region t (val = the continuing length, pass = the region holds nothing else, so
    // the chain goes on), a segmented suffix scan; the head (a region's last kept sequence)
    // takes T_{t+1} on top.
    uint32_t f_m = 0, f_len = 0, f_off = 0, l_off = 0;
    const uint32_t kc = walk([&](uint32_t, uint32_t m, uint32_t len, uint32_t off, uint32_t k) {
        if (k == 1) { f_m = m; f_len = len; f_off = off; }
        l_off = off;
    });
    uint32_t *segoff = (uint32_t *)S.u.stage;            // [1024] last kept offset
    uint32_t *segvp = segoff + kSThreads;                 // [1024] val | !pass << 31
    uint32_t *segT = segvp + kSThreads;                   // [1025] T_t
    segoff[tid] = l_off;
    __syncthreads();
    const bool cont = kc > 0 && ck != 0u && f_m == cover && f_off == segoff[ck & 1023u];
    const uint32_t val = cont ? f_len : 0u;
    const bool pass = kc == 0 || (cont && kc == 1);
    segvp[tid] = val | (pass ? 0u : 0x80000000u);
    if (tid == 0) segT[kSThreads] = 0u;
    __syncthreads();
    {   // thread t scans region 1023 - t: S_t = x_t + (reset_t ? 0 : S_{t-1})
        const uint32_t vp = segvp[kSThreads - 1 - tid];
        uint32_t x = vp & 0x7FFFFFFFu, fl = vp >> 31;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {   // wave segmented scan (flag, value) pairs
            const uint32_t px = __shfl_up(x, d), pf = __shfl_up(fl, d);
            if (lane >= d) {
                x = fl ? x : x + px;
                fl |= pf;
            }
        }
        // carry across waves: lanes without a reset before them take the previous waves'
        // running value (sequential over the 16 wave totals in LDS)
        if (lane == 63) {
            S.wsum[wave] = x;
            S.wmax[wave] = fl;
        }
        __syncthreads();
        uint32_t carry = 0;
        for (int w = 0; w < wave; w++) carry = S.wmax[w] ? S.wsum[w] : carry + S.wsum[w];
        if (!fl) x += carry;
        segT[kSThreads - 1 - tid] = x;
        __syncthreads();
    }
    const uint32_t tail = segT[tid + 1];   // T_{t+1}
    uint32_t sz = 0;
    walk([&](uint32_t lit0, uint32_t m, uint32_t len, uint32_t, uint32_t k) {
        if (k == 1 && cont) return;   // a continuation's bytes are its head's
        const uint32_t L = len + (k == kc ? tail : 0u);
        const int lit = (int)(m - lit0);
        sz += 1u + (uint32_t)extlen(lit) + (uint32_t)lit + 2u + (uint32_t)extlen((int)L - 4);
    });
    __syncthreads();   // segT / segvp (stage area) read before the emission writes it
    STAT(4);
    uint32_t body;
    const uint32_t obase = block_excl_sum(S, sz, wave, lane, &body);
    const int lastrun = n - (int)cover_all;
    const uint32_t total = body + 1u + (uint32_t)extlen(lastrun) + (uint32_t)lastrun;
    const uint32_t litonly = 1u + (uint32_t)extlen(n) + (uint32_t)n;

    STAT(5);
    if (total >= litonly) {
        // ---- incompressible: one literal run (what the reference emits for such input) ----
        if (litonly > (uint32_t)cap) {
            if (tid == 0) a.result[b] = 0;
            return;
        }
        const int hdr = 1 + extlen(n);
        uint8_t *d = (uint8_t *)dstp;
        for (int i = tid; i < hdr; i += kSThreads)
            d[i] = (uint8_t)(i == 0 ? (n >= 15 ? 0xF0 : n << 4) : (i < hdr - 1 ? 255 : (n - 15) % 255));
        for (int i = tid; i < n; i += kSThreads) d[hdr + i] = (uint8_t)ldsb(S, a0 + (uint32_t)i);
        if (tid == 0) a.result[b] = (int)litonly;
        return;
    }
    if (total > (uint32_t)cap) {
        if (tid == 0) a.result[b] = 0;
        return;
    }

#ifdef APE_SEG_NOEMIT   // diagnostic: everything but the emission
    if (tid == 0) a.result[b] = (int)total;
    return;
#endif
    // ---- EMIT: staging windows of kSStage bytes ----
#pragma unroll 1
    for (uint32_t w0 = 0; w0 < total; w0 += (uint32_t)kSStage) {
        __syncthreads();   // the index (first window) / the previous window's store is done
        uint32_t lsrc = 0, ldst = 0, llen = 0;   // this lane's long literal run, if any
        {
            uint32_t o = obase;
            walk([&](uint32_t lit0, uint32_t m, uint32_t len, uint32_t off, uint32_t k) {
                if (k == 1 && cont) return;   // continuation: written with its head
                if (k == kc) len += tail;
                const int lit = (int)(m - lit0), ml = (int)len - 4;
                put(S, o++, w0, ((uint32_t)(lit < 15 ? lit : 15) << 4) | (uint32_t)(ml < 15 ? ml : 15));
                if (lit >= 15) o = put_len(S, o, w0, lit);
                if (lit > kSLongRun) {
                    lsrc = lit0;
                    ldst = o;
                    llen = (uint32_t)lit;
                } else {
#pragma unroll 1
                    for (int i = 0; i < lit; i++) put(S, o + (uint32_t)i, w0, ldsb(S, a0 + lit0 + (uint32_t)i));
                }
                o += (uint32_t)lit;
                put(S, o++, w0, off & 255u);
                put(S, o++, w0, off >> 8);
                if (ml >= 15) o = put_len(S, o, w0, ml);
            });
            if (tid == kSThreads - 1) {   // the last literals (:732-751)
                uint32_t o2 = body;
                put(S, o2++, w0, (uint32_t)(lastrun < 15 ? lastrun : 15) << 4);
                if (lastrun >= 15) o2 = put_len(S, o2, w0, lastrun);
                // (a long last run is copied by the wave in the second pass below: a lane
                // has at most one long run among its own sequences, the first one's)
                if (lastrun <= kSLongRun)
#pragma unroll 1
                    for (int i = 0; i < lastrun; i++) put(S, o2 + (uint32_t)i, w0, ldsb(S, a0 + cover_all + (uint32_t)i));
            }
        }
        // long literal runs, copied by the whole wave one lane's run at a time
#pragma unroll 1
        for (int pass = 0; pass < 2; pass++) {
            uint32_t ps = lsrc, pd = ldst, pl = llen;
            if (pass == 1) {
                pl = 0;
                if (tid == kSThreads - 1 && lastrun > kSLongRun) {
                    ps = cover_all;
                    pd = body + 1u + (uint32_t)extlen(lastrun);
                    pl = (uint32_t)lastrun;
                }
            }
            uint64_t mk = wave_ballot(pl > 0);
            while (mk) {
                const int j = __builtin_ctzll(mk);
                mk &= mk - 1;
                const uint32_t s = lane_val(ps, j), d = lane_val(pd, j), L = lane_val(pl, j);
                // only the part inside the window
                const uint32_t lo = d > w0 ? 0u : w0 - d;
                const uint32_t hi = d + L < w0 + (uint32_t)kSStage ? L : (w0 + (uint32_t)kSStage > d ? w0 + (uint32_t)kSStage - d : 0u);
#pragma unroll 1
                for (uint32_t i = lo + (uint32_t)lane; i < hi; i += 64u)
                    S.u.stage[d + i - w0] = (uint8_t)ldsb(S, a0 + s + i);
            }
        }
        __syncthreads();
        // store the window
        const uint32_t wl = total - w0 < (uint32_t)kSStage ? total - w0 : (uint32_t)kSStage;
        uint8_t *d = (uint8_t *)dstp + w0;
        if (((uintptr_t)d & 3u) == 0) {
            const uint32_t nw = wl >> 2;
            for (uint32_t i = (uint32_t)tid; i < nw; i += kSThreads)
                ((uint32_t *)d)[i] = ((const uint32_t *)S.u.stage)[i];
            for (uint32_t i = (nw << 2) + (uint32_t)tid; i < wl; i += kSThreads) d[i] = S.u.stage[i];
        } else {
            for (uint32_t i = (uint32_t)tid; i < wl; i += kSThreads) d[i] = S.u.stage[i];
        }
    }
    STAT(6);
    STAT_ADD(10, 1);
    STATS_FLUSH(g_seg_stats);
#ifdef APE_SEG_GUARD
    if (g_trip) a.result[b] = -1000000 - g_trip * 1000 - (tid & 1023) * 0;
    else
#endif
    if (tid == 0) a.result[b] = (int)total;
}

hipError_t launch_encode_seg(const BlockArgs &a, hipStream_t s) {
    if (a.nblocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(lz4_encode_seg_kernel, dim3(a.nblocks), dim3(kSThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace apelz4
