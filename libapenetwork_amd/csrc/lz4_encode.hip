// lz4_encode.hip -- MI355X (gfx950) batched LZ4 block encoder.
//
// Replaces the per-block work of APE_LZ4_compress_default (ref src/ape_lz4.c:
// 811-815 -> LZ4_compress_generic :530-755, byU16 / noDict).  The output is a
// valid LZ4 v1.7.1 block -- it obeys every parsing rule decompress_safe enforces
// (:1346-1366, :1375, :1444-1447): matches start at <= n-12, end at <= n-5, the
// last >= 5 bytes are literals -- but it is produced by a parallel parse, not
// by the reference's sequential skip-search, so the bytes differ.
//
// One 512-thread workgroup per block, everything in LDS (~153 KiB, 1 block/CU):
//   in[64 KiB]     the input block
//   E[4096]        hash table, u32 = (latest position of earlier rounds) << 16
//                  | (earliest position of the current round, 0xFFFF = none)
//   info[2048]     per position of the current round: the two verified candidate
//                  offsets, replaced by (offset | length << 16) once resolved
//   out[~64.3 KiB] the compressed block, flushed to HBM with 16-byte stores.
// The block is processed in rounds of kRound = 2048 positions:
//   A. every position hashes its 5 bytes (the reference's 64-bit hash,
//      :456-462) and atomicMin's itself into the low half of E[h];
//   B. every position reads E[h]: candidate T (latest earlier-round position)
//      and L (earliest same-round position, if before it);
//   C. atomicMax rolls E[h] to (latest position of this round) | 0xFFFF; each
//      position verifies both candidates' first 4 bytes (no length yet);
//   D. wave 0 runs the greedy parse: 64 walkers each own 32 positions, jump
//      match-to-match through a per-segment "has match" bitmask, measure the
//      match they land on (lazily; cached), and iterate to the fixpoint where
//      every walker's entry equals the chain position reaching it (identical to
//      a sequential greedy parse from position 0);
//   E. wave 0 prefix-sums sequence sizes and emits tokens/literals/offsets.
// Atomic min/max make the table state independent of thread timing, so the
// output is a deterministic function of the input.
#include "lz4_gpu_internal.h"

namespace apelz4 {

namespace {

constexpr int kThreads = 512;
constexpr int kRound = 2048;            // positions per round (4 per thread)
constexpr int kHashLog = 12;
constexpr int kHashSize = 1 << kHashLog;
constexpr int kSegE = 32;               // positions per walker segment
constexpr int kOutCap = kMaxBlock + kMaxBlock / 255 + 16;  // compressBound(64 KiB)
constexpr int kLongLit = 64;
constexpr uint32_t kLaneExt = 256;      // lane-serial match measuring budget (bytes)

struct __attribute__((aligned(16))) EncShared {
    uint8_t out[kOutCap + 32];
    uint8_t in[kMaxBlock + 32];
    uint32_t E[kHashSize];
    uint32_t info[kRound];
    uint32_t mask[kRound / kSegE];
    uint32_t dl_src[64], dl_dst[64], dl_len[64];  // deferred long literal runs
    uint32_t carry_p, carry_a, cursor;
    int overflow;
};

// bytes [sh, sh+4) of the little-endian 8-byte word hi:lo
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * sh));
}

__device__ __forceinline__ uint32_t ld32(const uint8_t *in, uint32_t pos) {
    const uint32_t *w = (const uint32_t *)(in + (pos & ~3u));
    return funnel(w[1], w[0], pos & 3u);
}

__device__ __forceinline__ uint32_t hash5(uint32_t lo32, uint32_t b4) {
    uint64_t seq = (uint64_t)lo32 | ((uint64_t)b4 << 32);
    return (uint32_t)((seq * 889523592379ULL) >> (40 - kHashLog)) & (kHashSize - 1);
}

// Length of the match at m with offset off (first 4 bytes known equal), measured
// up to min(lim, kLaneExt).  exact = false when the budget ran out first.
__device__ __forceinline__ uint32_t measure(const uint8_t *in, uint32_t m, uint32_t off,
                                            uint32_t lim, bool &exact) {
    const uint32_t cap = lim < kLaneExt ? lim : kLaneExt;
    uint32_t l = 4;
    while (l < cap) {
        const uint32_t x = ld32(in, m + l) ^ ld32(in, m - off + l);
        if (x) {
            l += __builtin_ctz(x) >> 3;
            exact = true;
            return l < lim ? l : lim;
        }
        l += 4;
    }
    exact = l >= lim;
    return l < lim ? l : lim;
}

__device__ __forceinline__ uint32_t ext_bytes(uint32_t v) {  // bytes after a 15 nibble
    return v >= 15 ? (v - 15) / 255 + 1 : 0;
}

__device__ __forceinline__ uint32_t seq_size(uint32_t lit, uint32_t len) {
    return 1 + ext_bytes(lit) + lit + 2 + ext_bytes(len - 4);
}

__device__ __forceinline__ uint32_t put_len(uint8_t *o, uint32_t v) {  // returns bytes written
    if (v < 15) return 0;
    v -= 15;
    uint32_t k = 0;
    for (; v >= 255; v -= 255) o[k++] = 255;
    o[k++] = (uint8_t)v;
    return k;
}

}  // namespace

#ifdef APE_LZ4_STATS
__device__ unsigned long long g_enc_stats[16];
hipError_t enc_stats_read(unsigned long long *out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_enc_stats), sizeof(g_enc_stats));
    if (e == hipSuccess && reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_enc_stats), z, sizeof(z));
    }
    return e;
}
#endif

__global__ void __launch_bounds__(kThreads)
lz4_encode_kernel(BlockArgs a) {
    __shared__ EncShared S;
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    const uint8_t *src =
        (const uint8_t *)(a.src ? a.src[b] : a.src_base + (size_t)b * a.src_stride);
    uint8_t *dst = (uint8_t *)(a.dst ? a.dst[b] : a.dst_base + (size_t)b * a.dst_stride);
    const int n = a.src_size[b];
    const int cap = a.dst_cap ? a.dst_cap[b] : (int)a.dst_stride;
    if (n < 0 || n > kMaxBlock) {
        if (tid == 0) a.result[b] = n < 0 ? 0 : kErange;
        return;
    }
    uint8_t *out = S.out + ((uintptr_t)dst & 15);

    STATS_DECL
    // ---- load the block (16-byte loads when aligned) and init the table ----
    if ((((uintptr_t)src) & 15) == 0) {
        const int n16 = n & ~15;
        for (int k = 16 * tid; k < n16; k += 16 * kThreads)
            *(uint4 *)(S.in + k) = *(const uint4 *)(src + k);
        for (int k = n16 + tid; k < n; k += kThreads) S.in[k] = src[k];
    } else {
        for (int k = tid; k < n; k += kThreads) S.in[k] = src[k];
    }
    if (tid < 32) S.in[n + tid] = 0;
    for (int i = tid; i < kHashSize; i += kThreads) S.E[i] = 0x0000FFFFu;
    if (tid == 0) {
        S.carry_p = 0;
        S.carry_a = 0;
        S.cursor = 0;
        S.overflow = 0;
    }
    __syncthreads();
    STAT(0);

    const uint32_t hash_end = n >= 5 ? (uint32_t)(n - 5) : 0;  // hash positions p <= n-5
    const bool any_hash = n >= 5;
    const uint32_t mstart_end = n >= 12 ? (uint32_t)(n - 12) : 0;  // match starts p <= n-12
    const uint32_t mlimit = n >= 5 ? (uint32_t)(n - 5) : 0;        // match ends <= n-5

    for (uint32_t R0 = 0; R0 < (uint32_t)n; R0 += kRound) {
        // ---- A: hash own 4 positions, atomicMin into the low half ----
        const uint32_t p0 = R0 + 4 * tid;
        uint32_t h[4], lo32[4];
        {
            const uint32_t *w = (const uint32_t *)(S.in + p0);
            uint32_t w0 = w[0], w1 = w[1];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                lo32[j] = funnel(w1, w0, (uint32_t)j);
                uint32_t b4 = (w1 >> (8 * j)) & 0xFFu;
                h[j] = hash5(lo32[j], b4);
            }
        }
        if (tid < kRound / kSegE) S.mask[tid] = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t p = p0 + j;
            if (any_hash && p <= hash_end) {
                uint32_t e = S.E[h[j]];
                atomicMin(&S.E[h[j]], (e & 0xFFFF0000u) | p);
            }
        }
        __syncthreads();
        STAT(1);
        // ---- B: read candidates ----
        uint32_t cT[4], cL[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t e = S.E[h[j]];
            cT[j] = e >> 16;
            cL[j] = e & 0xFFFFu;
        }
        __syncthreads();
        STAT(2);
        // ---- C: roll the table, verify candidates ----
        // (positions before the carried chain position can never start a sequence)
        const uint32_t carry_now = S.carry_p;
        uint32_t nib = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t p = p0 + j;
            if (any_hash && p <= hash_end) atomicMax(&S.E[h[j]], (p << 16) | 0xFFFFu);
            uint32_t cand = 0;
            if (p >= 1 && p <= mstart_end && n >= 13 && p >= carry_now) {
                const bool okT = cT[j] < p && ld32(S.in, cT[j]) == lo32[j];
                const bool okL = cL[j] < p && cL[j] != cT[j] && ld32(S.in, cL[j]) == lo32[j];
                cand = (okT ? p - cT[j] : 0u) | ((okL ? p - cL[j] : 0u) << 16);
                if (cand) nib |= 1u << j;
            }
            S.info[p - R0] = cand;
        }
        if (nib) atomicOr(&S.mask[(4 * tid) / kSegE], nib << ((4 * tid) % kSegE));
        __syncthreads();
        STAT(3);

        // ---- D/E: greedy parse and emission (wave 0); skipped when the carried
        // match covers the whole round ----
        if (wave == 0 && carry_now < R0 + kRound) {
            const uint32_t seg_lo = R0 + lane * kSegE;
            const uint32_t seg_hi = seg_lo + kSegE;
            const uint32_t carry = carry_now;
            const uint32_t mword = S.mask[lane];
            uint32_t rmask = 0;  // my positions whose info holds (offset | length << 16)
            // Entries are lower-bounded by max(seg_lo, carry) and, on the true chain,
            // equal the max of all earlier walkers' exits (chain positions only grow).
            const uint32_t floor_e = seg_lo > carry ? seg_lo : carry;
            uint32_t entry = floor_e;
            uint32_t ex = 0, last_end = 0;  // last_end: end of my last match, 0 = none
            int conf = 1;                   // walkers [0, conf) have exact entries
            int it_done = 0;
            (void)it_done;
            for (int it = 0; it < 4 * 64; it++) {
                it_done = it + 1;
                // Only walkers with an exact entry may pay for extending a long match;
                // a guessing walker that meets one stops with an unknown exit.
                const bool trusted = lane < conf;
                uint32_t p = entry;
                last_end = 0;
                bool active = p < seg_hi, need = false, unknown = false;
                uint32_t nm = 0, noff = 0, nlen = 0;
                while (__any(active)) {
                    if (active && !need) {
                        const uint32_t w = mword & (0xFFFFFFFFu << (p - seg_lo));
                        if (!w) {
                            p = seg_hi;
                            active = false;
                        } else {
                            const uint32_t m = seg_lo + __builtin_ctz(w);
                            const uint32_t bit = 1u << (m - seg_lo);
                            const uint32_t v = S.info[m - R0];
                            uint32_t len = 0;
                            if (rmask & bit) {
                                len = v >> 16;
                            } else {
                                // measure both candidates; keep the longer (then closer)
                                const uint32_t lim = mlimit - m;
                                const uint32_t oT = v & 0xFFFFu, oL = v >> 16;
                                bool xT = true, xL = true;
                                const uint32_t lT = oT ? measure(S.in, m, oT, lim, xT) : 0;
                                const uint32_t lL = oL ? measure(S.in, m, oL, lim, xL) : 0;
                                // an inexact length is >= kLaneExt > any exact one below it
                                const uint32_t kT = xT ? lT : 0x10000u, kL = xL ? lL : 0x10000u;
                                const bool pickL = oL && (!oT || kL > kT || (kL == kT && oL < oT));
                                const uint32_t off = pickL ? oL : oT;
                                const bool exact = pickL ? xL : xT;
                                len = pickL ? lL : lT;
                                if (exact) {
                                    S.info[m - R0] = off | (len << 16);
                                    rmask |= bit;
                                } else if (trusted) {
                                    need = true;
                                    nm = m;
                                    noff = off;
                                    nlen = len;
                                } else {
                                    unknown = true;
                                    active = false;
                                }
                            }
                            if (!need && !unknown) {
                                p = m + len;
                                last_end = p;
                                active = p < seg_hi;
                            }
                        }
                    }
                    // cooperative extension of long matches (whole wave, 256 B/step)
                    unsigned long long nmask = __ballot(need);
                    while (nmask) {
                        const int l = __ffsll((long long)nmask) - 1;
                        nmask &= nmask - 1;
                        const uint32_t m = __shfl(nm, l, 64), off = __shfl(noff, l, 64);
                        const uint32_t lim = mlimit - m;
                        uint32_t len = __shfl(nlen, l, 64);
                        for (;;) {
                            const uint32_t k = len + 4u * lane;
                            uint32_t x = 0;
                            const bool in_range = k < lim;
                            if (in_range) x = ld32(S.in, m + k) ^ ld32(S.in, m - off + k);
                            const unsigned long long bad = __ballot(in_range && x != 0);
                            if (bad) {
                                const int fl = __ffsll((long long)bad) - 1;
                                const uint32_t xf = __shfl(x, fl, 64);
                                len = len + 4u * fl + (__builtin_ctz(xf) >> 3);
                                break;
                            }
                            len += 256;
                            if (len >= lim) break;
                        }
                        if (len > lim) len = lim;
                        if (lane == l) {
                            S.info[m - R0] = off | (len << 16);
                            rmask |= 1u << (m - seg_lo);
                            p = m + len;
                            last_end = p;
                            active = p < seg_hi;
                            need = false;
                        }
                    }
                }
                ex = (entry < seg_hi) ? p : entry;
                const uint32_t kv = unknown ? 0u : ex;
                uint32_t mx = kv;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    uint32_t y = __shfl_up(mx, d, 64);
                    if (lane >= d) mx = mx > y ? mx : y;
                }
                uint32_t prev = __shfl_up(mx, 1, 64);
                if (lane == 0) prev = 0;
                const uint32_t ne = prev > floor_e ? prev : floor_e;
                const bool bad = (ne != entry) || unknown;
                entry = ne;
                const unsigned long long bm = __ballot(bad);
                if (!bm) break;
                conf = __ffsll((long long)bm);  // first bad walker's new entry is exact
            }
            STAT(4);
            STAT_ADD(9, it_done);
            // anchors: inclusive max-scan of last match ends
            uint32_t incl = last_end;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                uint32_t y = __shfl_up(incl, d, 64);
                if (lane >= d) incl = incl > y ? incl : y;
            }
            uint32_t excl = __shfl_up(incl, 1, 64);
            const uint32_t anchor_in = (lane == 0) ? S.carry_a : (excl > S.carry_a ? excl : S.carry_a);
            // sizes
            uint32_t bytes = 0;
            {
                uint32_t p = entry, an = anchor_in;
                while (p < seg_hi) {
                    const uint32_t w = mword & (0xFFFFFFFFu << (p - seg_lo));
                    if (!w) break;
                    const uint32_t m = seg_lo + __builtin_ctz(w);
                    const uint32_t len = S.info[m - R0] >> 16;
                    bytes += seq_size(m - an, len);
                    p = an = m + len;
                }
            }
            STAT(5);
            const uint32_t base = S.cursor;
            const uint32_t o0 = base + wave_excl_scan(bytes);
            const uint32_t total = __shfl(o0 + bytes, 63, 64);
            const bool ovf = total + 16 > (uint32_t)kOutCap;  // keep room for the last token
            S.dl_len[lane] = 0;
            if (!ovf) {
                uint32_t p = entry, an = anchor_in, o = o0;
                while (p < seg_hi) {
                    const uint32_t w = mword & (0xFFFFFFFFu << (p - seg_lo));
                    if (!w) break;
                    const uint32_t m = seg_lo + __builtin_ctz(w);
                    const uint32_t v = S.info[m - R0];
                    const uint32_t len = v >> 16, off = v & 0xFFFFu;
                    const uint32_t lit = m - an, ml = len - 4;
                    out[o++] = (uint8_t)(((lit < 15 ? lit : 15) << 4) | (ml < 15 ? ml : 15));
                    o += put_len(out + o, lit);
                    if (lit <= (uint32_t)kLongLit) {
                        for (uint32_t k = 0; k < lit; k++) out[o + k] = S.in[an + k];
                    } else {
                        S.dl_src[lane] = an;
                        S.dl_dst[lane] = o;
                        S.dl_len[lane] = lit;
                    }
                    o += lit;
                    out[o] = (uint8_t)off;
                    out[o + 1] = (uint8_t)(off >> 8);
                    o += 2;
                    o += put_len(out + o, ml);
                    p = an = m + len;
                }
            }
            STAT(6);
            // deferred long literal runs, cooperatively
            unsigned long long lm = __ballot(!ovf && S.dl_len[lane] != 0);
            while (lm) {
                const int l = __ffsll((long long)lm) - 1;
                lm &= lm - 1;
                const uint32_t s0 = S.dl_src[l], d0 = S.dl_dst[l], ln = S.dl_len[l];
                for (uint32_t k = lane; k < ln; k += 64) out[d0 + k] = S.in[s0 + k];
            }
            if (lane == 63) {
                S.carry_p = ex;
                const uint32_t la = incl > S.carry_a ? incl : S.carry_a;
                S.carry_a = la;
                S.cursor = total;
                if (ovf) S.overflow = 1;
            }
        }
        __syncthreads();
        STAT(7);
        STAT_ADD(10, 1);
        if (S.overflow) break;
    }

    // ---- last literals (:732-751) and flush ----
    if (S.overflow) {
        if (tid == 0) a.result[b] = 0;
        return;
    }
    const uint32_t an = S.carry_a;
    const uint32_t lit = (uint32_t)n - an;
    uint32_t o = S.cursor;
    const uint32_t hdr = 1 + ext_bytes(lit);
    if (tid == 0) {
        out[o] = (uint8_t)((lit < 15 ? lit : 15) << 4);
        put_len(out + o + 1, lit);
    }
    o += hdr;
    if (o + lit <= (uint32_t)kOutCap)
        for (uint32_t k = tid; k < lit; k += kThreads) out[o + k] = S.in[an + k];
    __syncthreads();
    const uint32_t total = o + lit;
    if (total > (uint32_t)kOutCap) {  // cannot happen (output <= compressBound)
        if (tid == 0) a.result[b] = 0;
        return;
    }
    if (tid == 0) a.result[b] = (total <= (uint32_t)cap) ? (int)total : 0;
    if (total <= (uint32_t)cap) {
        const uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15);
        const uint32_t hh = head < total ? head : total;
        if ((uint32_t)tid < hh) dst[tid] = out[tid];
        const uint32_t body = (total - hh) & ~15u;
        for (uint32_t k = hh + 16 * tid; k < hh + body; k += 16 * kThreads)
            *(uint4 *)(dst + k) = *(const uint4 *)(out + k);
        for (uint32_t k = hh + body + tid; k < total; k += kThreads) dst[k] = out[k];
    }
    STAT(8);
    STAT_ADD(11, 1);
    STATS_FLUSH(g_enc_stats);
}

hipError_t launch_encode(const BlockArgs &a, hipStream_t s) {
    if (a.nblocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(lz4_encode_kernel, dim3(a.nblocks), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace apelz4
