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
//   info[2048]     per position of the current round: best match (offset |
//                  length << 16), length 0xFFFF = "at least kEager, extend on use"
//   out[~64.3 KiB] the compressed block, flushed to HBM with 16-byte stores.
// The block is processed in rounds of kRound = 2048 positions:
//   A. every position hashes its 5 bytes (the reference's 64-bit hash,
//      :456-462) and atomicMin's itself into the low half of E[h];
//   B. every position reads E[h]: candidate T (latest earlier-round position)
//      and L (earliest same-round position, if before it);
//   C. atomicMax rolls E[h] to (latest position of this round) | 0xFFFF; each
//      position verifies both candidates and measures them up to kEager bytes
//      with independent 8-byte LDS compares (all loads in flight at once);
//   D. wave 0 runs the greedy parse: 64 walkers each own 32 positions, jump
//      match-to-match through a per-segment "has match" bitmask, and iterate to
//      the fixpoint where every walker's entry equals the chain position reaching
//      it (identical to a sequential greedy parse from position 0); DPP scans
//      give entries, anchors and output offsets;
//   E. all 8 waves emit: 8 threads per walker segment, one sequence each.
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
constexpr uint32_t kEager = 36;         // phase C measures matches up to this length
constexpr uint32_t kTrunc = 0xFFFFu;    // info length field: "at least kEager"

// `in` first: its dword reads (ld32/ld64) must be 4-byte aligned in LDS, or
// every one of them takes the unaligned-access stall.
struct __attribute__((aligned(16))) EncShared {
    uint8_t in[kMaxBlock + 64];
    uint8_t out[(kOutCap + 32 + 15) & ~15];
    uint32_t E[kHashSize];
    uint32_t info[kRound];
    uint32_t mask[kRound / kSegE];
    uint32_t seg_entry[64], seg_anchor[64], seg_out[64];  // walker results for emission
    uint32_t carry_p, carry_a, cursor;
    int overflow;
};
static_assert(offsetof(EncShared, in) % 16 == 0 && offsetof(EncShared, out) % 16 == 0 &&
                  offsetof(EncShared, E) % 16 == 0,
              "LDS arrays read by dwords / written by 16-byte stores must be aligned");

// bytes [sh, sh+4) of the little-endian 8-byte word hi:lo
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * sh));
}

__device__ __forceinline__ uint32_t ld32(const uint8_t *in, uint32_t pos) {
    const uint32_t *w = (const uint32_t *)(in + (pos & ~3u));
    return funnel(w[1], w[0], pos & 3u);
}

// 8 bytes at pos (three aligned LDS dwords)
__device__ __forceinline__ uint64_t ld64(const uint8_t *in, uint32_t pos) {
    const uint32_t *w = (const uint32_t *)(in + (pos & ~3u));
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], sh = pos & 3u;
    return (uint64_t)funnel(w1, w0, sh) | ((uint64_t)funnel(w2, w1, sh) << 32);
}

// Common-prefix length (from byte 4 on) of positions p and c, up to kEager;
// the four 8-byte compares are independent loads, so they are all in flight.
__device__ __forceinline__ uint32_t eager_len(const uint8_t *in, uint32_t p, uint32_t c) {
    uint64_t x[4];
#pragma unroll
    for (int s = 0; s < 4; s++) x[s] = ld64(in, p + 4 + 8 * s) ^ ld64(in, c + 4 + 8 * s);
    uint32_t len = kEager;
#pragma unroll
    for (int s = 3; s >= 0; s--)
        if (x[s]) len = 4 + 8 * s + (__builtin_ctzll(x[s]) >> 3);
    return len;
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
    if (tid < 64) S.in[n + tid] = 0;
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
            uint32_t best = 0;
            if (p >= 1 && p <= mstart_end && n >= 13 && p >= carry_now) {
                const bool okT = cT[j] < p && ld32(S.in, cT[j]) == lo32[j];
                const bool okL = cL[j] < p && cL[j] != cT[j] && ld32(S.in, cL[j]) == lo32[j];
                const uint32_t lim = mlimit - p;
                // measure both (independent loads), keep the longer, then the closer
                uint32_t lT = okT ? eager_len(S.in, p, cT[j]) : 0u;
                uint32_t lL = okL ? eager_len(S.in, p, cL[j]) : 0u;
                if (lT > lim) lT = lim;
                if (lL > lim) lL = lim;
                const bool pickL = okL && (!okT || lL > lT || (lL == lT && cL[j] > cT[j]));
                const uint32_t len = pickL ? lL : lT;
                if (okT || okL) {
                    const uint32_t off = p - (pickL ? cL[j] : cT[j]);
                    // a match that reached kEager before the limit may be longer
                    best = off | ((len >= kEager && len < lim ? kTrunc : len) << 16);
                    nib |= 1u << j;
                }
            }
            S.info[p - R0] = best;
        }
        if (nib) atomicOr(&S.mask[(4 * tid) / kSegE], nib << ((4 * tid) % kSegE));
        __syncthreads();
        STAT(3);

        // ---- D/E: greedy parse and emission (wave 0); skipped when the carried
        // match covers the whole round ----
        const bool parse_round = carry_now < R0 + kRound;
        if (wave == 0 && parse_round) {
            const uint32_t seg_lo = R0 + lane * kSegE;
            const uint32_t seg_hi = seg_lo + kSegE;
            const uint32_t carry = carry_now;
            const uint32_t mword = S.mask[lane];
            // Entries are lower-bounded by max(seg_lo, carry) and, on the true chain,
            // equal the max of all earlier walkers' exits (chain positions only grow).
            const uint32_t floor_e = seg_lo > carry ? seg_lo : carry;
            uint32_t entry = floor_e;
            uint32_t ex = 0, last_end = 0;  // last_end: end of my last match, 0 = none
            uint32_t first_m = 0, rest = 0; // first match start; bytes of my sequences
                                            // except the first one's literal run
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
                first_m = 0xFFFFFFFFu;
                rest = 0;
                bool active = p < seg_hi, need = false, unknown = false;
                uint32_t nm = 0, noff = 0;
                while (__any(active)) {
                    if (active && !need) {
                        const uint32_t w = mword & (0xFFFFFFFFu << (p - seg_lo));
                        if (!w) {
                            p = seg_hi;
                            active = false;
                        } else {
                            const uint32_t m = seg_lo + __builtin_ctz(w);
                            const uint32_t v = S.info[m - R0];
                            uint32_t len = v >> 16;
                            if (len == kTrunc) {
                                // lane-serial extension within a budget; only a
                                // longer match needs the cooperative path
                                const uint32_t off = v & 0xFFFFu, lim = mlimit - m;
                                uint32_t l = kEager;
                                bool exact = false;
                                while (l < lim && l < kLaneExt) {
                                    const uint64_t x = ld64(S.in, m + l) ^ ld64(S.in, m - off + l);
                                    if (x) { l += __builtin_ctzll(x) >> 3; exact = true; break; }
                                    l += 8;
                                }
                                if (l >= lim) { l = lim; exact = true; }
                                if (exact) {
                                    S.info[m - R0] = off | (l << 16);
                                    len = l;
                                } else if (trusted) {
                                    need = true;
                                    nm = m;
                                    noff = off;
                                } else {
                                    unknown = true;
                                    active = false;
                                }
                            }
                            if (!need && !unknown) {
                                if (first_m == 0xFFFFFFFFu) {
                                    first_m = m;
                                    rest += 3 + ext_bytes(len - 4);
                                } else {
                                    rest += seq_size(m - last_end, len);
                                }
                                p = m + len;
                                last_end = p;
                                active = p < seg_hi;
                            }
                        }
                    }
                    // cooperative extension of long matches (whole wave, 512 B/step)
                    unsigned long long nmask = __ballot(need);
                    while (nmask) {
                        const int l = __ffsll((long long)nmask) - 1;
                        nmask &= nmask - 1;
                        const uint32_t m = lane_val(nm, l), off = lane_val(noff, l);
                        const uint32_t lim = mlimit - m;
                        uint32_t len = kLaneExt;
                        for (;;) {
                            const uint32_t k = len + 8u * lane;
                            uint64_t x = 0;
                            const bool in_range = k < lim;
                            if (in_range) x = ld64(S.in, m + k) ^ ld64(S.in, m - off + k);
                            const unsigned long long bad = __ballot(in_range && x != 0);
                            if (bad) {
                                const int fl = __ffsll((long long)bad) - 1;
                                const uint32_t xlo = lane_val((uint32_t)x, fl);
                                const uint32_t xhi = lane_val((uint32_t)(x >> 32), fl);
                                const uint64_t xf = ((uint64_t)xhi << 32) | xlo;
                                len = len + 8u * fl + (__builtin_ctzll(xf) >> 3);
                                break;
                            }
                            len += 512;
                            if (len >= lim) break;
                        }
                        if (len > lim) len = lim;
                        if (lane == l) {
                            S.info[m - R0] = off | (len << 16);
                            if (first_m == 0xFFFFFFFFu) {
                                first_m = m;
                                rest += 3 + ext_bytes(len - 4);
                            } else {
                                rest += seq_size(m - last_end, len);
                            }
                            p = m + len;
                            last_end = p;
                            active = p < seg_hi;
                            need = false;
                        }
                    }
                }
                ex = (entry < seg_hi) ? p : entry;
                const uint32_t prev = wave_shr1(wave_incl_max(unknown ? 0u : ex), 0u);
                const uint32_t ne = prev > floor_e ? prev : floor_e;
                const bool bad = (ne != entry) || unknown;
                entry = ne;
                const unsigned long long bm = __ballot(bad);
                if (!bm) break;
                conf = __ffsll((long long)bm);  // first bad walker's new entry is exact
            }
            STAT(4);
            STAT_ADD(9, it_done);
            // anchors: max of earlier walkers' last match ends (and the carried one)
            const uint32_t carry_a = S.carry_a;
            const uint32_t incl = wave_incl_max(last_end);
            const uint32_t excl = wave_shr1(incl, 0u);
            const uint32_t anchor_in = excl > carry_a ? excl : carry_a;
            uint32_t bytes = rest;
            if (first_m != 0xFFFFFFFFu) {
                const uint32_t lit = first_m - anchor_in;
                bytes += ext_bytes(lit) + lit;
            }
            const uint32_t o0 = S.cursor + wave_excl_scan(bytes);
            const uint32_t total = lane_val(o0 + bytes, 63);
            S.seg_entry[lane] = entry;
            S.seg_anchor[lane] = anchor_in;
            S.seg_out[lane] = o0;
            STAT(5);
            if (lane == 63) {
                S.carry_p = ex;
                S.carry_a = incl > carry_a ? incl : carry_a;
                S.cursor = total;
                if (total + 16 > (uint32_t)kOutCap) S.overflow = 1;  // keep room for the tail
            }
        }
        __syncthreads();
        // ---- E: emission by all 8 waves: 8 threads per walker segment; thread k
        // writes the k-th sequence (a segment holds <= 8), the 8 share long literals
        if (parse_round && !S.overflow) {
            const int l = tid >> 3, k = tid & 7;
            const uint32_t seg_lo = R0 + l * kSegE, seg_hi = seg_lo + kSegE;
            const uint32_t mword = S.mask[l];
            uint32_t p = S.seg_entry[l], an = S.seg_anchor[l], o = S.seg_out[l];
            for (int i = 0; p < seg_hi; i++) {
                const uint32_t w = mword & (0xFFFFFFFFu << (p - seg_lo));
                if (!w) break;
                const uint32_t m = seg_lo + __builtin_ctz(w);
                const uint32_t v = S.info[m - R0];
                const uint32_t len = v >> 16, off = v & 0xFFFFu;
                const uint32_t lit = m - an, ml = len - 4;
                const uint32_t hdr = 1 + ext_bytes(lit);
                if (i == k) {
                    out[o] = (uint8_t)(((lit < 15 ? lit : 15) << 4) | (ml < 15 ? ml : 15));
                    put_len(out + o + 1, lit);
                    uint8_t *q = out + o + hdr + lit;
                    q[0] = (uint8_t)off;
                    q[1] = (uint8_t)(off >> 8);
                    put_len(q + 2, ml);
                    if (lit <= (uint32_t)kLongLit)
                        for (uint32_t t = 0; t < lit; t++) out[o + hdr + t] = S.in[an + t];
                }
                if (lit > (uint32_t)kLongLit)  // all 8 threads of the segment
                    for (uint32_t t = k; t < lit; t += 8) out[o + hdr + t] = S.in[an + t];
                o += hdr + lit + 2 + ext_bytes(ml);
                p = an = m + len;
            }
        }
        STAT(6);
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
