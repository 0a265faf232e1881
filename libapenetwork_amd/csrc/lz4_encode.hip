// lz4_encode.hip -- MI355X (gfx950) batched LZ4 block encoder.
//
// Replaces the per-block work of APE_LZ4_compress_default (ref src/ape_lz4.c:
// 811-815 -> LZ4_compress_generic :530-755, byU16 / noDict).  The output is a
// valid LZ4 v1.7.1 block -- it obeys every parsing rule decompress_safe enforces
// (:1346-1366, :1375, :1444-1447): matches start at <= n-12, end at <= n-5, the
// last >= 5 bytes are literals -- but it is produced by a round-parallel parse,
// not by the reference's sequential search, so the bytes differ.
//
// One wave (one 64-thread workgroup) per block.  A batch holds ~1M blocks, so
// the parallelism comes from many blocks in flight; per wave the LDS holds only
// the reference's own hash table (8192 x u16, 13-bit hash of 5 bytes, :449-462)
// plus a 1 KiB scratch, ~17 KiB, so 9 blocks share a CU.  The input stays in
// HBM/L2 and is read with unaligned 16-byte loads.
//
// The block is parsed in rounds of 64 positions starting at the parse position P:
//  1. every lane p = P + lane loads in[p-4, p+28), hashes in[p, p+5) and reads
//     two candidates: T = table[h] (positions walked in earlier rounds, as the
//     reference inserts them: :595-619, :680-706) and L = the earliest lane of
//     this round with the same low hash bits (found with an LDS atomicMin);
//     it loads in[c-4, c+28) for both, verifies 4 bytes, measures the match up
//     to 28 bytes and how far it extends backwards (up to 4 bytes);
//  2. the scalar unit walks the greedy chain through the round: jump to the
//     next lane with a match (ballot mask), extend it backwards into pending
//     literals (the reference's catch-up, :628-629) and, for a match that
//     reached 28 bytes, forwards with the whole wave (1 KiB per step);
//  3. walked positions and match_end - 2 (:680) go into the table;
//  4. member lanes emit their sequences straight to dst (prefix sums give the
//     offsets), a literal run longer than 32 bytes is copied by the whole wave.
// Last literals (:732-751) are copied by the whole wave with 16-byte moves.
#include <string.h>

#include "lz4_gpu_internal.h"

namespace apelz4 {

namespace {

#ifndef APE_LZ4_HLOG
#define APE_LZ4_HLOG 13
#endif
constexpr int kHLog = APE_LZ4_HLOG;
constexpr int kHSize = 1 << kHLog;
constexpr uint32_t kEagerLen = 28;   // match bytes measured before the walk
constexpr uint32_t kLongLit = 32;    // longer literal runs are copied by the wave
#ifndef APE_LZ4_ERING
#define APE_LZ4_ERING 8192
#endif
constexpr uint32_t kRingE = APE_LZ4_ERING;  // per-wave ring of recent input bytes
constexpr uint32_t kChunkE = 512;    // ring refill granule (8 bytes per lane)
constexpr uint32_t kAhead = 1024;    // keep the ring filled this far past P

struct __attribute__((aligned(16))) EncLds {
    uint16_t tab[kHSize];
    uint32_t scr[256];
    uint32_t ring[kRingE / 4];       // input byte x at ring byte (x mod kRingE)
};

// Compiler barrier for lane-to-lane communication through LDS inside one wave.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 32 bytes in[pos, pos+32) as 8 dwords; bytes outside [0, n) read as 0.
__device__ __forceinline__ void ld32b(const uint8_t *in, int n, int pos, uint32_t (&X)[8]) {
    if (pos >= 0 && pos + 32 <= n) {
        uint4 a, b;
        __builtin_memcpy(&a, in + pos, 16);
        __builtin_memcpy(&b, in + pos + 16, 16);
        X[0] = a.x; X[1] = a.y; X[2] = a.z; X[3] = a.w;
        X[4] = b.x; X[5] = b.y; X[6] = b.z; X[7] = b.w;
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++) X[k] = 0;
        for (int k = 0; k < 32; k++) {
            const int q = pos + k;
            if (q >= 0 && q < n) X[k >> 2] |= (uint32_t)in[q] << (8 * (k & 3));
        }
    }
}

// 8 input bytes at a (zero beyond n): one ring refill lane
__device__ __forceinline__ uint2 chunk_load(const uint8_t *in, uint32_t n, uint32_t a) {
    uint2 v = make_uint2(0u, 0u);
    if (a + 8u <= n) {
        __builtin_memcpy(&v, in + a, 8);
    } else {
        for (uint32_t t = 0; t < 8u && a + t < n; t++) {
            const uint32_t by = (uint32_t)in[a + t] << (8 * (t & 3));
            if (t < 4) v.x |= by; else v.y |= by;
        }
    }
    return v;
}

__device__ __forceinline__ void chunk_store(EncLds &S, uint32_t f, int lane, uint2 v) {
    *(uint2 *)&S.ring[((f + 8u * (uint32_t)lane) & (kRingE - 1)) >> 2] = v;
}

// Fill the ring with [f0, f0 + 2*kChunkE) now (after a jump past the filled bytes).
__device__ __forceinline__ void ring_fill(EncLds &S, const uint8_t *in, uint32_t n, uint32_t f0,
                                          int lane) {
    const uint2 a = chunk_load(in, n, f0 + 8u * (uint32_t)lane);
    const uint2 b = chunk_load(in, n, f0 + kChunkE + 8u * (uint32_t)lane);
    chunk_store(S, f0, lane, a);
    chunk_store(S, f0 + kChunkE, lane, b);
}

// 32 bytes at pos from the ring (pos >= fill - kRingE, or pos < 0 while the
// ring's tail is still zero)
__device__ __forceinline__ void ring32(const EncLds &S, int pos, uint32_t (&X)[8]) {
    const uint32_t sh = (uint32_t)pos & 3u;
    const int w0 = pos >> 2;
    uint32_t W[9];
#pragma unroll
    for (int k = 0; k < 9; k++) W[k] = S.ring[(uint32_t)(w0 + k) & (kRingE / 4 - 1)];
#pragma unroll
    for (int k = 0; k < 8; k++) X[k] = __builtin_amdgcn_alignbyte(W[k + 1], W[k], sh);
}

// 4 input bytes at x from the ring
__device__ __forceinline__ uint32_t ring4(const EncLds &S, uint32_t x) {
    const uint32_t w = x >> 2;
    return __builtin_amdgcn_alignbyte(S.ring[(w + 1) & (kRingE / 4 - 1)],
                                      S.ring[w & (kRingE / 4 - 1)], x & 3u);
}

// the reference's hash of the 5 bytes at p (x1 = in[p..p+3], b4 = in[p+4])
__device__ __forceinline__ uint32_t hash5(uint32_t x1, uint32_t b4) {
    const uint64_t seq = (uint64_t)x1 | ((uint64_t)(b4 & 0xFFu) << 32);
    return (uint32_t)((seq * 889523592379ULL) >> (40 - kHLog)) & (kHSize - 1);
}

// common length of X and Y from byte 4 (dword 1) on, up to kEagerLen
__device__ __forceinline__ uint32_t eager(const uint32_t (&X)[8], const uint32_t (&Y)[8]) {
    uint32_t len = kEagerLen;
#pragma unroll
    for (int k = 7; k >= 2; k--) {
        const uint32_t d = X[k] ^ Y[k];
        if (d) len = 4u * (uint32_t)(k - 1) + (__builtin_ctz(d) >> 3);
    }
    return len;
}

// bytes equal just before the match (in[p-1] == in[c-1], ...), 0..4
__device__ __forceinline__ uint32_t back4(uint32_t x0, uint32_t y0) {
    const uint32_t d = x0 ^ y0;
    return d ? (__builtin_clz(d) >> 3) : 4u;
}

__device__ __forceinline__ uint32_t ext_bytes(uint32_t v) {  // bytes after a 15 nibble
    return v >= 15 ? (v - 15) / 255 + 1 : 0;
}

// write the length extension of v (>= 15) at o, returns bytes written
__device__ __forceinline__ uint32_t put_len(uint8_t *o, uint32_t v) {
    if (v < 15) return 0;
    v -= 15;
    uint32_t k = 0;
    for (; v >= 255; v -= 255) o[k++] = 255;
    o[k++] = (uint8_t)v;
    return k;
}

// Copy in[a, a+len) to dst[o, o+len) with the whole wave (16 bytes per lane per step).
__device__ __forceinline__ void wave_copy(const uint8_t *in, uint8_t *dst, uint32_t a, uint32_t o,
                                          uint32_t len, int lane) {
    for (uint32_t k = 16u * (uint32_t)lane; k < len; k += 1024u) {
        if (k + 16u <= len) {
            uint4 v;
            __builtin_memcpy(&v, in + a + k, 16);
            __builtin_memcpy(dst + o + k, &v, 16);
        } else {
            for (uint32_t t = k; t < len; t++) dst[o + t] = in[a + t];
        }
    }
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

__global__ void __launch_bounds__(64)
lz4_encode_kernel(BlockArgs a) {
    __shared__ EncLds S;
    const int b = blockIdx.x;
    const int lane = threadIdx.x;

    const uint8_t *in =
        (const uint8_t *)(a.src ? a.src[b] : a.src_base + (size_t)b * a.src_stride);
    uint8_t *dst = (uint8_t *)(a.dst ? a.dst[b] : a.dst_base + (size_t)b * a.dst_stride);
    const int n = a.src_size[b];
    const uint32_t cap = (uint32_t)(a.dst_cap ? a.dst_cap[b] : (int)a.dst_stride);
    if (n < 0 || n > kMaxBlock) {
        if (lane == 0) a.result[b] = n < 0 ? 0 : kErange;
        return;
    }
    if ((int)cap < 0) {
        if (lane == 0) a.result[b] = 0;
        return;
    }

    STATS_DECL
    // table = 0 (the reference's memset state: position 0 for every hash)
    for (int i = lane; i < kHSize / 8; i += 64) ((uint4 *)S.tab)[i] = make_uint4(0, 0, 0, 0);
    for (int i = lane; i < 256; i += 64) S.scr[i] = 0xFFFFFFFFu;
    for (int i = lane; i < (int)(kRingE / 16); i += 64) ((uint4 *)S.ring)[i] = make_uint4(0, 0, 0, 0);
    wave_sync();
    uint32_t fill = 2 * kChunkE;  // ring holds input [rlo, fill)
    uint32_t rlo = 0;
    ring_fill(S, in, (uint32_t)n, 0u, lane);
    wave_sync();

    uint32_t anchor = 0;     // start of the pending literals (wave-uniform)
    uint32_t o = 0;          // output cursor
    bool overflow = false;
    const uint32_t un = (uint32_t)n;
    const uint32_t mstart = un >= 12 ? un - 12 : 0;   // matches start at <= n-12 (:585)
    const uint32_t mlimit = un >= 5 ? un - 5 : 0;     // and end at <= n-5 (:633)
    uint32_t P = 0;
    if (n < kMinLength) P = un;                       // :584 -> last literals only

    while (P < un && !overflow) {
        // ---- 0. input ring: refill after a jump, prefetch the next chunk ----
        if (fill < P + 96u) {
            fill = (P >= 64u ? P - 64u : 0u) & ~7u;
            rlo = fill;
            wave_sync();
            ring_fill(S, in, un, fill, lane);
            fill += 2 * kChunkE;
            wave_sync();
        }
        const bool refill = fill < P + kAhead;
        uint2 pre = make_uint2(0u, 0u);
        if (refill) pre = chunk_load(in, un, fill + 8u * (uint32_t)lane);

        // ---- 1. candidates for p = P + lane ----
        const uint32_t p = P + (uint32_t)lane;
        uint32_t X[8];
        ring32(S, (int)p - 4, X);
        const bool hashable = p + 5 <= un;
        const uint32_t h = hash5(X[1], X[2]);
        const uint32_t cT = S.tab[h];
        const uint32_t hs = h & 255u;
        if (hashable) atomicMin(&S.scr[hs], (uint32_t)lane);
        wave_sync();
        const uint32_t jL = hashable ? S.scr[hs] : 0xFFFFFFFFu;
        wave_sync();
        if (hashable) S.scr[hs] = 0xFFFFFFFFu;
        const bool can = p >= 1u && p <= mstart && n >= kMinLength;
        const uint32_t cL = P + jL;
        const bool tryT = can && cT < p;
        const bool tryL = can && jL < (uint32_t)lane && cL != cT;
        uint32_t Y[8], Z[8];
#pragma unroll
        for (int k = 0; k < 8; k++) { Y[k] = 0; Z[k] = 0; }
        if (tryT) {
            // recent candidates come from the ring, older ones from HBM / L2
            if (cT >= rlo + 4u) ring32(S, (int)cT - 4, Y);
            else ld32b(in, n, (int)cT - 4, Y);
        }
#pragma unroll
        for (int k = 0; k < 8; k++) Z[k] = (uint32_t)__shfl((int)X[k], (int)(jL & 63u), 64);
        if (!tryL) {
#pragma unroll
            for (int k = 0; k < 8; k++) Z[k] = 0;
        }
        const bool okT = tryT && Y[1] == X[1];
        const bool okL = tryL && Z[1] == X[1];
        const uint32_t lim = can ? mlimit - p : 0u;  // longest match allowed here
        uint32_t lT = okT ? eager(X, Y) : 0u, lL = okL ? eager(X, Z) : 0u;
        // a length that reached kEagerLen is "at least"; compare as such
        const bool pickL = okL && (!okT || lL > lT || (lL == lT && cL > cT));
        const uint32_t c = pickL ? cL : cT;
        uint32_t len = pickL ? lL : lT;
        const bool trunc = len >= kEagerLen && lim > kEagerLen;
        if (len > lim) len = lim;
        const uint32_t bk = umin(back4(X[0], pickL ? Z[0] : Y[0]), c);  // c - back >= 0
        const bool has = okT || okL;
        // lane info: len (16) | back (3) << 16 | trunc << 19
        const uint32_t info = len | (bk << 16) | (trunc ? (1u << 19) : 0u);
        const uint64_t Mm = __ballot(has);
        STAT(0);

        // ---- 2. greedy walk (scalar) ----
        const uint32_t anchor0 = anchor;
        uint32_t q = P;                 // walk position
        uint64_t walked = 0, members = 0;
        uint32_t m_back = 0, m_len = 0; // per member lane
        for (;;) {
            const uint32_t rel = q - P;
            if (rel >= 64u) break;
            const uint64_t w = Mm >> rel;
            if (w == 0) {
                walked |= ~0ull << rel;
                q = P + 64u;
                break;
            }
            const uint32_t j = rel + (uint32_t)__builtin_ctzll(w);
            walked |= (~0ull << rel) & (j == 63 ? ~0ull : ((2ull << j) - 1ull));
            const uint32_t v = lane_val(info, (int)j);
            const uint32_t m = P + j;
            uint32_t L = v & 0xFFFFu;
            if (v & (1u << 19)) {
                // forward extension with the whole wave, 1 KiB per step
                const uint32_t cm = lane_val(c, (int)j);
                const uint32_t lm = mlimit - m;
                for (;;) {
                    const uint32_t k = L + 16u * (uint32_t)lane;
                    uint32_t d = 0;
                    uint32_t at = 0;
                    if (k < lm) {
                        uint4 x, y;
                        if (m + k + 16u <= un) {
                            __builtin_memcpy(&x, in + m + k, 16);
                            __builtin_memcpy(&y, in + cm + k, 16);
                        } else {
                            uint32_t xb[4] = {0, 0, 0, 0}, yb[4] = {0, 0, 0, 0};
                            for (uint32_t t = 0; t < 16u && m + k + t < un; t++) {
                                xb[t >> 2] |= (uint32_t)in[m + k + t] << (8 * (t & 3));
                                yb[t >> 2] |= (uint32_t)in[cm + k + t] << (8 * (t & 3));
                            }
                            x = make_uint4(xb[0], xb[1], xb[2], xb[3]);
                            y = make_uint4(yb[0], yb[1], yb[2], yb[3]);
                        }
                        const uint32_t e0 = x.x ^ y.x, e1 = x.y ^ y.y, e2 = x.z ^ y.z, e3 = x.w ^ y.w;
                        if (e0) { d = 1; at = __builtin_ctz(e0) >> 3; }
                        else if (e1) { d = 1; at = 4 + (__builtin_ctz(e1) >> 3); }
                        else if (e2) { d = 1; at = 8 + (__builtin_ctz(e2) >> 3); }
                        else if (e3) { d = 1; at = 12 + (__builtin_ctz(e3) >> 3); }
                    }
                    const uint64_t bad = __ballot(d != 0 || k >= lm);
                    if (bad) {
                        const int fl = __builtin_ctzll(bad);
                        const uint32_t kk = L + 16u * (uint32_t)fl;
                        L = kk >= lm ? lm : kk + lane_val(at, fl);
                        break;
                    }
                    L += 1024u;
                }
                if (L > lm) L = lm;
                STAT_ADD(12, 1);
            }
            uint32_t bkj = (v >> 16) & 7u;
            if (bkj > m - anchor) bkj = m - anchor;   // never back into emitted bytes
            if (lane == (int)j) { m_back = bkj; m_len = L + bkj; }
            members |= 1ull << j;
            q = m + L;
            anchor = q;
        }
        STAT(1);

        // ---- 3. table updates: walked positions, then match_end - 2 ----
        if (((walked >> lane) & 1ull) && hashable) S.tab[h] = (uint16_t)p;
        const bool mem = (members >> lane) & 1ull;
        if (mem) {
            const uint32_t e2 = p + (m_len - m_back) - 2u;   // match end - 2
            if (e2 + 5u <= un) {
                uint32_t lo32 = 0, b4 = 0;
                if (e2 >= rlo && e2 + 8u <= fill) {
                    lo32 = ring4(S, e2);
                    b4 = ring4(S, e2 + 4u);
                } else if (e2 + 8u <= un) {
                    uint2 t;
                    __builtin_memcpy(&t, in + e2, 8);
                    lo32 = t.x;
                    b4 = t.y;
                } else {
                    for (uint32_t t = 0; t < 5u; t++) {
                        const uint32_t by = in[e2 + t];
                        if (t < 4) lo32 |= by << (8 * t); else b4 = by;
                    }
                }
                wave_sync();
                S.tab[hash5(lo32, b4)] = (uint16_t)e2;
            }
        }
        wave_sync();
        STAT(2);

        // ---- 4. emission ----
        if (members) {
            const uint32_t ms = p - m_back;              // match start after catch-up
            const uint32_t end = ms + m_len;
            const uint32_t an = umax(wave_shr1(wave_incl_max(mem ? end : 0u), 0u), anchor0);
            const uint32_t lit = mem ? ms - an : 0u;
            const uint32_t ml = m_len - kMinMatch;
            const uint32_t hdr = 1u + ext_bytes(lit);
            const uint32_t size = mem ? hdr + lit + 2u + ext_bytes(ml) : 0u;
            const uint32_t ex = wave_excl_scan(size);
            const uint32_t tot = lane_val(ex + size, 63);
            if ((uint64_t)o + tot > cap) {
                overflow = true;
                break;
            }
            const uint32_t ol = o + ex;
            if (mem) {
                uint8_t *d = dst + ol;
                d[0] = (uint8_t)(((lit < 15u ? lit : 15u) << 4) | (ml < 15u ? ml : 15u));
                put_len(d + 1, lit);
                if (lit <= kLongLit) {
                    // exact-length copy: whole dwords, then the tail bytes
                    uint32_t k = 0;
                    const bool inring = an >= rlo;   // an + lit <= fill always
                    for (; k + 4u <= lit; k += 4u) {
                        uint32_t v;
                        if (inring) v = ring4(S, an + k);
                        else __builtin_memcpy(&v, in + an + k, 4);
                        __builtin_memcpy(d + hdr + k, &v, 4);
                    }
                    if (k < lit) {
                        uint32_t v;
                        if (inring) v = ring4(S, an + k);
                        else { v = 0; for (uint32_t t = 0; k + t < lit; t++) v |= (uint32_t)in[an + k + t] << (8 * t); }
                        for (; k < lit; k++, v >>= 8) d[hdr + k] = (uint8_t)v;
                    }
                }
                const uint32_t off = p - c;
                uint8_t *t = d + hdr + lit;
                t[0] = (uint8_t)off;
                t[1] = (uint8_t)(off >> 8);
                put_len(t + 2, ml);
            }
            // long literal runs: the whole wave copies them, one member at a time
            uint64_t longm = __ballot(mem && lit > kLongLit);
            while (longm) {
                const int l = __builtin_ctzll(longm);
                longm &= longm - 1ull;
                const uint32_t la = lane_val(an, l), ll = lane_val(lit, l);
                const uint32_t lo = lane_val(ol + hdr, l);
                wave_copy(in, dst, la, lo, ll, lane);
            }
            o += tot;
            STAT_ADD(11, __popcll(members));
        }
        if (refill) {
            wave_sync();
            chunk_store(S, fill, lane, pre);
            fill += kChunkE;
            rlo = umax(rlo, fill - kRingE);
        }
        STAT(3);
        STAT_ADD(10, 1);
        P = q;
    }

    // ---- last literals (:732-751) ----
    if (!overflow) {
        const uint32_t lit = un - anchor;
        const uint32_t hdr = 1u + ext_bytes(lit);
        const uint32_t total = o + hdr + lit;
        if (total > cap) {
            overflow = true;
        } else {
            if (lane == 0) {
                dst[o] = (uint8_t)((lit < 15u ? lit : 15u) << 4);
                put_len(dst + o + 1, lit);
            }
            wave_copy(in, dst, anchor, o + hdr, lit, lane);
            o = total;
        }
    }
    if (lane == 0) a.result[b] = overflow ? 0 : (int)o;
    STAT(4);
    STAT_ADD(13, 1);
    STATS_FLUSH(g_enc_stats);
}

hipError_t launch_encode(const BlockArgs &a, hipStream_t s) {
    if (a.nblocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(lz4_encode_kernel, dim3(a.nblocks), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace apelz4
