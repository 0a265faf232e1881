// lz4_encode_v2.hip -- a second MI355X (gfx950) LZ4 block encoder pipeline, selected by
// APE_LZ4_ENCODER=v2 for A/B measurement against the product (lz4_encode.hip); same
// parse policy and output, fewer VALU instructions, but latency-bound.
//
// Replaces the per-block work of APE_LZ4_compress_default (ref src/ape_lz4.c:
// 811-815 -> LZ4_compress_generic :530-755, byU16 / noDict).  The output is a
// valid LZ4 v1.7.1 block -- it obeys every parsing rule decompress_safe enforces
// (:1346-1366, :1375, :1444-1447): matches start at <= n-12, end at <= n-5, the
// last >= 5 bytes are literals -- but it is produced by a chunk-parallel parse,
// not by the reference's sequential search, so the bytes differ.
//
// One 192-thread workgroup (three waves, one role each) per block; a batch holds
// ~1M blocks, so most of the parallelism comes from many blocks in flight (8 per
// CU).  Per block the LDS holds the reference's hash table (8192 x u16, 13-bit
// hash of 5 bytes, :449-462) and the hand-over records between the roles.  The
// block is cut into chunks of 64 positions, one per lane; the waves run in lock
// step, two workgroup barriers per step s:
//
//   PRODUCER (wave 1), four chunks in flight (every load is consumed one step after
//   it is issued, so no wait ever covers a load of the same step):
//     L(s+2)  load own bytes in[p-4, p+12) of every position p;
//     H(s+1)  hash in[p, p+5), T = table[h] (positions walked earlier and
//             match_end - 2, :595-619, :680-706), L = the earliest lane of the chunk
//             with the same low hash bits; issue the loads of both candidates'
//             bytes [c-4, c+12);
//     M(s)    verify 4 bytes of T and L, measure both to 12 bytes and up to 4 bytes
//             back (:623-627), keep the longer -> match record of chunk s.  Only
//             the lanes whose match reached 12 bytes ("saturated", ~13 of 64 on the
//             benchmark data) go on: they are compacted into a queue and each gets
//             64 / 32 / 16 more bytes measured by 4 / 2 / 1 lanes (16 bytes per
//             lane, issued now) -- the measurement work scales with the candidates
//             that need it, not with the 64 positions;
//     F(s-1)  finish those lengths (group minimum over the lanes of a candidate).
//   WALKER (wave 0), chunk s-2: the greedy chain on the scalar unit -- a position
//     with a match jumps past it, any other position is a literal -- with the
//     catch-up limit, the sequence sizes and the running output offset computed per
//     member in scalar registers (one v_readlane per member); a match the producer
//     left unfinished (> 76 bytes) is extended by the whole wave.  Second half: the
//     walked positions and match_end - 2 go into the table, the member records
//     {literal start, output offset} to the emitter.
//   EMITTER (wave 2), chunk s-3: every member lane writes its own sequence (token,
//     literal length bytes, literals, offset, match length bytes) at its output
//     offset; the last literals (:732-751) are copied with 16-byte moves.
#include "lz4_gpu_internal.h"
#include <stdlib.h>
#include <type_traits>

namespace apelz4 {

#ifdef APE_LZ4_STATS
__device__ unsigned long long g_enc_stats_v2[16];
hipError_t enc_stats_v2_read(unsigned long long *out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_enc_stats_v2), sizeof(g_enc_stats_v2));
    if (e == hipSuccess && reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_enc_stats_v2), z, sizeof(z));
    }
    return e;
}
#endif


namespace {

constexpr int kHLog = 13;
constexpr int kHSize = 1 << kHLog;
constexpr uint32_t kM1 = 12;   // stage 1 measures a match to this many bytes from p
constexpr int kNI = 4;         // info / hash rings, in chunks (s-3 .. s)
constexpr int kSmall = 128;    // smaller blocks take the byte-load path

// info.x: len (bits 0-15; bit 15 = TRUNC: measured to (len & 0x7FFF), longer) |
//         back (16-18) | HAS (19) | HASHABLE (20)
// info.y: offset (0-15) | hash (16-28)
constexpr uint32_t X_TRUNC = 0x8000u, X_HAS = 1u << 19, X_HASHABLE = 1u << 20;

struct __attribute__((aligned(16))) EncLds {
    uint16_t tab[kHSize];      // the reference's byU16 table (positions)
    uint2 info[kNI][64];       // producer -> walker, emitter: chunk k at [k % 4]
    uint16_t hr[kNI * 64];     // hash of position x at hr[x % 256] (walker: match_end - 2)
    uint32_t scr[64];          // producer: earliest lane per low 6 hash bits
    uint32_t sq[64];           // producer: stage-2 queue, owner lane | candidate << 8
    uint32_t q[2][64];         // walker -> emitter: a batch of up to 64 sequences, member i
                               // in lane i: {p | back << 16, len | offset << 16}
    uint32_t qcnt;             // its count (0 = none pending; the emitter resets it)
    uint2 wq[16];              // walker: one chunk's sequences (<= 16: matches are >= 4 long)
    uint32_t xw[2][40];        // producer: chunk k's bytes in[64k-4, 64k+140) at [k % 2] (from
                               // L(k) to M(k)): every lane's own window, the in-chunk
                               // candidate and the stage-2 own segments (36 dwords + pad)
};
static_assert(sizeof(EncLds) <= 20480, "8 blocks per CU: 8 x 20 KiB = the 160 KiB LDS");

// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt at their maxima = no wait).  The
// producer states its pipeline's waits explicitly: the compiler's own counter
// analysis treats a load whose consumer sits in a skipped branch as still in flight
// and then waits for every load before the register is reused.
template <int N>
__device__ __forceinline__ void vm_wait() {
    static_assert(N >= 0 && N < 16, "vmcnt");
    __builtin_amdgcn_s_waitcnt(N | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// v_ffbl_b32 / v_ffbh_u32: lowest set bit / leading zeros, 0xFFFFFFFF for 0 (inline
// asm so that the compiler does not turn the zero case into compare + select)
__device__ __forceinline__ uint32_t ffbl(uint32_t d) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(d));
    return r;
}
__device__ __forceinline__ uint32_t ffbh(uint32_t d) {
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(d));
    return r;
}

// Hash of the 5 bytes at p (x1 = in[p..p+3], b4 = in[p+4]) into kHLog bits.  The
// reference multiplies the 40-bit sequence by 889523592379 (:456-473), which needs
// quarter-rate 32-bit multiplies here; any hash gives a valid stream, so this one
// uses two 24 x 24-bit multiplies (v_mul_u32_u24) of bytes 0-2 and bytes 3-4.
// Same ratio on the App. C data (tools/enc_model.c: 3.1613 vs 3.1600).
__device__ __forceinline__ uint32_t hash5(uint32_t x1, uint32_t b4) {
    const uint32_t lo = x1 & 0xFFFFFFu, hi = (x1 >> 24) | ((b4 & 0xFFu) << 8);
    return ((uint32_t)__umul24(lo, 0x9E3779u) + (uint32_t)__umul24(hi, 0xC2B2AEu)) >> (32 - kHLog);
}

// e / 255 with one 24-bit multiply: 255 * 0x8081 = 2^23 + 127, so
// floor(e * 0x8081 / 2^23) = floor(e / 255) for e < 66060 (lengths here are < 65537)
__device__ __forceinline__ uint32_t div255(uint32_t e) {
    return (uint32_t)__umul24(e, 0x8081u) >> 23;
}
// bytes after a 15 nibble: v < 15 -> 0, else (v - 15) / 255 + 1 = (v + 240) / 255
__device__ __forceinline__ uint32_t ext_bytes(uint32_t v) { return div255(v + 240u); }
__host__ __device__ __forceinline__ uint32_t ext_s(uint32_t v) {   // scalar form
    return ((v + 240u) * 0x8081u) >> 23;
}

// write the length extension of v (>= 15) at o, at most `room` bytes (never past cap)
__device__ __forceinline__ void put_len(gu8 *o, uint32_t v) {
    if (v < 15) return;
    v -= 15;
    uint32_t k = 0;
    for (; v >= 255; v -= 255) o[k++] = 255;
    o[k] = (uint8_t)v;
}

// X = L shifted by d bytes (X byte i = L byte i + d, 0 outside L), |d| < 16, with
// compile-time register indices only.
__device__ __forceinline__ void shift16(const uint32_t (&L)[4], int d, uint32_t (&X)[4]) {
    uint32_t T[4];
#pragma unroll
    for (int k = 0; k < 4; k++) T[k] = L[k];
    const bool down = d >= 0;
    const int ad = down ? d : -d, w = ad >> 2;
    const uint32_t r = (uint32_t)ad & 3u;
#pragma unroll
    for (int bit = 2; bit >= 1; bit >>= 1) {
        if (w & bit) {
            if (down) {
#pragma unroll
                for (int k = 0; k < 4; k++) T[k] = (k + bit < 4) ? T[k + bit] : 0u;
            } else {
#pragma unroll
                for (int k = 3; k >= 0; k--) T[k] = (k - bit >= 0) ? T[k - bit] : 0u;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (down) X[k] = __builtin_amdgcn_alignbyte(k + 1 < 4 ? T[k + 1] : 0u, T[k], r);
        else X[k] = r ? __builtin_amdgcn_alignbyte(T[k], k >= 1 ? T[k - 1] : 0u, 4u - r) : T[k];
    }
}

// 16 bytes in[pos, pos+16) (bytes outside [0, n) read as 0).  fast (wave-uniform): every
// lane's window lies inside [0, n).  SMALL: byte loads.  Otherwise (n >= 16) one
// unaligned 16-byte load from the clamped window, fixed up with ALU only.
template <bool SMALL>
__device__ __forceinline__ void load16(gcu8 *in, int n, int pos, uint32_t (&X)[4], bool fast) {
    if (!SMALL && fast) {
        const uint4 a = gload16(in + (uint32_t)pos);
        X[0] = a.x; X[1] = a.y; X[2] = a.z; X[3] = a.w;
        return;
    }
    if (SMALL) {
#pragma unroll
        for (int k = 0; k < 4; k++) X[k] = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int q = pos + k;
            if (q >= 0 && q < n) X[k >> 2] |= (uint32_t)in[(uint32_t)q] << (8 * (k & 3));
        }
        return;
    }
    const int ca = pos < 0 ? 0 : (pos > n - 16 ? n - 16 : pos);
    const uint4 a = gload16(in + (uint32_t)ca);
    const uint32_t L[4] = {a.x, a.y, a.z, a.w};
    const int d = pos - ca;
    if (d == 0) {
#pragma unroll
        for (int k = 0; k < 4; k++) X[k] = L[k];
    } else {
        shift16(L, d < -15 ? -15 : (d > 15 ? 15 : d), X);
        if (d > 15 || d < -15) {
#pragma unroll
            for (int k = 0; k < 4; k++) X[k] = 0;
        }
    }
}

// Copy in[a, a+len) to dst[o, o+len) with the whole wave (16 bytes per lane per step).
__device__ __forceinline__ void wave_copy(gcu8 *in, gu8 *dst, uint32_t a, uint32_t o,
                                          uint32_t len, int lane) {
    for (uint32_t k = 16u * (uint32_t)lane; k < len; k += 1024u) {
        if (k + 16u <= len) {
            gstore16(dst + (o + k), gload16(in + (a + k)));
        } else {
            for (uint32_t t = k; t < len; t++) dst[o + t] = in[a + t];
        }
    }
}

struct Blk {
    gcu8 *in;
    gu8 *dst;
    int n;
    uint32_t un, cap, mstart, mlimit;
    int nch;                         // chunks of 64 positions
    int k0;                          // first chunk to encode: positions [0, 64 k0) are the
                                     // history prefix (withPrefix encode), only hashed
    uint32_t nr;                     // bytes to encode (n - 64 k0)
    bool noL;                        // acceleration > 1: no in-chunk candidate
};

// ---------------- producer ----------------
// Per chunk in flight (the step loop is unrolled by two, so no register set is ever
// copied): own bytes X of the chunk H and M work on; candidates and hash from H.
// Set k % 2 holds chunk k's own bytes X (L(k) .. M(k)), candidates, hash and their
// bytes Y / Z (H(k) .. M(k)), and the stage-2 bytes (M(k) .. F(k)); the two chunks
// in flight with one parity never overlap in the fields they use.
struct PSet {
    uint32_t X[4];                   // own bytes [p-4, p+12)
    uint32_t cT, cL, h;              // candidates (~0 = none), hash
    uint32_t Y[4], Z[4];             // T / L candidate bytes [c-4, c+12)
    uint32_t A[4], Bc[4];            // stage-2 bytes: own / candidate segment
    uint32_t q2;                     // stage-2 owner lane | seg << 8, ~0 = idle lane
    uint32_t lg;                     // stage-2 lanes per candidate, log2 (wave-uniform)
};

// L(k): the chunk's 144 bytes in[64k-4, 64k+140), one dword per lane 0..35 (bytes
// outside [0, n) read as 0) -- through the texture path once instead of as 64
// overlapping 16-byte windows plus the stage-2 own segments; x_spread makes the
// windows.  Outside SMALL one load instruction.
template <bool SMALL, bool FAST>
__device__ __forceinline__ void p_load(const Blk &B, int k, int lane, uint32_t &xd) {
    // lanes 36..63 repeat lane 35's address (no branch: the compiler's wait-count
    // model would take a skippable load as not issued and wait for older loads)
    const int w = (k < B.nch ? 64 * k : 0) - 4 + 4 * (lane < 36 ? lane : 35);
    if (SMALL) {
        uint32_t v = 0;
#pragma unroll
        for (int t = 0; t < 4; t++)
            if (w + t >= 0 && w + t < B.n) v |= (uint32_t)B.in[(uint32_t)(w + t)] << (8 * t);
        xd = v;
    } else if (FAST) {
        xd = gload4(B.in + (uint32_t)w);
    } else {   // clamped into [0, n - 4] (n >= 128 here), then shifted into place
        const int a = w < 0 ? 0 : (w > B.n - 4 ? B.n - 4 : w);
        const uint32_t v = gload4(B.in + (uint32_t)a);
        const int d = w - a;   // -4 .. 4
        const uint32_t dn = d > 0 ? (d < 4 ? v >> (8 * d) : 0u) : 0u;
        const uint32_t up = d < 0 ? (d > -4 ? v << (-8 * d) : 0u) : 0u;
        xd = d == 0 ? v : (d > 0 ? dn : up);
    }
}

// 16 bytes at byte offset j (0..128) of a chunk image: five dwords, four alignbytes
__device__ __forceinline__ void x_window(const uint32_t *img, uint32_t j, uint32_t (&X)[4]) {
    const uint32_t *w = img + (j >> 2);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    const uint32_t r = j & 3u;
    X[0] = __builtin_amdgcn_alignbyte(w1, w0, r);
    X[1] = __builtin_amdgcn_alignbyte(w2, w1, r);
    X[2] = __builtin_amdgcn_alignbyte(w3, w2, r);
    X[3] = __builtin_amdgcn_alignbyte(w4, w3, r);
}

// the loaded dwords of chunk k -> its LDS image -> every lane's own window in[p-4, p+12)
__device__ __forceinline__ void x_spread(EncLds &S, int k, int lane, uint32_t xd, uint32_t (&X)[4]) {
    uint32_t *img = S.xw[k & 1];
    if (lane < 36) img[lane] = xd;
    wave_sync();
    x_window(img, (uint32_t)lane, X);
}

// H(k): hash, table + in-chunk candidates, hash ring, candidate loads
template <bool SMALL, bool FAST>
__device__ __forceinline__ void p_lookup(EncLds &S, const Blk &B, int k, int lane, PSet &C) {
    const uint32_t (&X)[4] = C.X;
    const uint32_t p = 64u * (uint32_t)k + (uint32_t)lane;
    const bool live = k < B.nch;
    const bool hashable = live && p + 5u <= B.un;
    const uint32_t h = hash5(X[1], X[2]);
    const uint32_t cT = S.tab[h];
    S.hr[p & (kNI * 64 - 1)] = (uint16_t)h;
    uint32_t jL = 0xFFFFFFFFu;
    if (!B.noL) {   // wave-uniform
        const uint32_t hs = h & 63u;
        if (hashable) atomicMin(&S.scr[hs], (uint32_t)lane);
        wave_sync();
        jL = hashable ? S.scr[hs] : 0xFFFFFFFFu;
        wave_sync();
        if (hashable) S.scr[hs] = 0xFFFFFFFFu;
    }
    // Candidates below position 4 are skipped: their 4 bytes of backward context would
    // start before the block (and a candidate is always < p <= n - 12, so its 16 bytes
    // lie inside the block).
    // only positions that may start a match (p <= n - 12, :585) keep candidates, so a
    // candidate c < p has its 16 bytes [c - 4, c + 12) inside the block
    const bool can = hashable && p >= 1u && p <= B.mstart && B.n >= kMinLength;
    const uint32_t cL = 64u * (uint32_t)k + jL;
    const bool okT = can && cT < p && cT >= 4u;
    const bool okL = can && jL < (uint32_t)lane && cL >= 4u && cL != cT;
    C.h = h;
    C.cT = okT ? cT : 0xFFFFFFFFu;
    C.cL = okL ? cL : 0xFFFFFFFFu;
    // dummy loads of idle lanes read the block start (n >= 16 outside SMALL); the
    // in-chunk candidate's bytes come from the chunk image in M
    load16<SMALL>(B.in, B.n, okT ? (int)cT - 4 : 0, C.Y, !SMALL);
}

// first differing byte of A vs B over 4 dwords (0..15), 0x1FFFFFFF if all 16 equal:
// ffbl per dword, the dword's bit offset ORed in (a full-rate or instead of an add),
// then a min over the four
__device__ __forceinline__ uint32_t first_diff16(const uint32_t (&A)[4], const uint32_t (&B)[4]) {
    const uint32_t m0 = ffbl(A[0] ^ B[0]), m1 = ffbl(A[1] ^ B[1]) | 32u;
    const uint32_t m2 = ffbl(A[2] ^ B[2]) | 64u, m3 = ffbl(A[3] ^ B[3]) | 96u;
    return umin(umin(m0, m1), umin(m2, m3)) >> 3;
}

// M(k): verify + measure both candidates to 12 bytes, back-extension, pick -> info;
// queue the saturated lanes and issue their stage-2 loads.
template <bool SMALL, bool FAST>
__device__ __forceinline__ void p_measure(EncLds &S, const Blk &B, int k, int lane, PSet &C) {
    const uint32_t (&X)[4] = C.X;
    const PSet &Sh = C;
    // in-chunk candidate bytes [cL-4, cL+12) = image bytes [cL - 64k, +16)
    x_window(S.xw[k & 1], C.cL != 0xFFFFFFFFu ? C.cL & 63u : 0u, C.Z);
    const uint32_t p = 64u * (uint32_t)k + (uint32_t)lane;
    const bool live = k < B.nch;
    const bool can = live && p >= 1u && p <= B.mstart && B.n >= kMinLength;
    const uint32_t lim = can ? B.mlimit - p : 0u;
    // bytes 4..11 from p: dwords 2, 3 of the own / candidate windows (window = c - 4)
    const bool vT = can && C.cT != 0xFFFFFFFFu && Sh.Y[1] == X[1];
    const bool vL = can && C.cL != 0xFFFFFFFFu && Sh.Z[1] == X[1];
    const uint32_t bT = umin(umin(ffbl(X[2] ^ Sh.Y[2]), ffbl(X[3] ^ Sh.Y[3]) | 32u) >> 3, 8u);
    const uint32_t bL = umin(umin(ffbl(X[2] ^ Sh.Z[2]), ffbl(X[3] ^ Sh.Z[3]) | 32u) >> 3, 8u);
    // L (the closer one) wins when longer, or equally long below 12
    const bool pickL = vL && (!vT || bL > bT || (bL == bT && bT < 8u));
    const uint32_t c = pickL ? C.cL : C.cT;
    const bool has = vT || vL;
    uint32_t len = 4u + (pickL ? bL : bT);
    const uint32_t w0 = pickL ? Sh.Z[0] : Sh.Y[0];
    const uint32_t back = umin(ffbh(X[0] ^ w0) >> 3, 4u);   // in[p-1..p-4] == in[c-1..c-4]
    len = umin(len, lim);
    const bool sat = has && len == kM1 && lim > kM1;
    const bool hashable = live && p + 5u <= B.un;
    S.info[k % kNI][lane] =
        make_uint2((has ? len : 0u) | (back << 16) | (has ? X_HAS : 0u) | (hashable ? X_HASHABLE : 0u),
                   (has ? p - c : 0u) | (C.h << 16));
    // ---- stage 2: compact the saturated lanes, 64 / nsat lanes (4, 2 or 1) each ----
    const uint64_t sm = wave_ballot(sat);
    const uint32_t nsat = (uint32_t)__popcll(sm);
    const uint32_t idx = __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
    if (sat) S.sq[idx] = (uint32_t)lane | (c << 8);
    wave_sync();
    const uint32_t lg = nsat <= 16u ? 2u : (nsat <= 32u ? 1u : 0u);
    const uint32_t slot = (uint32_t)lane >> lg, seg = (uint32_t)lane & ((1u << lg) - 1u);
    const bool act = slot < nsat;
    const uint32_t e = S.sq[act ? slot : 0u];
    const uint32_t j = e & 63u, cc = e >> 8;
    const uint32_t P = 64u * (uint32_t)k;
    C.q2 = act ? (j | (seg << 8)) : 0xFFFFFFFFu;
    C.lg = lg;
    // own segment p_j + 12 + 16 seg from the chunk image (byte j + 16 + 16 seg <= 127),
    // candidate segment c + 12 + 16 seg (16 bytes each); idle lanes load the block start
    x_window(S.xw[k & 1], act ? j + kM1 + 4u + 16u * seg : 0u, C.A);
    (void)P;
    const int pc = act ? (int)(cc + kM1 + 16u * seg) : 0;
    load16<SMALL>(B.in, B.n, pc, C.Bc, FAST);
}

// F(k): finish the saturated lengths of chunk k (loads issued one step earlier)
__device__ __forceinline__ void p_finish(EncLds &S, const Blk &B, int k, int lane, const PSet &Sh) {
    const uint32_t lg = __builtin_amdgcn_readfirstlane(Sh.lg);
    if (k < 0) return;
    uint32_t v = umin(first_diff16(Sh.A, Sh.Bc) + 16u * ((Sh.q2 >> 8) & 3u), 0xFFFFu);
    // minimum over the 1 << lg lanes of a candidate (quad_perm swaps), to its first lane
    if (lg >= 1u) v = umin(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false));
    if (lg >= 2u) v = umin(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false));
    const uint32_t span = 16u << lg;
    if (Sh.q2 < 64u) {   // the candidate's first lane (seg 0)
        const uint32_t j = Sh.q2;
        const uint32_t lim = B.mlimit - (64u * (uint32_t)k + j);
        const bool full = v >= 0xFFFFu;                  // equal over the whole span
        uint32_t len = kM1 + (full ? span : v);
        const bool trunc = full && lim > kM1 + span;
        len = umin(len, lim);
        *(uint16_t *)&S.info[k % kNI][j].x = (uint16_t)(len | (trunc ? X_TRUNC : 0u));
    }
}

// ---------------- walker ----------------
// forward extension of the match at m (candidate cm) from L bytes on, with the whole
// wave, 1 KiB per step; returns the full length (<= mlimit - m)
__device__ __forceinline__ uint32_t extend_match(const Blk &B, uint32_t m, uint32_t cm, uint32_t L,
                                                 int lane) {
    const uint32_t lm = B.mlimit - m;
    for (;;) {
        const uint32_t kk = L + 16u * (uint32_t)lane;
        uint32_t d = 0, at = 0;
        if (kk < lm) {
            uint32_t xb[4] = {0, 0, 0, 0}, yb[4] = {0, 0, 0, 0};
            if (m + kk + 16u <= B.un) {
                const uint4 x = gload16(B.in + (m + kk)), y = gload16(B.in + (cm + kk));
                xb[0] = x.x; xb[1] = x.y; xb[2] = x.z; xb[3] = x.w;
                yb[0] = y.x; yb[1] = y.y; yb[2] = y.z; yb[3] = y.w;
            } else {
#pragma unroll
                for (uint32_t t = 0; t < 16u; t++) {
                    if (m + kk + t < B.un) {
                        xb[t >> 2] |= (uint32_t)B.in[m + kk + t] << (8 * (t & 3));
                        yb[t >> 2] |= (uint32_t)B.in[cm + kk + t] << (8 * (t & 3));
                    }
                }
            }
#pragma unroll
            for (int t = 3; t >= 0; t--) {
                const uint32_t e = xb[t] ^ yb[t];
                if (e) { d = 1; at = 4u * (uint32_t)t + (__builtin_ctz(e) >> 3); }
            }
        }
        const uint64_t bad = wave_ballot(d != 0 || kk >= lm);
        if (bad) {
            const int fl = __builtin_ctzll(bad);
            const uint32_t k2 = L + 16u * (uint32_t)fl;
            L = k2 >= lm ? lm : k2 + lane_val(at, fl);
            break;
        }
        L += 1024u;
    }
    return L > lm ? lm : L;
}

struct Walk {
    uint32_t q;          // walk position (next position to search)
    uint32_t a;          // anchor: start of the pending literals
    uint32_t qn;         // sequences in the queue registers
    uint32_t Q0, Q1;     // per lane: queued sequence {p | back << 16, len | offset << 16}
    uint32_t nx;         // (diagnostic) walker extensions
};
struct WalkOut {
    bool walked;         // this lane's position was walked (table insert)
    bool member;         // a match starts here
    uint32_t x, y;       // info of the lane (final lengths)
    uint64_t M;          // match starts of the chunk
    uint32_t rel0;       // first position the walk searched (64: none)
};

// hand the queued sequences to the emitter (it consumes them in the next step)
__device__ __forceinline__ void walk_flush(EncLds &S, int lane, Walk &W) {
    S.q[0][lane] = W.Q0;
    S.q[1][lane] = W.Q1;
    if (lane == 0) S.qcnt = W.qn;
    W.qn = 0;
}

// per-lane bit of a wave-uniform 64-bit mask: v_cndmask with the mask as the condition
__device__ __forceinline__ bool lane_bit(uint64_t m) {
    uint32_t r;
    asm("v_cndmask_b32 %0, 0, 1, %1" : "=v"(r) : "s"(m));
    return r != 0u;
}

// First half: the greedy chain (:591-627) over chunk k.  Only the chain itself runs on
// the scalar unit -- next match start, one v_readlane of its length, jump past it; the
// rest follows lane-parallel from the member set: one max-scan of the members' ends
// gives every member its catch-up limit (<= 4 bytes back, never into the previous
// match, :623-627) and every lane whether a match covers it; the members' sequences
// then move to the next free lanes of the queue registers through a small LDS buffer,
// so the emitter later writes 64 sequences per pass.
__device__ __forceinline__ void walk_chain(const Blk &B, int k, int lane, Walk &W, WalkOut &O,
                                           const uint2 iv) {
    const uint32_t P = 64u * (uint32_t)k;
    O.x = iv.x;
    O.y = iv.y;
    O.walked = O.member = false;
    O.M = 0;
    O.rel0 = 64u;
    if (W.q >= P + 64u) return;               // a match from an earlier chunk covers it
    const uint64_t Hm = wave_ballot((iv.x & X_HAS) != 0u);
    const uint32_t rel0 = W.q - P;
    uint32_t rel = rel0;
    uint64_t M = 0;
    for (;;) {
        const uint64_t w = Hm >> rel;
        if (w == 0) { rel = 64u; break; }
        const uint32_t j = rel + (uint32_t)__builtin_ctzll(w);
        uint32_t len = lane_val(O.x, (int)j) & 0xFFFFu;
        if (len & X_TRUNC) {                  // unfinished by the producer (rare)
            W.nx++;
            const uint32_t m = P + j;
            len = extend_match(B, m, m - (lane_val(O.y, (int)j) & 0xFFFFu), len & 0x7FFFu, lane);
            if ((uint32_t)lane == j) O.x = (O.x & 0xFFFF0000u) | len;
        }
        M |= 1ull << j;
        rel = j + len;
        if (rel >= 64u) break;
    }
    W.q = P + rel;
    O.M = M;
    O.rel0 = rel0;
}

// Second half, before the inserts: the member set's lane-parallel consequences.
__device__ __forceinline__ void walk_post(EncLds &S, int k, int lane, Walk &W, WalkOut &O) {
    const uint32_t P = 64u * (uint32_t)k;
    if (O.rel0 >= 64u) return;
    const uint64_t M = O.M;
    const uint32_t p = P + (uint32_t)lane;
    const bool mem = lane_bit(M);
    const uint32_t len = O.x & 0xFFFFu;
    const uint32_t im = wave_incl_max(mem ? p + len : 0u);   // latest match end up to here
    const uint32_t prev = umax(wave_shr1(im, 0u), W.a);      // ... before this lane
    O.member = mem;
    O.walked = (uint32_t)lane >= O.rel0 && prev <= p;         // not inside a match
    W.a = umax(W.a, lane_val(im, 63));
    if (!M) return;
    // the members' sequences, in order, to queue lanes qn, qn + 1, ...
    const uint32_t back = umin((O.x >> 16) & 7u, p - prev);
    const uint32_t nm = (uint32_t)__popcll(M);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
    if (mem) S.wq[rank] = make_uint2(p | (back << 16), len | (O.y << 16));
    wave_sync();
    const uint32_t d = (uint32_t)lane - W.qn;                // lanes qn .. qn + nm - 1
    const uint2 e = S.wq[d < nm ? d : 0u];
    if (d < nm) { W.Q0 = e.x; W.Q1 = e.y; }
    if (W.qn + nm >= 64u) {                                   // a full batch: hand it over
        const uint32_t done = 64u - W.qn;                     // members that fit it
        W.qn = 64u;
        walk_flush(S, lane, W);
        const uint32_t rest = nm - done;                      // the others start the next
        const uint2 f = S.wq[(uint32_t)lane < rest ? done + (uint32_t)lane : 0u];
        if ((uint32_t)lane < rest) { W.Q0 = f.x; W.Q1 = f.y; }
        W.qn = rest;
    } else {
        W.qn += nm;
    }
}

// Second half: walked positions and match_end - 2 (:680) into the table (never
// overlapping the producer's lookups, which happen in first halves).
__device__ __forceinline__ void walk_publish(EncLds &S, const Blk &B, int k, int lane,
                                             const WalkOut &O) {
    const uint32_t p = 64u * (uint32_t)k + (uint32_t)lane;
    if (O.walked && (O.x & X_HASHABLE) && p < B.un) S.tab[O.y >> 16] = (uint16_t)p;
    // one wave's LDS operations complete in order: the walked-position inserts above
    // land before these (compiler barrier only)
    __builtin_amdgcn_sched_barrier(0);
    const bool mem = O.member;
    const uint32_t e2 = p + (O.x & 0xFFFFu) - 2u;
    bool ok = mem && e2 + 5u <= B.un;
    // the hash ring holds chunks k .. k+3 (positions [64k, 64k + 256)); a match reaching
    // past it (rare) hashes its bytes itself
    const bool inring = e2 < 64u * (uint32_t)k + (uint32_t)(kNI * 64);
    if (wave_any(ok && !inring)) {
        if (ok && !inring) {
            const uint32_t at = umin(e2, B.un - 8u);
            const uint2 v = gload8(B.in + at);
            const uint32_t sh = e2 - at;
            S.tab[hash5(__builtin_amdgcn_alignbyte(v.y, v.x, sh), v.y >> (8u * sh))] = (uint16_t)e2;
        }
        ok = ok && inring;
    }
    if (ok) S.tab[S.hr[e2 & (kNI * 64 - 1)]] = (uint16_t)e2;
}

// ---------------- emitter ----------------
// A batch of up to 64 sequences (member i in lane i, in block order) per pass: literal
// starts from the previous member's end (one lane shift), sizes and output offsets
// from one wave scan, then every lane writes its own sequence (token, literal length
// bytes, literals, offset, match length bytes) at its offset.  Sequences that would end
// past the capacity are not written (the block then fails: result 0).  Two phases, one
// per half step, so the literal load's latency is covered by the barrier between them.
struct Em {
    uint32_t o, ob, oo, lit, ml, off, a;
    bool ok;
    int cnt;
    uint32_t Lw[4];
};

// phase 1; ca / co: the running anchor and output offset (wave-uniform, updated)
template <bool SMALL>
__device__ __forceinline__ void emit_load(EncLds &S, const Blk &B, int lane, Em &E, uint32_t &ca,
                                          uint32_t &co) {
    E.cnt = (int)__builtin_amdgcn_readfirstlane(S.qcnt);
    if (E.cnt == 0) return;
    const bool valid = lane < E.cnt;
    const uint32_t q0 = S.q[0][lane], q1 = S.q[1][lane];
    const uint32_t p = q0 & 0xFFFFu, back = q0 >> 16, len = q1 & 0xFFFFu;
    E.off = q1 >> 16;
    const uint32_t end = p + len;
    E.a = wave_shr1(end, ca);                     // previous member's end
    E.lit = p - back - E.a;
    E.ml = len + back - kMinMatch;
    const uint32_t el = ext_bytes(E.lit), em = ext_bytes(E.ml);
    const uint32_t size = valid ? 3u + E.lit + el + em : 0u;
    const uint32_t incl = wave_incl_sum(size);
    E.o = co + incl - size;
    E.ob = E.o + 1u + el;                         // first literal byte
    E.oo = E.ob + E.lit;                          // offset
    E.ok = valid && E.o + size <= B.cap;
    if (lane == 0) S.qcnt = 0;
    // up to 16 literals come from one 16-byte load of in[a, a+16) (a + 16 <= n: a
    // literal run ends at a match start <= n - 12 ... the generic path near the end)
    ca = lane_val(end, E.cnt - 1);
    co += lane_val(incl, 63);
    const bool sl = E.ok && E.lit <= 16u;
    const uint32_t amax = lane_val(E.a, E.cnt - 1);   // literal starts increase with the lane
    load16<SMALL>(B.in, B.n, sl ? (int)E.a : 0, E.Lw, !SMALL && amax + 16u <= B.un);
}

// phase 2: the stores
__device__ __forceinline__ void emit_store(const Blk &B, int lane, const Em &E) {
    if (E.cnt == 0) return;
    // the literal load, once: inside the branchy store sequence below the compiler would
    // otherwise wait for vmcnt(0) -- every earlier store included -- before each use
    vm_wait<0>();
    gu8 *dst = B.dst;
    const bool ok = E.ok;
    if (ok) dst[E.o] = (uint8_t)((umin(E.lit, 15u) << 4) | umin(E.ml, 15u));
    if (wave_any(ok && E.lit >= 15u)) {
        if (ok) put_len(dst + E.o + 1u, E.lit);
    }
    for (uint64_t lm = wave_ballot(ok && E.lit > 16u); lm; lm &= lm - 1) {   // long runs:
        const int j = __builtin_ctzll(lm);                                     // the whole wave
        wave_copy(B.in, dst, lane_val(E.a, j), lane_val(E.ob, j), lane_val(E.lit, j), lane);
    }
    const uint32_t nl = (ok && E.lit <= 16u) ? E.lit : 0u;
#pragma unroll
    for (uint32_t t = 0; t < 16u; t++) {
        if (!wave_any(t < nl)) break;
        if (t < nl) dst[E.ob + t] = (uint8_t)(E.Lw[t >> 2] >> (8u * (t & 3u)));
    }
    if (ok) {
        dst[E.oo] = (uint8_t)E.off;
        dst[E.oo + 1u] = (uint8_t)(E.off >> 8);
    }
    if (wave_any(ok && E.ml >= 15u)) {
        if (ok) put_len(dst + E.oo + 2u, E.ml);
    }
}

// ---------------- history prefix (withPrefix encode) ----------------
// Positions [0, 64 k0) precede the block in memory (the previous <= 64 KiB of the
// stream, as compress_fast_continue sees it, ref src/ape_lz4.c:1160-1220).  The
// producer wave hashes every third of them into the table, as loadDict does
// (:1127-1130; catch-up recovers the bytes a skipped start loses), oldest first (one
// wave: its LDS writes land in order, so the newest position wins deterministically).
__device__ __forceinline__ void prefix_history(EncLds &S, const Blk &B, int lane) {
    const uint32_t D = 64u * (uint32_t)B.k0;
    constexpr int kU = 8;   // loads in flight per trip (the loop is latency bound)
    for (uint32_t v0 = 0; v0 < D; v0 += 192u * kU) {
        uint2 x[kU];
        bool ok[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const uint32_t v = v0 + 192u * u + 3u * (uint32_t)lane;
            ok[u] = v < D && v + 8u <= B.un;   // (the last few of a tiny block stay out)
            x[u] = gload8(B.in + (ok[u] ? v : 0u));
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const uint32_t v = v0 + 192u * u + 3u * (uint32_t)lane;
            if (ok[u]) S.tab[hash5(x[u].x, x[u].y)] = (uint16_t)v;
        }
    }
}

// ---------------- block ----------------
//   step s, first half : producer F(s-1) M(s) H(s+1) L(s+2) | walker walks s-2 |
//                        emitter writes s-3
//   step s, second half: walker inserts s-2 into the table and publishes it
// Table inserts (second half) never overlap the producer's lookups (first half); the
// info ring slots are s (M), s-1 (F), s-2 (walker), s-3 (emitter): all distinct.
template <bool SMALL>
__device__ __forceinline__ void encode_block(EncLds &S, const Blk &B, int wave, int lane,
                                             int *result) {
    STATS_DECL
    const int k0 = B.k0;
    const int nch = B.nr >= (uint32_t)kMinLength ? B.nch : k0;   // :584, shorter -> last literals only
    const int nsteps = k0 + ((nch - k0 + 5) & ~1);   // >= nch + 4 steps, even count

    if (wave == 1) {   // producer
        PSet C0, C1;
        uint32_t XS = 0;   // chunk dword of the chunk in flight between L(k) and H(k)
        // Load waits (vmcnt counts a wave's loads in issue order).  Issue order per step
        // s: first half Y(s+1) X(s+2), second half Bc(s) -- one load instruction each
        // outside SMALL (whose byte loads are waited for whole).
        // H(s+1): X(s+1) is followed by Bc(s-1): 1 younger.
        // F(s-1), then M(s): Bc(s-1) (and the older Y(s)) are followed by Y(s+1) X(s+2):
        // 2 younger.  The step is two halves: H and F run beside the walker's chain, M
        // beside its table inserts.
        constexpr int kW1 = SMALL ? 0 : 1, kW2 = SMALL ? 0 : 2;
        auto pstep = [&](auto fast, int s, PSet &cur, PSet &nxt) {
            constexpr bool F = decltype(fast)::value;
            // First half: H(s+1) -- the table reads (the walker inserts in second halves)
            vm_wait<kW1>();                    // X(s+1)
            x_spread(S, s + 1, lane, XS, nxt.X);
            p_lookup<SMALL, F>(S, B, s + 1, lane, nxt);
            p_load<SMALL, F>(B, s + 2, lane, XS);
            // F(s-1) (info of chunk s-1: read by the walker in step s+1)
            vm_wait<kW2>();                    // A/Bc(s-1), Y/Z(s)
            p_finish(S, B, s - 1, lane, nxt);
            STAT(5);
            __builtin_amdgcn_sched_barrier(0);
            __syncthreads();
            STAT(6);
            __builtin_amdgcn_sched_barrier(0);
            // Second half: M(s)
            p_measure<SMALL, F>(S, B, s, lane, cur);
#ifdef APE_FINE_STATS
            STAT(8);
#endif
            // nothing may be scheduled across the step boundary: the compiler would
            // hoist the next step's use of this step's loads above the barrier and
            // wait for them here
            __builtin_amdgcn_sched_barrier(0);
            __syncthreads();
            STAT(7);
            __builtin_amdgcn_sched_barrier(0);
        };
        if (k0 > 0) prefix_history(S, B, lane);
        // prologue: the loads in flight at the loop entry in the steady-state order --
        // Y(k0), X(k0+1), Bc(k0-1) (idle stand-in)
        p_load<SMALL, false>(B, k0, lane, XS);
        __builtin_amdgcn_s_waitcnt(0);
        x_spread(S, k0, lane, XS, C0.X);
        p_lookup<SMALL, false>(S, B, k0, lane, C0);
        p_load<SMALL, false>(B, k0 + 1, lane, XS);
        C1.q2 = 0xFFFFFFFFu;
        C1.lg = 0;
#pragma unroll
        for (int t = 0; t < 4; t++) C1.A[t] = 0;
        load16<SMALL>(B.in, B.n, 0, C1.Bc, !SMALL);
        __syncthreads();   // table cleared, scratch ready
        // Steps whose loads all lie inside the block run a loop without edge paths:
        // X(s+2): 64(s+2)+140 <= n (stage 2 of chunk s reads c + 76 < p + 76 <= n).
        const int nfast = SMALL || B.n < 268 ? 0 : (B.n - 268) / 64 + 1;
        int s = k0;
        // the first step always runs the edge path (chunk k0's backward context)
        pstep(std::false_type{}, s, C0, C1);
        pstep(std::false_type{}, s + 1, C1, C0);
        s += 2;
        for (; s + 1 < nfast; s += 2) {
            pstep(std::true_type{}, s, C0, C1);
            pstep(std::true_type{}, s + 1, C1, C0);
        }
        for (; s < nsteps; s += 2) {
            pstep(std::false_type{}, s, C0, C1);
            pstep(std::false_type{}, s + 1, C1, C0);
        }
        __builtin_amdgcn_s_waitcnt(0);
        STATS_FLUSH_TID(g_enc_stats_v2, 64);
        return;
    }
    if (wave == 0) {   // walker: chunk s-2 during step s
        // the walker's scalar chain is the latency-critical path of a step: it issues
        // ahead of the other two roles sharing its SIMD
        __builtin_amdgcn_s_setprio(3);
        Walk W;
        W.q = 64u * (uint32_t)k0;
        W.a = W.q;
        W.qn = 0;
        W.Q0 = W.Q1 = 0;
        W.nx = 0;
        WalkOut O;
        O.member = O.walked = false;
        O.x = O.y = 0;
        uint2 iv = make_uint2(0u, 0u);   // info of the chunk walked next (read a half early)
        __syncthreads();
        for (int s = k0; s < nsteps; s++) {
            // chunk s-2 is final: M(s-2) ran in the second half of step s-2, F(s-2) in the
            // first half of step s-1; its info was read in the second half of step s-1
            const bool work = s >= k0 + 2 && s - 2 < nch;
            if (work) walk_chain(B, s - 2, lane, W, O, iv);
            STAT(0);
            __syncthreads();
            STAT(4);
            iv = S.info[(s - 1) & (kNI - 1)][lane];   // chunk s-1: final since F(s-1) above
            if (work) {
                walk_post(S, s - 2, lane, W, O);
                walk_publish(S, B, s - 2, lane, O);
            }
            // one step after the last chunk: hand over what is still queued (a full batch
            // may have gone out with the last chunk; the emitter reads it in this step's
            // first half, and this one in the next step, which exists: nsteps >= nch + 4)
            if (s - 2 == nch && W.qn) walk_flush(S, lane, W);
            STAT(1);
            STAT_ADD(10, 3);
            __syncthreads();
            STAT(3);
        }
        STAT_ADD(11, W.nx);
        STATS_FLUSH(g_enc_stats_v2);
        return;
    }
    // emitter: a batch the walker queued in step s-1, records + literal loads in the
    // first half of step s, stores in the second
    __builtin_amdgcn_s_setprio(2);
    __syncthreads();
    Em E;
    uint32_t ca = 64u * (uint32_t)k0, co = 0;   // running anchor / output offset
    for (int s = k0; s < nsteps; s++) {
        emit_load<SMALL>(S, B, lane, E, ca, co);
        STAT(2);
        __syncthreads();
        STAT(14);
        emit_store(B, lane, E);
        STAT(12);
#ifndef APE_FINE_STATS
        STAT_ADD(8, E.cnt);      // sequences emitted
        STAT_ADD(9, E.cnt != 0); // batches
#endif
        __syncthreads();
        STAT(15);
    }
    // ---- last literals (:732-751), from the final anchor ----
    const uint32_t anchor = ca;
    const uint32_t o = co;
    const uint32_t lit = B.un - anchor;
    const uint32_t hdr = 1u + ext_bytes(lit);
    const uint32_t total = o + hdr + lit;
    const bool overflow = total > B.cap;
    if (!overflow) {
        if (lane == 0) {
            B.dst[o] = (uint8_t)((lit < 15u ? lit : 15u) << 4);
            put_len(B.dst + o + 1, lit);
        }
        wave_copy(B.in, B.dst, anchor, o + hdr, lit, lane);
    }
    if (lane == 0) *result = overflow ? 0 : (int)total;
    STAT_ADD(13, 1);
    STATS_FLUSH_TID(g_enc_stats_v2, 128);
}

}  // namespace

__global__ void __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(6)))
lz4_encode_v2_kernel(BlockArgs a) {
    __shared__ EncLds S;
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    // readfirstlane: the wave index is wave-uniform, and the compiler must know it,
    // or every value merged after the producer/consumer branches becomes a VGPR
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    Blk B;
    B.in = (gcu8 *)(a.src ? a.src[b] : a.src_base + (size_t)b * a.src_stride);
    B.dst = (gu8 *)(a.dst ? a.dst[b] : a.dst_base + (size_t)b * a.dst_stride);
    const int nr = a.src_size[b];
    const int icap = a.dst_cap ? a.dst_cap[b] : (int)a.dst_stride;
    if (nr < 0 || nr > kMaxBlock || icap < 0) {
        if (tid == 0) a.result[b] = (nr > kMaxBlock) ? kErange : 0;
        return;
    }
    // withPrefix: the history before the block becomes positions [0, D) of one
    // 64 KiB window (D a multiple of 64 chunks' worth, so chunk k0 starts the block)
    int D = 0;
    if (a.dict_size) {
        const int pre = a.dict_size[b];
        D = (pre > 0 ? (pre < kMaxBlock - nr ? pre : kMaxBlock - nr) : 0) & ~63;
        if (D < 64) D = 0;
    }
    B.in -= D;
    B.n = D + nr;
    B.nr = (uint32_t)nr;
    B.k0 = D / 64;
    // compress_fast's acceleration (:789-808) trades ratio for speed; here that is the
    // in-chunk candidate
    B.noL = a.accel > 1;
    B.cap = (uint32_t)icap;
    B.un = (uint32_t)B.n;
    B.mstart = B.un >= 12 ? B.un - 12 : 0;   // matches start at <= n-12 (:585)
    B.mlimit = B.un >= 5 ? B.un - 5 : 0;     // and end at <= n-5 (:633)
    B.nch = (B.n + 63) / 64;

    // table = 0 (the reference's memset state: position 0 for every hash)
    for (int i = tid; i < kHSize / 8; i += 192) ((uint4 *)S.tab)[i] = make_uint4(0, 0, 0, 0);
    if (tid < 64) S.scr[tid] = 0xFFFFFFFFu;
    if (tid == 0) S.qcnt = 0;
    __syncthreads();
    if (B.n < kSmall) encode_block<true>(S, B, wave, lane, &a.result[b]);
    else encode_block<false>(S, B, wave, lane, &a.result[b]);
}

hipError_t launch_encode_v2(const BlockArgs &a, hipStream_t s) {
    if (a.nblocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(lz4_encode_v2_kernel, dim3(a.nblocks), dim3(192), 0, s, a);
    return hipGetLastError();
}

}  // namespace apelz4
