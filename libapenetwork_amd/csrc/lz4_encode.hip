// lz4_encode.hip -- MI355X (gfx950) batched LZ4 block encoder: the product encoder.
// (A second pipeline measured in round 2 lives only in the git history)
//
// Replaces the per-block work of APE_LZ4_compress_default (ref src/ape_lz4.c:
// 811-815 -> LZ4_compress_generic :530-755, byU16 / noDict).  The output is a
// valid LZ4 v1.7.1 block -- it obeys every parsing rule decompress_safe enforces
// (:1346-1366, :1375, :1444-1447): matches start at <= n-12, end at <= n-5, the
// last >= 5 bytes are literals -- but it is produced by a chunk-parallel parse,
// not by the reference's sequential search, so the bytes differ.
//
// One 192-thread workgroup (three waves, one role each) per block; a batch holds
// ~1M blocks, so most of the parallelism comes from many blocks in flight (9 per
// CU).  Per block the LDS (17.5 KiB) holds a hash table like the reference's (:449-462:
// u16 positions, a hash of 5 bytes; 7200 entries instead of 8192, see kHSize), a 1 KiB
// ring of recent input and the hand-over records between the roles.  The input stays in
// HBM/L2.
//
// The block is cut into chunks of 64 positions, one per lane.  The waves run in
// lock step, two workgroup barriers per step s (each waits only on its own memory
// operations; s_waitcnt vmcnt counts a wave's loads and stores together, in order):
//   PRODUCER (wave 1), three chunks in flight:
//     R(s+2)  copy chunk s+2 (loaded a step ago) into the ring;
//     A(s+3)  load in[p, p+8) for every position p of the chunk;
//     B(s+2)  hash in[p, p+5), read candidate T = table[h] (positions walked
//             earlier plus match_end - 2, inserted as the reference does:
//             :595-619, :680-706) and L = the earliest lane of the chunk with the
//             same hash bits; load in[T-4, T+16);
//     C1(s+1) own bytes from the ring, verify 4 bytes for T and L, measure T to 16
//             bytes and L to 12 forward and both 4 backward, keep the longer;
//     S2(s+1) (second half) the truncated candidates, ranked and pushed into groups
//             of 4 lanes, each group loading the 64 bytes that follow;
//     C2(s)   finish the truncated lengths (+64 bytes) -> match info of chunk s.
//   WALKER (wave 0), chunk s-1: the greedy chain on the scalar unit (a 9-instruction
//     loop over the match lanes of a ballot mask, one v_readlane per member), the
//     wave-wide extension of matches >= 80 bytes; second half: catch-up into pending
//     literals (:623-627), table inserts of the walked positions and match_end - 2
//     (:680, hashed from ring bytes read before the walk), never overlapping B, and the
//     chunk's sequence records queued for the emitter.
//   EMITTER (wave 2), every <= 8 steps: up to 64 queued records sized, prefix-summed
//     and staged in LDS (token, lengths, offset, literals from the ring), then stored
//     with one 16-byte store per lane; the last literals (:732-751) are copied with
//     16-byte moves.
#include "lz4_gpu_internal.h"
#include <type_traits>

namespace apelz4 {

#ifdef APE_LZ4_STATS
__device__ unsigned long long g_enc_stats[16];
// per-phase cycle sums of the encoder
hipError_t enc_stats_read(unsigned long long *out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_enc_stats), sizeof(g_enc_stats));
    if (e == hipSuccess && reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_enc_stats), z, sizeof(z));
    }
    return e;
}
#endif

namespace {


#ifndef APE_LZ4_HLOG
#define APE_LZ4_HLOG 13
#endif
constexpr int kHLog = APE_LZ4_HLOG;
// Table entries.  The reference's 8192 (2^13) entries make the block's LDS 20.4 KiB, so
// 8 blocks fit a CU; 7200 entries (the hash scaled onto [0, 7200)) make it 17.5 KiB (17904 B),
// inside the 35 x 512-byte LDS granules that fit 9 blocks = 27 waves per CU (7 per SIMD:
// <= 72 VGPRs).  Measured on 131072 blocks: 6912 entries -4.6 % encode time vs 8192, ratio
// 3.1464 -> 3.1279; 7200 (once the info array was single-buffered) 3.1329 at the same time
// (tools/enc_model.c models the ratio per table size).
// Hash key: the bytes the table hash covers (the reference: 5, :456-473).  7 by default, with
// every position in the table (kAllPos): the longer key keeps short chance matches from
// pre-empting longer ones -- ratio above the round-5 encoder's on App. C data and on real
// files, 23 % fewer sequences (tools/enc_model.c key study)
#ifndef APE_LZ4_HKEY
#define APE_LZ4_HKEY 7
#endif
constexpr int kKey = APE_LZ4_HKEY;
static_assert(kKey >= 5 && kKey <= 8, "hash key of 5..8 bytes");
// Table inserts: 1 = the producer writes every hashable position of a chunk into the table
// right after the chunk's lookups (no lag: chunk k sees every position of chunks < k, and the
// walker inserts nothing); 0 = the reference's policy (:595-619, :680-706), walked positions
// and match_end - 2, inserted by the walker a chunk behind (chunk k then sees chunks <= k - 4:
// the repeats at 64..256 bytes that real files are full of were lost -- 6.6 % below the
// reference's ratio on Python sources at round 5).  -8 % encode time.
#ifndef APE_LZ4_ALLPOS
#define APE_LZ4_ALLPOS 1
#endif
constexpr bool kAllPos = APE_LZ4_ALLPOS != 0;
// One workgroup barrier per step instead of two (1).  The mid-step barrier orders the walker's
// table inserts after the producer's lookups and the walker's read of the single info array
// before the producer's next write; with kAllPos the walker inserts nothing, and the info array
// can be double-buffered by chunk parity (its 512 bytes from the table), so each role runs its
// whole step and the three meet once.  Measured: encode time unchanged (44.07 vs 44.06 ms per
// 131072 blocks; the texture path and VALU issue, not the barriers, set the step), ratio
// -0.24 % from the smaller table -- off
#ifndef APE_LZ4_ONEBAR
#define APE_LZ4_ONEBAR 0
#endif
constexpr bool kOneBar = APE_LZ4_ONEBAR != 0;
static_assert(!kOneBar || kAllPos, "one barrier per step needs the producer-only table");
constexpr uint32_t kInfoBufs = kOneBar ? 2u : 1u;
// The in-chunk candidate L (the earliest lane of the chunk with the same 6 hash bits; an LDS
// scratch, 4 ds_bpermute, a 12-byte measure and the pick): 1 = none.  With every position in
// the table (kAllPos) T finds the repeats from earlier chunks at no lag, so L only adds a
// first repeat inside one chunk: without it encode -8.7 %, decode -2.5 %, ratio -0.7 % on App.
// C data and -1.3 % on real files (profiles/r6_encoder_policy_ab.txt).  Its scratch's 256 bytes
// go to the table: 7328 entries.
#ifndef APE_LZ4_NOL
#define APE_LZ4_NOL 1
#endif
#ifndef APE_LZ4_TSIZE
#if APE_LZ4_NOL && APE_LZ4_ONEBAR
#define APE_LZ4_TSIZE 7072           // (the second info buffer takes 256 entries)
#elif APE_LZ4_NOL
#define APE_LZ4_TSIZE 7328
#else
#define APE_LZ4_TSIZE 7200
#endif
#endif
constexpr int kHSize = APE_LZ4_TSIZE;
static_assert(kHSize <= (1 << kHLog) && kHSize % 8 == 0, "table size");
#ifndef APE_LZ4_WAVES_PER_EU
#define APE_LZ4_WAVES_PER_EU 7
#endif
// T measured to 12 bytes (as L): with stage 2 finishing only the runs' last lanes, the extra
// truncated lanes cost less than C1's fifth dword (the 16-byte C1 of rounds 2-3 measured +1.5 %;
// same decisions -- L is taken only when T < 12 -- so the same bytes; both bases 12)
#ifndef APE_LZ4_EAGER_T
#define APE_LZ4_EAGER_T 12
#endif
constexpr uint32_t kEagerLen = APE_LZ4_EAGER_T;   // match bytes measured by C1 (T candidate)
static_assert(kEagerLen == 8 || kEagerLen == 12 || kEagerLen == 16 || kEagerLen == 20,
              "C1 measures T to 8, 12, 16 or 20 bytes");
constexpr int kYW = (int)(kEagerLen + 4u) / 4;   // T-candidate dwords loaded: in[T-4, T+kEagerLen)
constexpr uint32_t kEagerL = 12;     // ... for the in-chunk candidate L
// Stage 2 (C2) measures only the candidates C1 left truncated (~13 % of the lanes on App.
// C data), compacted into groups of 4 lanes that compare 16 bytes each: 64 more bytes
// per candidate, 16 candidates per pass (a second pass is rare).
constexpr uint32_t kExt2 = 64;
constexpr uint32_t kGroups = 16;
// Stage 2 only for the last lane of each run of truncated lanes with the same offset and base
// (the others' lengths follow from it, exactly: DESIGN.md 3.1)
#ifndef APE_LZ4_S2RUN
#define APE_LZ4_S2RUN 1
#endif
#ifndef APE_LZ4_ERING
#define APE_LZ4_ERING 1024
#endif
constexpr uint32_t kRingE = APE_LZ4_ERING;  // recent input bytes (own, stage 2, end-2, literals)
static_assert(kRingE < 65536u, "the ring holds recent input, not the block's window (DESIGN.md 3.1.1)");
#ifndef APE_LZ4_SCRBITS
#define APE_LZ4_SCRBITS 6
#endif
[[maybe_unused]] constexpr uint32_t kScr = 1u << APE_LZ4_SCRBITS;  // in-chunk candidate scratch
constexpr int kSmall = 128;          // smaller blocks take the byte-load path
// Sequence records in flight between the walker and the emitter.  The emitter reads up to
// 64 records into registers at a fetch (its slots are free from then on); it fetches when
// kFetchAt are queued or every APE_EMIT_EVERY steps, and while a batch is pending it
// finishes that batch at once (emit_all, no fetch) when kEmitAll are queued.  The walker adds
// at most kChunkRecs per step (a match covers >= 4 of the chunk's 64 positions).  Worst
// case: kEmitAll - 1 queued at a pending step, + kChunkRecs before emit_all, + kChunkRecs
// before the next fetch -- that must fit the ring, or the walker overwrites unread records.
constexpr uint32_t kQ = 128;
constexpr uint32_t kFetchAt = 48, kEmitAll = 80, kChunkRecs = 64u / 4u;
static_assert((kQ & (kQ - 1u)) == 0u, "record ring indexed by & (kQ - 1)");
static_assert(kEmitAll - 1u + 2u * kChunkRecs <= kQ, "walker -> emitter record ring overflow");
static_assert(kFetchAt < kEmitAll, "a fetch precedes emit_all");
// acceleration > 1 keeps the in-chunk candidate: the reference's table holds every earlier
// probe with no lag, the GPU's lags a chunk or two, and at sparse probes L is what finds the
// near matches (ratio within 1 % of the reference at a = 2, 4, 8 with it, 2.5-2.7 % below
// without: DESIGN.md 3.1); 0 = the faster search without it
#ifndef APE_LZ4_ACC_L
#define APE_LZ4_ACC_L 1
#endif
constexpr bool kNoL = APE_LZ4_NOL != 0;
#ifndef APE_LZ4_APF
#define APE_LZ4_APF 1                // producer: own-bytes load A two steps ahead (else one)
#endif
#ifndef APE_LZ4_CAPBITS
#define APE_LZ4_CAPBITS 1            // length caps folded into the bit-index mins (v_min3)
#endif
#ifndef APE_EMIT_EVERY
#define APE_EMIT_EVERY 8             // emitter: a batch every this many steps (at most)
#endif
constexpr uint32_t kStage = 512;     // emitter: output bytes per batch
constexpr uint32_t kStageAlloc = kStage + 16u + 16u + 64u;   // + alignment, slack, dummies


// info.x: len (7) | trunc << 7 | back << 8 (3) | hashable << 13;   info.y: offset | h << 16
// The low byte is the walker's hop as it is: 0 = no candidate (a found match has len >= 4),
// len, or len | 0x80 = unfinished (len <= kEagerLen + kExt2 < 128).
constexpr uint32_t I_TRUNC = 1u << 7, I_HASHABLE = 1u << 13;
static_assert(kEagerLen + kExt2 < 128u, "len fits 7 bits");

struct __attribute__((aligned(16))) EncLds {
    // input byte x at ring byte (x mod kRingE); the first 64 bytes are mirrored
    // after the end, so a 36-byte read never wraps (immediate LDS offsets).  At LDS offset
    // 0, so that a read's dwords share one address register (ds_read2 offsets)
    uint32_t ring[kRingE / 4 + 16];
    uint16_t tab[kHSize];
    uint2 info[kInfoBufs][64];       // producer -> walker: chunk k in [k % kInfoBufs], written in the second half of
                                     // step k, read at the start of step k + 1 (before the
                                     // producer writes chunk k + 1 after the mid barrier)
#if !APE_LZ4_NOL
    uint32_t scr[kScr];              // producer scratch: earliest lane per low hash bits
#endif
    uint2 q[kQ];                     // walker -> emitter: sequence records, record r in
                                     // [r % kQ]: {lit | (match length - 4) << 16, offset}
    uint32_t qn[2];                  // walker -> emitter: records published ([0]; kOneBar: by step
                                     // parity, the emitter of step s reading step s - 1's)
    uint8_t __attribute__((aligned(16))) stage[kStageAlloc];   // emitter: one batch's bytes
};

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

// X = L shifted by d bytes (X byte i = L byte i + d, 0 outside L), |d| < 32,
// with compile-time register indices only (a barrel shifter).
__device__ __forceinline__ void shift_bytes(const uint32_t (&L)[8], int d, uint32_t (&X)[8]) {
    uint32_t T[8];
#pragma unroll
    for (int k = 0; k < 8; k++) T[k] = L[k];
    const bool down = d >= 0;
    const int ad = down ? d : -d, w = ad >> 2;
    const uint32_t r = (uint32_t)ad & 3u;
#pragma unroll
    for (int bit = 4; bit >= 1; bit >>= 1) {
        if (w & bit) {
            if (down) {
#pragma unroll
                for (int k = 0; k < 8; k++) T[k] = (k + bit < 8) ? T[k + bit] : 0u;
            } else {
#pragma unroll
                for (int k = 7; k >= 0; k--) T[k] = (k - bit >= 0) ? T[k - bit] : 0u;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (down) X[k] = __builtin_amdgcn_alignbyte(k + 1 < 8 ? T[k + 1] : 0u, T[k], r);
        else X[k] = r ? __builtin_amdgcn_alignbyte(T[k], k >= 1 ? T[k - 1] : 0u, 4u - r) : T[k];
    }
}

// 32 bytes in[pos, pos+32) (bytes outside [0, n) read as 0).
// SMALL: byte loads.  Otherwise (n >= 32): two unaligned 16-byte loads from the
// clamped window, fixed up with ALU only (so the wave's vmcnt accounting stays
// static in the pipelined loop).
// fast (wave-uniform): every lane's window is known to lie inside [0, n).
template <bool SMALL>
__device__ __forceinline__ void load32(gcu8 *in, int n, int pos, uint32_t (&X)[8],
                                       bool fast = false) {
    if (!SMALL && fast) {
        gcu8 *q = in + (uint32_t)pos;   // saddr + voffset, +16 as the immediate offset
        const uint4 a = gload16(q), b = gload16(q + 16);
        X[0] = a.x; X[1] = a.y; X[2] = a.z; X[3] = a.w;
        X[4] = b.x; X[5] = b.y; X[6] = b.z; X[7] = b.w;
        return;
    }
    if (SMALL) {
#pragma unroll
        for (int k = 0; k < 8; k++) X[k] = 0;
#pragma unroll
        for (int k = 0; k < 32; k++) {
            const int q = pos + k;
            if (q >= 0 && q < n) X[k >> 2] |= (uint32_t)in[(uint32_t)q] << (8 * (k & 3));
        }
        return;
    }
    const int ca = pos < 0 ? 0 : (pos > n - 32 ? n - 32 : pos);
    gcu8 *q = in + (uint32_t)ca;
    const uint4 a = gload16(q), b = gload16(q + 16);
    const uint32_t L[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    if (ca == pos) {
#pragma unroll
        for (int k = 0; k < 8; k++) X[k] = L[k];
    } else {
        // the clamped window ends at n / starts at 0, so shifting it zero-fills
        // exactly the bytes outside [0, n)
        const int d = pos - ca;   // |d| >= 32 only for lanes past the block end
        shift_bytes(L, d < -31 ? -31 : (d > 31 ? 31 : d), X);
        if (d > 31 || d < -31) {
#pragma unroll
            for (int k = 0; k < 8; k++) X[k] = 0;
        }
    }
}

// Hash of the kKey bytes at p (x0 = in[p..p+3], x1 = in[p+4..p+7]) onto [0, kHSize).  The
// reference multiplies the 40-bit sequence by 889523592379 (:456-473), which needs
// quarter-rate 32-bit multiplies here; any hash gives a valid stream, so this one uses
// full-rate 24 x 24-bit multiplies (v_mul_u32_u24 / v_mad_u32_u24, which read only the low
// 24 bits of their operands) of bytes 0-2 and 3-5 (and 6 or 6-7).  With kKey = 5 it is the
// round-5 hash (same ratio as the reference's on App. C data, tools/enc_model.c).
__device__ __forceinline__ uint32_t hashk(uint32_t x0, uint32_t x1) {
    uint32_t hi;
    if constexpr (kKey == 5) hi = (x0 >> 24) | ((x1 & 0xFFu) << 8);
    else hi = __builtin_amdgcn_alignbyte(x1, x0, 3u);   // bytes 3..6 (the multiply takes 3..5)
    // (__umul24 returns int: do the sums and the shift unsigned)
    uint32_t v = (uint32_t)__umul24(x0, 0x9E3779u) + (uint32_t)__umul24(hi, 0xC2B2AEu);
    if constexpr (kKey == 7) v += (uint32_t)__umul24((x1 >> 16) & 0xFFu, 0x27D4EBu);
    if constexpr (kKey == 8) v += (uint32_t)__umul24(x1 >> 16, 0x27D4EBu);
    if constexpr (kHSize == (1 << kHLog)) return v >> (32 - kHLog);
    else return __umulhi(v, (uint32_t)kHSize);   // v scaled onto [0, kHSize): one v_mul_hi_u32
}

// v_ffbl_b32 / v_ffbh_u32: lowest / highest set bit, 0xFFFFFFFF for 0 (inline asm
// so that the compiler does not turn the zero case into compare + select)
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

// first differing bit of dwords A[K0..K1) vs B (bit index from A[K0]'s bit 0), or
// 0xFFFFFFFF: ffbl + saturating add + min3 per dword, no compares or selects
template <int K0, int K1, int NA, int NB>
__device__ __forceinline__ uint32_t first_diff_bit(const uint32_t (&A)[NA], const uint32_t (&B)[NB]) {
    static_assert(K1 <= NA && K1 <= NB, "dwords");
    uint32_t m = ffbl(A[K0] ^ B[K0]);
#pragma unroll
    for (int k = K0 + 1; k < K1; k++)
        m = umin(m, __builtin_elementwise_add_sat(ffbl(A[k] ^ B[k]), 32u * (uint32_t)(k - K0)));
    return m;
}

// common length of X and Y from byte 4 (dword 1) on, up to kEagerLen.  The cap is applied to
// the bit index (one v_min3 with the dwords' own min) instead of to the byte count afterwards
__device__ __forceinline__ uint32_t eager(const uint32_t (&X)[6], const uint32_t (&Y)[6]) {
#if APE_LZ4_CAPBITS
    return (umin(first_diff_bit<2, kYW>(X, Y), 8u * (kEagerLen - 4u)) >> 3) + 4u;
#else
    return umin((first_diff_bit<2, kYW>(X, Y) >> 3) + 4u, kEagerLen);
#endif
}

// bytes equal just before the match (in[p-1] == in[c-1], ...), 0..4
__device__ __forceinline__ uint32_t back4(uint32_t x0, uint32_t y0) {
    return umin(ffbh(x0 ^ y0) >> 3, 4u);
}

// e / 255 with one full-rate 24-bit multiply: 255 * 0x8081 = 2^23 + 127, so
// floor(e * 0x8081 / 2^23) = floor(e / 255) for e < 66060 (lengths here are < 65537)
__device__ __forceinline__ uint32_t div255(uint32_t e) {
    return (uint32_t)__umul24(e, 0x8081u) >> 23;
}

// 255 x (low 24 bits of v), one full-rate v_mul_u32_u24 (written out: the compiler
// turns __umul24(v, 255) into a mask and a quarter-rate v_mul_lo_u32)
__device__ __forceinline__ uint32_t mul255(uint32_t v) {
    uint32_t r;
    asm("v_mul_u32_u24 %0, 0xff, %1" : "=v"(r) : "v"(v));
    return r;
}

// bytes after a 15 nibble: v < 15 -> 0, else (v - 15) / 255 + 1 -- both are
// (v + 240) / 255 (v + 240 < 255 below 15; one full-rate multiply, no select)
__device__ __forceinline__ uint32_t ext_bytes(uint32_t v) {
    return div255(v + 240u);
}

// write the length extension of v (>= 15) at o
__device__ __forceinline__ void put_len(gu8 *o, uint32_t v) {
    if (v < 15) return;
    v -= 15;
    uint32_t k = 0;
    for (; v >= 255; v -= 255) o[k++] = 255;
    o[k] = (uint8_t)v;
}

// 16 / 8 input bytes at x from the ring (the mirrored tail keeps a read that starts in
// the last 64 bytes contiguous): aligned dword reads + v_alignbyte.  (Measured against
// single unaligned ds_read_b128 / _b64 (round 4): 12.5 vs 11.3 ms per 16384
// blocks -- fewer VALU instructions, but a 1-byte lane stride makes the unaligned reads
// slow.)
__device__ __forceinline__ uint4 ring16(const EncLds &S, uint32_t x) {
    const uint32_t *r = S.ring + ((x >> 2) & (kRingE / 4 - 1));
    const uint32_t sh = x & 3u;
    const uint32_t w0 = r[0], w1 = r[1], w2 = r[2], w3 = r[3], w4 = r[4];
    return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                      __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
}
__device__ __forceinline__ uint2 ring8(const EncLds &S, uint32_t x) {
    const uint32_t *r = S.ring + ((x >> 2) & (kRingE / 4 - 1));
    const uint32_t sh = x & 3u;
    const uint32_t w0 = r[0], w1 = r[1], w2 = r[2];
    return make_uint2(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh));
}

// NW dwords in[pos, pos + 4 NW) (NW = 4 or 6).  fast: the window lies inside [0, n)
// (vector loads); otherwise byte loads, bytes outside [0, n) read as 0 (the edge steps
// and blocks below kSmall only).
template <int NW, int NA>
__device__ __forceinline__ void loadv(gcu8 *in, uint32_t un, uint32_t pos, uint32_t (&X)[NA],
                                      bool fast) {
    static_assert(NW >= 3 && NW <= 6 && NW <= NA, "loadv");
    if (fast) {
        if constexpr (NW == 3) {
            const uint3 a = gload12(in + pos);
            X[0] = a.x; X[1] = a.y; X[2] = a.z;
            return;
        }
        const uint4 a = gload16(in + pos);
        X[0] = a.x; X[1] = a.y; X[2] = a.z; X[3] = a.w;
        if constexpr (NW == 6) {
            const uint2 b = gload8(in + pos + 16u);
            X[4] = b.x; X[5] = b.y;
        } else if constexpr (NW == 5) {
            X[4] = gload4(in + pos + 16u);
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < NW; k++) X[k] = 0;
#pragma unroll
    for (uint32_t t = 0; t < 4u * NW; t++)
        if (pos + t < un) X[t >> 2] |= (uint32_t)in[pos + t] << (8 * (t & 3));
}

// lane l receives v of lane idx (idx mod 64)
__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t idx) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(idx << 2), (int)v);
}
// rank of this lane among the set lanes of m below it
__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
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
    uint32_t stride;                 // acceleration (compress_fast): the first search step
};

// ---------------- producer ----------------
struct Part {                        // C1 result of one chunk, finished by C2
    uint32_t len, c, bk, lim, base;      // base: bytes C1 measured (kEagerLen / kEagerL)
    uint32_t iy;                     // info.y: offset (0 = no candidate) | h << 16, formed in C1
                                     // while `has` is a lane mask (a bool carried to C2 was
                                     // materialised as 0/1 and compared again)
    uint32_t rank, ntr, eo;          // stage-2 queue rank, queue size, own bytes of the group
    bool hashable;
    uint64_t tmask;                  // lanes whose candidate reached its measured length (a
                                     // wave mask: no per-lane 0/1 to materialise)
    uint64_t smask;                  // ... of them, the lanes stage 2 measures
};

// One parity of the producer pipeline (the step loop is unrolled by two, so no
// register set is ever copied): X from A for B, Y/cT/jL/h from B for C1, q/E from
// C1 for C2.
struct PSet {
    uint32_t X[2];                   // own bytes in[p, p+8) of the chunk B works on next
    uint32_t Y[6];                   // T-candidate bytes in[T-4, T+kEagerLen)
    uint32_t E[4];                   // stage-2 candidate bytes of this lane's group
    uint32_t cT, jL, h;
    Part q;
};

// A(k): own bytes in[p, p+8) for the hash (0 past the block end)
template <bool SMALL, bool FAST = false>
__device__ __forceinline__ void prod_load(const Blk &B, int k, int lane, uint32_t (&X)[2]) {
    const uint32_t pos = (FAST || k < B.nch ? 64u * (uint32_t)k : 0u) + (uint32_t)lane;
    if (FAST || (!SMALL && 64 * k + 72 <= B.n)) {   // wave-uniform: the whole window is inside
        const uint2 v = gload8(B.in + pos);
        X[0] = v.x;
        X[1] = v.y;
        return;
    }
    X[0] = X[1] = 0;
#pragma unroll
    for (uint32_t t = 0; t < 8u; t++)
        if (pos + t < B.un) X[t >> 2] |= (uint32_t)B.in[pos + t] << (8 * (t & 3));
}

// T candidate bytes in[T-4, T+kEagerLen) of chunk k (issued one step before C1 consumes them).
// Candidates below position 4 are skipped: their 4 bytes of backward context would start
// before the block (never-written slots read as 0).
template <bool SMALL, bool FAST = false>
__device__ __forceinline__ void prod_fetch_t(const Blk &B, int k, int lane, uint32_t cT,
                                             uint32_t (&Y)[6]) {
    const uint32_t p = 64u * (uint32_t)k + (uint32_t)lane;
    if (FAST) {   // any address in [0, p): a lane whose T is not a candidate (C1 rechecks
                  // cT < p and cT >= 4) loads harmless bytes -- min + saturating subtract
        loadv<kYW>(B.in, B.un, __builtin_elementwise_sub_sat(umin(cT, p - 1u), 4u), Y, true);
        return;
    }
    const bool tryT = k < B.nch && cT < p && cT >= 4u;
    loadv<kYW>(B.in, B.un, tryT ? cT - 4u : 0u, Y, !SMALL && 64 * k + 83 <= B.n);
}

// B(k): hash, table + in-chunk candidates, T fetch issue
template <bool SMALL, bool FAST = false>
__device__ __forceinline__ void prod_lookup(EncLds &S, const Blk &B, int k, int lane,
                                            const uint32_t (&X)[2], uint32_t &cT, uint32_t &jL,
                                            uint32_t &h, uint32_t (&Y)[6]) {
    const uint32_t p = 64u * (uint32_t)k + (uint32_t)lane;
    // (FAST: chunk k lies inside the block with room to spare, every lane is hashable)
    const bool hashable = FAST || (k < B.nch && p + 5u <= B.un);
    h = hashk(X[0], X[1]);
    cT = S.tab[h];
    jL = 0xFFFFFFFFu;
    if (!kNoL && !B.noL) {   // wave-uniform
#if !APE_LZ4_NOL
        const uint32_t hs = h & (kScr - 1u);
        if (hashable) atomicMin(&S.scr[hs], (uint32_t)lane);
        wave_sync();
        jL = hashable ? S.scr[hs] : 0xFFFFFFFFu;
        wave_sync();
        if (hashable) S.scr[hs] = 0xFFFFFFFFu;
#endif
    }
    if constexpr (kAllPos) {
        // after this chunk's lookups (one wave's LDS operations complete in order); lanes with
        // the same slot: the last lane's write lands last, the latest position wins
        if (hashable) S.tab[h] = (uint16_t)p;
    }
    prod_fetch_t<SMALL, FAST>(B, k, lane, cT, Y);
}

// R(k): ring copy of chunk k (own bytes for C1 and stage 2, match_end - 2, literals; zero
// past the block end), at the start of step k - 2, right before C1(k - 1) reads chunks k - 1
// and k from the ring (same wave: in order)
template <bool FAST = false>
__device__ __forceinline__ void prod_ring(EncLds &S, const Blk &B, int k, int lane,
                                          const uint32_t (&X)[2]) {
    if (FAST || k < B.nch) {
        const uint32_t p = 64u * (uint32_t)k + (uint32_t)lane;
        const uint8_t by = (uint8_t)X[0];
        ((uint8_t *)S.ring)[p & (kRingE - 1)] = by;
        if (((64u * (uint32_t)k) & (kRingE - 1)) == 0u) ((uint8_t *)S.ring)[kRingE + lane] = by;
    }
}

// own bytes in[p-4, p+20) of chunk k from the ring (ring tail = 0 before 0)
__device__ __forceinline__ void prod_own(const EncLds &S, int k, int lane, uint32_t (&X)[6]) {
    const uint32_t p = 64u * (uint32_t)k + (uint32_t)lane;
    // 7 aligned dwords, 6 alignbytes
    const uint32_t *r = S.ring + (((p - 4u) >> 2) & (kRingE / 4 - 1));
    const uint32_t sh = p & 3u;
    uint32_t W[7];
#pragma unroll
    for (int t = 0; t < 7; t++) W[t] = r[t];
#pragma unroll
    for (int t = 0; t < 6; t++) X[t] = __builtin_amdgcn_alignbyte(W[t + 1], W[t], sh);
}

// Stage-2 group of this lane for the truncated lanes of ranks [first, first + kGroups):
// the lane of rank first + g pushes its continuation points to lane 4g (ds_permute, a
// forward permute; the other lanes push to odd lanes, never read), and the quad
// broadcasts them; lane 4g + i then compares the 16 bytes at offset 16 i.  Returns
// whether the group has an entry; cb / eo = candidate / own position of those bytes.
__device__ __forceinline__ bool stage2_group(const Part &R, int lane, uint32_t first, uint32_t p,
                                             uint32_t &cb, uint32_t &eo) {
    const uint32_t r = R.rank - first, i16 = 16u * ((uint32_t)lane & 3u);
    const bool push = lane_in(R.smask) && r < kGroups;
    const int tgt = (int)((push ? 4u * r : ((uint32_t)lane | 1u)) << 2);
    cb = dpp_z<0x00>((uint32_t)__builtin_amdgcn_ds_permute(tgt, (int)(R.c + R.base))) + i16;
    eo = dpp_z<0x00>((uint32_t)__builtin_amdgcn_ds_permute(tgt, (int)(p + R.base))) + i16;
    return first + ((uint32_t)lane >> 2) < R.ntr;
}

// Stage-2 result of entry `first + g` (all four lanes of group g): bytes equal from the
// continuation point, 0..kExt2
__device__ __forceinline__ uint32_t stage2_len(const EncLds &S, int lane, uint32_t eo,
                                               const uint32_t (&E)[4]) {
    const uint4 o = ring16(S, eo);
    const uint32_t O[4] = {o.x, o.y, o.z, o.w};
    const uint32_t li = 128u * ((uint32_t)lane & 3u);
#if APE_LZ4_CAPBITS   // the cap 8 kExt2 bits joins the lane's own min (no min after the quad's)
    uint32_t d = umin(first_diff_bit<0, 4>(O, E), 8u * kExt2 - li) + li;   // (no overflow)
#else
    uint32_t d = __builtin_elementwise_add_sat(first_diff_bit<0, 4>(O, E), li);
#endif
    d = umin(d, dpp<0xB1>(0u, d));   // quad_perm [1,0,3,2]
    d = umin(d, dpp<0x4E>(0u, d));   // quad_perm [2,3,0,1]
#if APE_LZ4_CAPBITS
    const uint32_t len = d >> 3;     // <= kExt2
#else
    const uint32_t len = umin(d >> 3, kExt2);
#endif
#if APE_LZ4_S2RUN   // continuation point + length: a run member subtracts its own
    return eo + len;
#else
    return len;
#endif
}

// C1(k): verify / measure to kEagerLen bytes / pick; queue the truncated candidates and issue
// the stage-2 loads of the first kGroups of them
template <bool SMALL, bool FAST = false>
__device__ __forceinline__ void prod_measure(EncLds &S, const Blk &B, int k, int lane,
                                             const uint32_t (&X)[6], const uint32_t (&Y)[6],
                                             uint32_t cT, uint32_t jL, uint32_t h, Part &R) {
    const uint32_t p = 64u * (uint32_t)k + (uint32_t)lane;
    // FAST (chunk k + 1 lies inside the block with 83 bytes to spare, k >= 1): every lane is
    // live, hashable and may start a match
    const bool live = FAST || k < B.nch;
    R.hashable = FAST || (live && p + 5u <= B.un);
    const bool can = FAST || (live && p >= 1u && p <= B.mstart && B.n >= kMinLength);
    const uint32_t cL = 64u * (uint32_t)k + jL;
    // L candidate bytes in[cL-4, cL+12) from lane jL's own bytes (4 ds_bpermute; reading
    // them from the ring beside X, in the same LDS round trip, measured +2.3 % encode time:
    // 5 ds_read + 4 v_alignbyte)
    uint32_t Z[4];
#pragma unroll
    for (int t = 0; t < 4; t++) Z[t] = bperm(X[t], jL);
    // (bitwise on bools: lane masks combined by the scalar unit, no materialised 0/1)
    const bool okT = can & (cT < p) & (cT >= 4u) & (Y[1] == X[1]);
    // (no cL != cT test: when L's candidate is T's, L is kept only when T < 12 bytes, and then
    // both give the same position, length and preceding bytes)
    const bool okL = !kNoL && (can & (jL < (uint32_t)lane) & (Z[1] == X[1]));   // jL = ~0 if noL
    // (FAST: the match limit lies >= 132 bytes past every lane, beyond anything C1 and C2
    // measure, so it never cuts a length: no limit arithmetic at all)
    R.lim = FAST ? 0xFFFFu : (can ? B.mlimit - p : 0u);   // (a FAST chunk finished by a
                                                            // general step: no cut either)
    // measured unconditionally (selects, no branches): every lane reads Y, so the
    // compiler sees the candidate load consumed on every path.  T to 16 bytes, L to 12:
    // L (the closer one) is taken when T is shorter than 12 and L at least as long,
    // and C2 continues the taken candidate from where C1 stopped
    // (tools/enc_model.c model4, pol 7 vs 0: ratio -0.1 %; measured -0.06 %, -3.4 % VALU).
    const uint32_t eT = eager(X, Y);
#if APE_LZ4_CAPBITS
    const uint32_t eL = (umin(first_diff_bit<2, 4>(X, Z), 8u * (kEagerL - 4u)) >> 3) + 4u;
#else
    const uint32_t eL = umin((first_diff_bit<2, 4>(X, Z) >> 3) + 4u, kEagerL);
#endif
    const uint32_t lT = okT ? eT : 0u, lL = okL ? eL : 0u;
    const bool pickL = okL & (!okT | ((lT < kEagerL) & (lL >= lT)));
    R.c = pickL ? cL : cT;
    R.len = pickL ? lL : lT;
    R.base = pickL ? kEagerL : kEagerLen;
    // (two ballots of compares fold into the compares; a ballot of their AND made the
    // compiler materialise a 0/1 and compare it again)
    if (FAST) {
        R.tmask = wave_ballot(R.len >= R.base);
    } else {
        R.tmask = wave_ballot(R.len >= R.base) & wave_ballot(R.lim > R.base);
        R.len = umin(R.len, R.lim);
    }
#if APE_LZ4_S2RUN
    {   // lane i + 1 truncated with the same offset and base: in[p, p+1) == in[c, c+1), so the
        // match from p is one byte longer than lane i + 1's (and lim one larger): only the
        // run's last lane is measured
        const uint32_t key = (R.c - (uint32_t)lane) + (R.base << 24);
        const uint32_t keyn = dpp_z<kDppWaveShl1>(key);   // lane 63: 0, never a key
        R.smask = R.tmask & ~((R.tmask >> 1) & wave_ballot(key == keyn));
    }
#else
    R.smask = R.tmask;
#endif
    R.bk = umin(back4(X[0], pickL ? Z[0] : Y[0]), R.c);  // c - back >= 0
    R.iy = ((okT | okL) ? p - R.c : 0u) | (h << 16);
}

// S2(k), at the start of the second half (off C1's latency chain, next to C2(k-1)):
// rank the truncated lanes and issue the stage-2 loads of the first kGroups of them
template <bool SMALL, bool FAST = false>
__device__ __forceinline__ void prod_stage2_issue(const EncLds &S, const Blk &B, int k, int lane,
                                                  Part &R, uint32_t (&E)[4]) {
    const uint32_t p = 64u * (uint32_t)k + (uint32_t)lane;
    const uint64_t tb = R.smask;   // (a run member's rank is its run's last lane's)
    R.ntr = (uint32_t)__popcll(tb);
    R.rank = lane_rank(tb);
    uint32_t cb;
    const bool ga = stage2_group(R, lane, 0u, p, cb, R.eo);
    // cb + 16 <= c + base + kExt2 < p + 80 (c < p)
    loadv<4>(B.in, B.un, ga ? cb : 0u, E, FAST || (!SMALL && 64 * k + 148 <= B.n));
}

// C2(k): finish the truncated lengths against the ring -> info
template <bool SMALL, bool FAST = false>
__device__ __forceinline__ void prod_finish(EncLds &S, const Blk &B, int k, int lane,
                                            const Part &R, const uint32_t (&E)[4]) {
    const uint32_t p = 64u * (uint32_t)k + (uint32_t)lane;
    uint32_t len = R.len;
    bool trunc = false;
    {   // unconditional: a chunk without a truncated lane is rare (~1 in 250)
        uint32_t mine = bperm(stage2_len(S, lane, R.eo, E), 4u * R.rank);
        for (uint32_t first = kGroups; first < R.ntr; first += kGroups) {   // rare
            uint32_t cb, eo, E2[4];
            const bool ga = stage2_group(R, lane, first, p, cb, eo);
            loadv<4>(B.in, B.un, ga ? cb : 0u, E2, FAST || (!SMALL && 64 * k + 148 <= B.n));
            const uint32_t m2 = bperm(stage2_len(S, lane, eo, E2), 4u * (R.rank - first));
            if (R.rank - first < kGroups) mine = m2;
        }
        if (lane_in(R.tmask)) {
#if APE_LZ4_S2RUN   // mine - p = the run's last lane's length + the distance to it
            const uint32_t cap = R.base + kExt2, full = mine - p;
            len = FAST ? umin(full, cap) : umin(umin(full, cap), R.lim);
            trunc = full >= cap && (FAST || R.lim > cap);
#else
            len = FAST ? R.base + mine : umin(R.base + mine, R.lim);
            trunc = mine == kExt2 && (FAST || R.lim > R.base + kExt2);
#endif
        }
    }
    // (FAST: the chunk lies inside the block, every lane hashable -- also the prologue's
    // chunk when the first step is FAST)
    S.info[(uint32_t)k & (kInfoBufs - 1u)][lane] = make_uint2(len | (R.bk << 8) | (trunc ? I_TRUNC : 0u) |
                                  ((FAST || R.hashable) ? I_HASHABLE : 0u),
                                     R.iy);
}

// ---------------- walker ----------------
struct Walk {
    uint32_t q;          // walk position (the next probe)
    uint32_t anchor;     // start of the pending literals (= the last match end)
};

// compress_fast's search pattern (ref :591-600, :710-720): after a match end e the
// reference tests e, searches from e + 1 with step 1 once, then takes the j-th step
// searchMatchNb >> skipTrigger = acc + ((j - 1) >> 6): probes e, e+1, e+2, then
// y = e + 2 + {acc, 2 acc, .., 64 acc, 64 acc + (acc+1), ..} -- regime r (gap acc + r) starts
// after S_r = 64 (acc r + r (r - 1) / 2).  `Probe` is the regime of the chunk's first lane
// relative to a far origin e0 (a chunk spans at most two regimes: each covers >= 128 positions
// when acc >= 2); lanes whose origin is a match end inside the chunk are in regime 0.
struct Probe {
    uint32_t s0, s1, g0;   // S_r, S_{r+1}, acc + r
};
__device__ __forceinline__ Probe probe_regime(uint32_t P, uint32_t e0, uint32_t acc) {
    const uint32_t y0 = P > e0 + 2u ? P - e0 - 2u : 0u;   // wave-uniform
    uint32_t s = 0, g = acc;
    while (y0 > s + 64u * g) {   // (scalar; a few trips per chunk at most)
        s += 64u * g;
        g++;
    }
    Probe R;
    R.s0 = s;
    R.s1 = s + 64u * g;
    R.g0 = g;
    return R;
}
// is position e + d probed?  far: e is the regime's origin e0; else d < 64 (regime 0)
__device__ __forceinline__ bool probed(uint32_t d, bool far, const Probe &R, uint32_t acc) {
    const uint32_t y = d - 2u;
    const bool hi = far && y > R.s1;
    const uint32_t base = far ? (hi ? R.s1 : R.s0) : 0u;
    const uint32_t g = far ? (hi ? R.g0 + 1u : R.g0) : acc;
    return d <= 2u || (y - base) % g == 0u;
}

// forward extension of the match at m (candidate cm) from L bytes on, with the
// whole wave, 1 KiB per step; returns the full length (<= mlimit - m)
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

// Walk chunk k (first half of step k + 1), then (second half) insert the walked
// positions and match_end - 2 into the table and hand the members to the emitter.
// The greedy chain (:591-627: a position with a match jumps past it, any other
// position is a literal): the scalar unit hops over the match lanes only (ballot
// mask, one v_readlane per member); walked positions, catch-up limits (:623-627)
// and the new anchor follow for all 64 lanes at once from the member set.  A match
// the producer could not finish (TRUNC, >= 60 bytes) is extended by the whole wave.
struct WalkOut {
    uint64_t walked, members;
    uint32_t m_back, m_len, an;   // per member lane
    uint2 iv;
    uint32_t q0, Lf;              // walk start; forward match length per lane
    uint2 e2v;                    // in[e2, e2 + 8), e2 = match_end - 2 (read before the walk)
    uint32_t e2h;                 // its hash
    uint32_t pmv, pe;             // kWalkPm: per member lane, the end of the match before it
                                  // (relative to the chunk start); the last match end (relative)
};

// The walker's catch-up limits from the hop chain itself (1): the chain writes each member's
// previous match end into its lane (v_writelane) as it finds it, instead of a wave-wide max
// scan over the member ends afterwards (with kAllPos and no acceleration only: the walked set,
// which needs the limit on every lane, is not used then).  Same bytes, -0.4..-0.5 % encode
// time (profiles/r6_encoder_policy_ab.txt call 21)
#ifndef APE_LZ4_WPM
#define APE_LZ4_WPM 1
#endif
constexpr bool kWalkPm = APE_LZ4_WPM != 0 && kAllPos;

// The walker's hop chain from walk position rel (< 64): shift, find-first, add, mark,
// v_readlane, compare, branch -- 9 scalar-unit instructions per member (the compiler's loop
// took 13).  nxt (per lane) = the walk position after the lane's match; leaves with rel >= 64
// (64: no match lane left), j = the last member, its bit set in M.
[[maybe_unused]] __device__ __forceinline__ void hop_chain(uint64_t Hm, uint32_t nxt, uint32_t &rel, uint64_t &M,
                                          uint32_t &j) {
    uint64_t t;
    asm volatile(
        "1:\n\t"
        "s_lshr_b64 %[t], %[hm], %[rel]\n\t"
        "s_cmp_eq_u64 %[t], 0\n\t"
        "s_cbranch_scc1 2f\n\t"
        "s_ff1_i32_b64 %[j], %[t]\n\t"
        "s_add_u32 %[j], %[j], %[rel]\n\t"
        "s_bitset1_b64 %[m], %[j]\n\t"
        "v_readlane_b32 %[rel], %[nxt], %[j]\n\t"
        "s_cmp_lt_u32 %[rel], 64\n\t"
        "s_cbranch_scc1 1b\n\t"
        "s_branch 3f\n"
        "2:\n\t"
        "s_mov_b32 %[rel], 64\n"
        "3:"
        : [rel] "+s"(rel), [m] "+s"(M), [j] "+s"(j), [t] "=&s"(t)
        : [hm] "s"(Hm), [nxt] "v"(nxt)
        : "scc");
}
// ... also writing pe (the previous match end) into lane j of pmv for each member j, pe then
// the member's end (12 instructions per member).  The lane select goes through m0 (a VALU
// instruction reads one SGPR on gfx9); nothing else in this kernel uses m0 (LDS instructions
// do not on gfx950; tests/test_product_abi.py::test_encoder_m0_only_in_hop_chain checks the ISA)

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"   // (m0 declared clobbered: see above)
__device__ __forceinline__ void hop_chain_pm(uint64_t Hm, uint32_t nxt, uint32_t &rel, uint64_t &M,
                                             uint32_t &j, uint32_t &pe, uint32_t &pmv) {
    uint64_t t;
    asm volatile(
        "1:\n\t"
        "s_lshr_b64 %[t], %[hm], %[rel]\n\t"
        "s_cmp_eq_u64 %[t], 0\n\t"
        "s_cbranch_scc1 2f\n\t"
        "s_ff1_i32_b64 %[j], %[t]\n\t"
        "s_add_u32 %[j], %[j], %[rel]\n\t"
        "s_bitset1_b64 %[m], %[j]\n\t"
        "s_mov_b32 m0, %[j]\n\t"   // (one SGPR operand per VALU instruction: the lane in m0)
        "v_writelane_b32 %[pmv], %[pe], m0\n\t"
        "v_readlane_b32 %[rel], %[nxt], %[j]\n\t"
        "s_mov_b32 %[pe], %[rel]\n\t"
        "s_cmp_lt_u32 %[rel], 64\n\t"
        "s_cbranch_scc1 1b\n\t"
        "s_branch 3f\n"
        "2:\n\t"
        "s_mov_b32 %[rel], 64\n"
        "3:"
        : [rel] "+s"(rel), [m] "+s"(M), [j] "+s"(j), [t] "=&s"(t), [pe] "+s"(pe), [pmv] "+v"(pmv)
        : [hm] "s"(Hm), [nxt] "v"(nxt)
        : "scc", "m0");
}
#pragma clang diagnostic pop

// First half: the hop chain only (the latency-bound part); second half, before the
// inserts: the lane-parallel catch-up limits, walked set and anchor (walk_finish).
template <bool ACC>
__device__ __forceinline__ void walk_chain(const EncLds &S, const Blk &B, int k, int lane, Walk &W,
                                           WalkOut &O) {
    const uint32_t P = 64u * (uint32_t)k;
    O.walked = O.members = 0;
    O.m_back = O.m_len = O.an = 0;
    O.iv = S.info[(uint32_t)k & (kInfoBufs - 1u)][lane];
    O.q0 = W.q;
    O.pe = W.anchor - P;                                 // (kWalkPm; u32 wrap below P)
    O.Lf = O.iv.x & 0x7Fu;                               // forward match length
    // match_end - 2 (:680) of every lane's match, read from the ring now so that the
    // second half's hash needs no LDS round trip (the ring holds chunks k - 13 .. k + 2,
    // and a match the producer finished ends before p + 81; a match the walker extends
    // is hashed from the input instead)
    if constexpr (!kAllPos) O.e2v = ring8(S, P + (uint32_t)lane + O.Lf - 2u);
    if (W.q >= P + 64u) return;               // a match from earlier chunks covers it
    const uint2 iv = O.iv;
    const uint64_t Hm = wave_ballot(O.Lf != 0u);          // lanes with a match
    const uint32_t Lh = iv.x & 0xFFu;                     // hop; | 0x80 = unfinished
    uint32_t rel = W.q - P;
    uint64_t M = 0;
    if constexpr (!ACC) {
        // The hop chain with one v_readlane per member: nxt = the walk position after the
        // lane's match, +256 marking a match the producer could not finish.
        const uint32_t nxt = (uint32_t)lane + (iv.x & 0x7Fu) + ((iv.x & 0x80u) << 1);
        uint32_t j = 0;
        if constexpr (kWalkPm) hop_chain_pm(Hm, nxt, rel, M, j, O.pe, O.pmv);
        else hop_chain(Hm, nxt, rel, M, j);
        while (__builtin_expect(rel >= 256u, 0)) {   // unfinished (rare): the wave extends it
            const uint32_t me = P + j;
            const uint32_t cm = me - (lane_val(iv.y, (int)j) & 0xFFFFu);
            const uint32_t Le = extend_match(B, me, cm, rel - 256u - j, lane);
            if ((uint32_t)lane == j) O.Lf = Le;
            rel = j + Le;
            O.pe = rel;
            if (rel >= 64u) break;
            if constexpr (kWalkPm) hop_chain_pm(Hm, nxt, rel, M, j, O.pe, O.pmv);
            else hop_chain(Hm, nxt, rel, M, j);
        }
        O.members = M;
        W.q = P + rel;
        return;
    }
    // acceleration: a member is taken only at a probe position (probe_regime): from the last
    // match end before the chunk (far), then from each member's end (near)
    const Probe R = probe_regime(P, W.anchor, B.stride);
    uint32_t e = W.anchor;
    bool far = true;
    for (;;) {
        const uint32_t x = P + (uint32_t)lane;
        const uint64_t pm = wave_ballot(x >= e && probed(x - e, far, R, B.stride));
        const uint64_t w = (Hm & pm) >> rel;
        if (w == 0) {   // no probe with a match left in the chunk
            rel = 64u;
            break;
        }
        const uint32_t j = rel + (uint32_t)__builtin_ctzll(w);
        const uint32_t h = lane_val(Lh, (int)j);
        M |= 1ull << j;
        if (h & 0x80u) {
            const uint32_t me = P + j;
            const uint32_t cm = me - (lane_val(iv.y, (int)j) & 0xFFFFu);
            const uint32_t Le = extend_match(B, me, cm, h & 0x7Fu, lane);
            if ((uint32_t)lane == j) O.Lf = Le;
            rel = j + Le;
        } else {
            rel = j + h;
        }
        e = P + rel;
        far = false;
        if (rel >= 64u) break;
    }
    O.members = M;
    W.q = P + rel;
}

template <bool ACC>
__device__ __forceinline__ void walk_finish(const Blk &B, int k, int lane, Walk &W, WalkOut &O) {
    const uint32_t P = 64u * (uint32_t)k;
    // match_end - 2's hash, from the bytes read before the walk (every lane; a match the
    // walker extended is rehashed in walk_publish): independent of the scan below, so it
    // fills the scan's DPP wait states.  (No early exit for a chunk a match from earlier
    // chunks covers: it has no members, nothing is walked, the anchor stays.)
    if constexpr (!kAllPos) O.e2h = hashk(O.e2v.x, O.e2v.y);
    // catch-up limits: a member's backward extension stops at the previous end
    const uint32_t anchor0 = W.anchor;
    const bool mem = lane_in(O.members);
    const uint32_t p = P + (uint32_t)lane;
    uint32_t pm, lastend;
    if constexpr (kWalkPm && !ACC) {   // (member lanes only: the others' limit is unused)
        pm = P + O.pmv;
        lastend = P + O.pe;
    } else {
        const uint32_t end = mem ? p + O.Lf : 0u;
        const uint32_t imax = wave_incl_max(end);
        pm = umax(wave_shr1(imax, 0u), anchor0);
        lastend = umax(anchor0, lane_val(imax, 63));
    }
    uint32_t bk = umin((O.iv.x >> 8) & 7u, p - pm);
    if (ACC) {
        // acceleration probes every stride-th position, so a match found at a probe often
        // starts further back than the 4 bytes C1 measured: the reference's catch-up
        // (:623-627) is unbounded -- continue it byte by byte here (up to 16 more bytes; the
        // ACC path only), stopping at the pending literals' start and the window start
        const uint32_t c = p - (O.iv.y & 0xFFFFu);
        const uint32_t room = umin(p - pm, c);
        if (mem && bk == 4u && room > 4u) {
            const uint32_t lim = umin(room - 4u, 16u);
            uint32_t more = 0;
            for (uint32_t t = 1; t <= lim; t++) {
                if (B.in[p - 4u - t] != B.in[c - 4u - t]) break;
                more = t;
            }
            bk += more;
        }
    }
    O.m_back = bk;
    O.m_len = O.Lf + bk;
    O.an = pm;
    // walked = every position from the walk start that no match of this chunk covers
    // (with acceleration: the probed ones, every stride-th from the last match end)
    bool w = p >= umax(O.q0, pm);
    if (ACC) {   // the probed ones (the origin: the last match end before the lane)
        const Probe R = probe_regime(P, anchor0, B.stride);
        w = w && probed(p - pm, pm == anchor0, R, B.stride);
    }
    O.walked = wave_ballot(w);
    W.anchor = lastend;
}

__device__ __forceinline__ void walk_publish(EncLds &S, const Blk &B, int k, int lane,
                                             const WalkOut &O, uint32_t &qn, int step) {
    const uint32_t p = 64u * (uint32_t)k + (uint32_t)lane;
    const uint2 iv = O.iv;
    const bool mem = lane_in(O.members);
    if constexpr (!kAllPos) {   // (kAllPos: the producer has inserted every position)
    if (lane_in(O.walked) && (iv.x & I_HASHABLE)) S.tab[iv.y >> 16] = (uint16_t)p;
    const uint32_t fwd = O.m_len - O.m_back;      // match length from p
    // match_end - 2 (:680) of the members, hashed here (off the producer's chain): from the
    // ring bytes read before the walk, or, for a match the walker extended, from the input
    const uint32_t e2 = p + fwd - 2u;
    const bool e2ok = mem && e2 + 5u <= B.un;
    uint32_t e2h = O.e2h;   // (ring bytes read before the walk: -1.6 % encode time)
    if (e2ok && (iv.x & I_TRUNC)) {   // rare: a match the walker extended
        uint32_t w[2] = {0u, 0u};   // in[e2, e2 + 8), 0 past the block end (as A loads it)
        for (uint32_t t = 0; t < 8u; t++)
            if (e2 + t < B.un) w[t >> 2] |= (uint32_t)B.in[e2 + t] << (8 * (t & 3));
        e2h = hashk(w[0], w[1]);
    }
    // one wave's LDS operations complete in order: the walked-position inserts above
    // land before these (compiler barrier only)
    __builtin_amdgcn_sched_barrier(0);
    if (e2ok) S.tab[e2h] = (uint16_t)e2;
    }
    // the chunk's sequences, in order, as records for the emitter: literals from the
    // anchor to the match start (after catch-up), the match length and its offset
    if (mem) S.q[(qn + lane_rank(O.members)) & (kQ - 1u)] =
        make_uint2(((p - O.m_back) - O.an) | ((O.m_len - kMinMatch) << 16), iv.y & 0xFFFFu);
    qn += (uint32_t)__popcll(O.members);
    if (lane == 0) S.qn[kOneBar ? (step & 1) : 0] = qn;
}

// ---------------- emitter ----------------
// Sequences are written one per lane from the walker's records, a batch at a time (every
// 4 steps, ~18 records on App. C data):
//   F (first half of a step): read the records, size them, prefix-sum output offsets and
//     input positions, take the leading records whose output fits the 512-byte staging
//     buffer, check the capacity, and write their bytes into the staging buffer -- token,
//     length extensions, offset, and the literals copied from the input ring (the ring
//     holds the last 13-16 chunks, and a batch's records are at most ~6 chunks old);
//   C (second half): the staged bytes -> dst with one 16-byte store per lane.
// No global memory is read, and one store instruction per batch is written: emitter
// memory instructions stall the whole block (byte stores to scattered addresses, or a
// literal re-read from global memory, measured +8-30 % encode time).  The staging buffer
// keeps dst's 16-byte alignment (batch byte 0 at stage[o0 % 16]); only whole 16-byte
// chunks go out, the last partial chunk stays and becomes the next batch's chunk 0.  A
// "big" record -- literals no longer in the ring, or a record larger than the buffer
// (long literal runs, in practice) -- is written straight to dst by the whole wave after
// the copy.
struct Emit {
    uint32_t o;          // output cursor
    uint32_t ein;        // input position of the next record's literals (its anchor)
    uint32_t qc;         // records consumed
    int last;            // step of the last batch
    bool overflow;
    bool part;           // stage[0, o % 16) does not hold dst's bytes there
    int pend;            // the pending batch's next piece: 0 none, 1 L, 2 H, 3 C
    bool nv;             // per lane: a staged (not big) record
    uint32_t o0, tot;    // output offset and bytes of the pending batch
    uint64_t bigm;       // its big records, and per lane their token's staging index,
    uint32_t r, lit, mlm4, off, ba;   // literal count, match length - 4, offset, literals
};

// one staging byte per lane, branch-free: lanes with nothing to write hit their own dummy
// byte past the buffer
__device__ __forceinline__ void stage_put(EncLds &S, int lane, bool w, uint32_t at, uint32_t b) {
    S.stage[w ? at : kStageAlloc - 64u + (uint32_t)lane] = (uint8_t)b;
}

// F: up to min(avail, 64) records from E.qc: sizes, offsets, capacity; input positions
// below `rlo` will no longer be in the ring when the literals are copied (piece L).
__device__ __forceinline__ void emit_fetch(EncLds &S, const Blk &B, int lane, Emit &E,
                                           uint32_t avail, uint32_t rlo) {
    const bool v0 = (uint32_t)lane < avail;
    const uint2 rec = S.q[(E.qc + (uint32_t)lane) & (kQ - 1u)];
    const uint32_t lit = v0 ? (rec.x & 0xFFFFu) : 0u, mlm4 = v0 ? (rec.x >> 16) : 0u;
    const uint32_t size = v0 ? 3u + ext_bytes(lit) + lit + ext_bytes(mlm4) : 0u;
    const uint32_t isz = wave_incl_sum(size);
    // the leading records that fit the staging buffer (at least one)
    const uint32_t nrec = umax((uint32_t)__popcll(wave_ballot(v0) & wave_ballot(isz <= kStage)), 1u);
    const bool v = (uint32_t)lane < nrec;
    const uint32_t adv = v ? lit + mlm4 + kMinMatch : 0u;
    const uint32_t iadv = wave_incl_sum(adv);
    const uint32_t tot = lane_val(isz, (int)nrec - 1), tadv = lane_val(iadv, (int)nrec - 1);
    E.qc += nrec;
    if (E.overflow) return;
    // (32-bit: o <= cap < 2^31 and a batch's output < 2^21)
    if (E.o + tot > B.cap) {
        E.overflow = true;
        return;
    }
    E.ba = E.ein + (iadv - adv);                 // literal source
    E.r = (E.o & 15u) + (isz - size);            // token's staging index
    E.lit = v ? lit : 0u;
    E.mlm4 = mlm4;
    E.off = rec.y;
    const bool big = v && (E.ba < rlo || size > kStage);
    E.bigm = wave_ballot(big);
    E.nv = v && !big;
    E.o0 = E.o;
    E.tot = tot;
    E.o += tot;
    E.ein += tadv;
    E.pend = 1;
}

// L: the literals, from the input ring -> staging, 16 bytes per lane per trip (aligned
// ring dwords + v_alignbyte: one LDS round trip), written as unaligned dwords.  A lane's
// last dword may run up to 3 bytes past its literals: onto its own offset and the byte
// after it (a match-length extension or the next record's token) -- header bytes, which
// piece H writes afterwards.  (No other lane's literals start before those 3 bytes end.)
__device__ __forceinline__ void emit_lits(EncLds &S, int lane, Emit &E) {
    const bool nv = E.nv;
    const uint32_t lit = E.lit, a = E.ba;
    const uint32_t lo = E.r + 1u + ext_bytes(lit);
    typedef uint32_t u32a __attribute__((aligned(1)));
    for (uint32_t t = 0; wave_any(nv && t < lit); t += 16u) {
        const uint4 w = ring16(S, a + t);
        const uint32_t W[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (uint32_t u = 0; u < 4u; u++) {
            const bool wr = nv && t + 4u * u < lit;
            *(u32a *)(S.stage + (wr ? lo + t + 4u * u : kStageAlloc - 64u + 4u * ((uint32_t)lane & 15u))) = W[u];
        }
    }
    E.pend = 2;
}

// H: token, literal-length extension, offset, match-length extension -> staging
__device__ __forceinline__ void emit_heads(EncLds &S, int lane, Emit &E) {
    const bool nv = E.nv;
    const uint32_t lit = E.lit, mlm4 = E.mlm4, r = E.r;
    const uint32_t elit = ext_bytes(lit), eml = ext_bytes(mlm4);
    stage_put(S, lane, nv, r, (umin(lit, 15u) << 4) | umin(mlm4, 15u));
    for (uint32_t k = 0; wave_any(nv && k < elit); k++)
        stage_put(S, lane, nv && k < elit, r + 1u + k, umin(lit - 15u - mul255(k), 255u));
    const uint32_t oo = r + 1u + elit + lit;
    stage_put(S, lane, nv, oo, E.off);
    stage_put(S, lane, nv, oo + 1u, E.off >> 8);
    for (uint32_t k = 0; wave_any(nv && k < eml); k++)
        stage_put(S, lane, nv && k < eml, oo + 2u + k, umin(mlm4 - 15u - mul255(k), 255u));
    E.pend = 3;
}

// one sequence written straight to dst by the whole wave (big records)
__device__ __forceinline__ void emit_one(const Blk &B, int lane, uint32_t o, uint32_t a,
                                         uint32_t lit, uint32_t mlm4, uint32_t off) {
    gu8 *dst = B.dst;
    const uint32_t elit = ext_bytes(lit), eml = ext_bytes(mlm4);
    const uint32_t oo = o + 1u + elit + lit;
    if (lane == 0) dst[o] = (uint8_t)((umin(lit, 15u) << 4) | umin(mlm4, 15u));
    for (uint32_t k = (uint32_t)lane; k < elit; k += 64u)
        dst[o + 1u + k] = (uint8_t)umin(lit - 15u - 255u * k, 255u);
    wave_copy(B.in, dst, a, o + 1u + elit, lit, lane);
    if (lane < 2) dst[oo + (uint32_t)lane] = (uint8_t)(off >> (8 * lane));
    for (uint32_t k = (uint32_t)lane; k < eml; k += 64u)
        dst[oo + 2u + k] = (uint8_t)umin(mlm4 - 15u - 255u * k, 255u);
}

// C: the staged batch -> dst.  stage[16 c, 16 c + 16) holds dst[a + 16 c, a + 16 c + 16),
// a = o0 rounded down to 16; the batch covers stage[s0, s0 + tot), s0 = o0 % 16.  Only
// whole chunks go out; the last partial chunk moves to stage[0, 16).  After a batch with a
// big record everything goes out, the partial chunk by byte stores, and the next batch's
// chunk 0 then holds only its own bytes (E.part).
__device__ __forceinline__ void emit_copy(EncLds &S, const Blk &B, int lane, Emit &E) {
    E.pend = 0;
    const uint32_t s0 = E.o0 & 15u, end = s0 + E.tot;
    gu8 *out = B.dst + (E.o0 - s0);
    const uint32_t c0 = 16u * (uint32_t)lane;
    const uint64_t bigm = E.bigm;
    const uint32_t nfull = end >> 4;   // (a batch with one big record can pass kStage:
                                       // only its staged chunks, the rest is direct)
    const bool head = E.part && s0 != 0u;   // chunk 0 is partial: dst holds its start
    if ((uint32_t)lane < umin(nfull, kStage / 16u + 1u) && !(head && lane == 0))
        gstore16(out + c0, *(const uint4 *)(S.stage + c0));
    if (head || (bigm && (end & 15u) && nfull <= kStage / 16u)) {   // rare: byte stores
        const uint32_t pc = (head && lane == 0) ? 0u : 16u * nfull;
        const bool act = (head && lane == 0) || (bigm && (end & 15u) && lane == 1);
        const uint4 w = *(const uint4 *)(S.stage + (act ? pc : 0u));
        const uint32_t W[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (uint32_t t = 0; t < 16u; t++)
            if (act && pc + t >= s0 && pc + t < end) out[pc + t] = (uint8_t)(W[t >> 2] >> (8 * (t & 3)));
    }
    if (bigm) {
        vm_wait<0>();   // the copy above first: a big record's bytes overwrite it
        for (uint64_t m = bigm; m; m &= m - 1) {
            const int j = __builtin_ctzll(m);
            emit_one(B, lane, E.o0 - s0 + lane_val(E.r, j), lane_val(E.ba, j), lane_val(E.lit, j),
                     lane_val(E.mlm4, j), lane_val(E.off, j));
        }
        E.part = true;
    } else {
        if (lane == 0) {   // carry the partial chunk to stage[0, 16)
            const uint4 t = *(const uint4 *)(S.stage + 16u * nfull);
            *(uint4 *)S.stage = t;
        }
        // (a partial chunk 0 that is still partial keeps its bytes in dst only)
        E.part = head && nfull == 0u;
    }
}

// the pending batch's next piece (or all of them)
__device__ __forceinline__ void emit_step(EncLds &S, const Blk &B, int lane, Emit &E) {
    if (E.pend == 1) emit_lits(S, lane, E);
    else if (E.pend == 2) emit_heads(S, lane, E);
    else if (E.pend == 3) emit_copy(S, B, lane, E);
}
__device__ __forceinline__ void emit_all(EncLds &S, const Blk &B, int lane, Emit &E) {
    if (E.pend == 1) emit_lits(S, lane, E);
    if (E.pend == 2) emit_heads(S, lane, E);
    if (E.pend == 3) emit_copy(S, B, lane, E);
}

// the carried partial chunk (output bytes [o rounded down to 16, o)) -> dst
__device__ __forceinline__ void emit_tail(EncLds &S, const Blk &B, int lane, Emit &E) {
    const uint32_t s0 = E.o & 15u;
    if (!E.part && s0 != 0u && (uint32_t)lane < s0)
        B.dst[E.o - s0 + (uint32_t)lane] = S.stage[lane];
}

// ---------------- history prefix (withPrefix encode) ----------------
// Positions [0, 64 k0) precede the block in memory (the previous <= 64 KiB of the
// stream, as compress_fast_continue sees it, ref src/ape_lz4.c:1160-1220).  The
// producer wave hashes every third of them into the table, as loadDict does
// (:1127-1130; catch-up recovers the bytes a skipped start loses), oldest first (one
// wave: its LDS writes land in order, so the newest position wins deterministically),
// and copies the last 64 into the ring for the first chunk's backward context.
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
            if (ok[u]) S.tab[hashk(x[u].x, x[u].y)] = (uint16_t)v;
        }
    }
    const uint32_t p = D - 64u + (uint32_t)lane;
    const uint8_t by = B.in[p];
    ((uint8_t *)S.ring)[p & (kRingE - 1)] = by;
    if (((D - 64u) & (kRingE - 1)) == 0u) ((uint8_t *)S.ring)[kRingE + lane] = by;
}

// ---------------- block ----------------
// Three waves per block, one role each, in lock step (two barriers per step):
//   step s, first half : producer A(s+3) B(s+2) C1(s+1) | walker walks s-1 | emitter writes
//                                                         |   the pair (s-4, s-3) (every 2nd step)
//   step s, second half: producer C2(s) -> info     | walker inserts s-1, publishes
//                                                         | emitter sizes s-2
// Table inserts (second half) never overlap the producer's lookups (first half).
template <bool SMALL, bool ACC>
__device__ __forceinline__ void encode_block(EncLds &S, const Blk &B, int wave, int lane,
                                             int *result) {
    STATS_DECL
    const int k0 = B.k0;
    const int nch = B.nr >= (uint32_t)kMinLength ? B.nch : k0;   // :584, shorter -> last literals only
    const int nsteps = k0 + ((nch - k0 + 3) & ~1);   // >= nch + 2 steps (emission lags two)

    // Each role runs its own loop (same barrier count: 1 + 2 per step), so the
    // compiler's memory-counter waits in each loop see only that role's operations.
    if (wave == 1) {
        PSet P0, P1;
        // one producer step; `cur` = set of parity s, `nxt` = parity s + 1
        auto pstep = [&](auto fast, int s, PSet &cur, PSet &nxt) {
            constexpr bool F = decltype(fast)::value;
            // Every stage runs on every step, past the last chunk too (it then loads
            // from the block start and records nothing), so the number of loads per
            // step -- and with it the waits -- is the same on every path.
            // In flight, oldest first: A(s+2), Y(s+1), A(s+3), E(s) -> A(s+2) at 3 (APF; without:
            // A(s+2), Y(s+1), E(s)).
            vm_wait<3>();
            STAT(9);   // (stats build: load waits)
            // ring copy of chunk s+2 (loaded a step ago), then C1(s+1)'s own bytes (chunks
            // s+1 and s+2) from the ring: one wave's LDS operations complete in order.  (Until
            // round 3 chunk s+3 was copied in the second half of step s, which then waited
            // for a load issued half a step earlier: -2.7 % encode time.)
            prod_ring<F>(S, B, s + 2, lane, cur.X);
            uint32_t X6[6];   // C1(s+1)'s own bytes: in the ring since last step, read first
            prod_own(S, s + 1, lane, X6);
#if APE_LZ4_APF
            prod_lookup<SMALL, F>(S, B, s + 2, lane, cur.X, cur.cT, cur.jL, cur.h, cur.Y);
            // A two steps ahead, into the set B(s+2) has just consumed: the block's own input
            // streams in from HBM, and one step (~1 us) did not cover it (the producer's load
            // waits were the A load at the step start)
            prod_load<SMALL, F>(B, s + 4, lane, cur.X);
            // Y(s+1), A(s+3), E(s), Y(s+2), A(s+4) -> Y(s+1) at 4
#else
            prod_load<SMALL, F>(B, s + 3, lane, nxt.X);
            prod_lookup<SMALL, F>(S, B, s + 2, lane, cur.X, cur.cT, cur.jL, cur.h, cur.Y);
            // Y(s+1) x2, E(s), A(s+3), Y(s+2) x2 -> Y(s+1) at 4
#endif
            STAT(5);
            vm_wait<4>();
            STAT(9);
            prod_measure<SMALL, F>(S, B, s + 1, lane, X6, nxt.Y, nxt.cT, nxt.jL, nxt.h, nxt.q);
            STAT(5);
            if constexpr (!kOneBar) __syncthreads();
            STAT(6);
            prod_stage2_issue<SMALL, F>(S, B, s + 1, lane, nxt.q, nxt.E);
            // E(s), A(s+3), Y(s+2) x2, E(s+1) -> E(s) at 4 (A(s+3), issued half a step ago,
            // is not needed before the next step)
            STAT(7);
            vm_wait<(APE_LZ4_APF ? 3 : 4)>();   // (APF: Y(s+2), A(s+4), E(s+1) after E(s))
            STAT(9);
            prod_finish<SMALL, F>(S, B, s, lane, cur.q, cur.E);
            STAT(7);
            __syncthreads();
            STAT(8);
        };
        if (k0 > 0) prefix_history(S, B, lane);
        if (nch > k0) {  // prologue: A(k0), A(k0+1), B(k0), A(k0+2), B(k0+1), C1(k0)
            prod_load<SMALL>(B, k0, lane, P0.X);
            prod_load<SMALL>(B, k0 + 1, lane, P1.X);
            prod_ring(S, B, k0, lane, P0.X);
            prod_lookup<SMALL>(S, B, k0, lane, P0.X, P0.cT, P0.jL, P0.h, P0.Y);
            prod_load<SMALL>(B, k0 + 2, lane, P0.X);
            prod_ring(S, B, k0 + 1, lane, P1.X);
            prod_lookup<SMALL>(S, B, k0 + 1, lane, P1.X, P1.cT, P1.jL, P1.h, P1.Y);
            if (APE_LZ4_APF) prod_load<SMALL>(B, k0 + 3, lane, P1.X);   // (step k0 + 1's X)
            prod_ring(S, B, k0 + 2, lane, P0.X);
            uint32_t X6[6];
            prod_own(S, k0, lane, X6);
            prod_measure<SMALL>(S, B, k0, lane, X6, P0.Y, P0.cT, P0.jL, P0.h, P0.q);
            prod_stage2_issue<SMALL>(S, B, k0, lane, P0.q, P0.E);
        }
        // nothing in flight at the loop entry, so the loop's counter waits depend only
        // on its own issue order (once per block)
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        // Steps whose three loads all lie inside the block (A(s+3): 64(s+3)+72 <= n,
        // Y(s+2): 64(s+2)+83, E(s+1): 64(s+1)+148) run a loop without the edge paths;
        // the last few steps run the general one.
        // (APF: A(s+4), 64(s+4)+72 <= n)
        constexpr int kFastEnd = APE_LZ4_APF ? 328 : 264;
        const int nfast_abs = SMALL ? 0 : (int)umin((uint32_t)(B.n >= kFastEnd ? (B.n - kFastEnd) / 64 + 1 : 0),
                                                    (uint32_t)nsteps);
        const int nfast = nfast_abs > k0 ? k0 + ((nfast_abs - k0) & ~1) : k0;
        int s = k0;
#ifdef APE_EXP_PUNROLL
#pragma unroll APE_EXP_PUNROLL
#endif
        for (; s < nfast; s += 2) {   // no conditional step: see pstep
            pstep(std::true_type{}, s, P0, P1);
            pstep(std::true_type{}, s + 1, P1, P0);
        }
        for (; s < nsteps; s += 2) {
            pstep(std::false_type{}, s, P0, P1);
            pstep(std::false_type{}, s + 1, P1, P0);
        }
        STATS_FLUSH_TID(g_enc_stats, 64);
        return;
    }
    if (wave == 0) {   // walker: chunk s-1 during step s
        Walk W;
        uint32_t qn = 0;
        W.q = 64u * (uint32_t)k0;
        W.anchor = W.q;
        WalkOut O;
        __syncthreads();
        // chunk s - 1 is walked during step s for s in [k0 + 1, nch]; the first step and
        // the steps past the last chunk only keep the barrier count (separate loops, so
        // the walking loop carries no per-step predicate)
        const int s2 = nch + 1;
        __syncthreads();   // step k0
        if constexpr (!kOneBar) __syncthreads();
        int s = k0 + 1;
#ifdef APE_EXP_WUNROLL
#pragma unroll APE_EXP_WUNROLL
#endif
        for (; s < s2; s++) {
            walk_chain<ACC>(S, B, s - 1, lane, W, O);
            STAT(0);
            if constexpr (!kOneBar) __syncthreads();
            STAT(4);
            walk_finish<ACC>(B, s - 1, lane, W, O);
            walk_publish(S, B, s - 1, lane, O, qn, s);
            STAT_ADD(11, __popcll(O.members));
            STAT(1);
            STAT_ADD(10, 3);
            __syncthreads();
            STAT(3);
        }
        for (; s < nsteps; s++) {
            __syncthreads();
            if constexpr (!kOneBar) __syncthreads();
        }
        STATS_FLUSH(g_enc_stats);
        return;
    }
    // emitter: a batch every 4 steps (F in a first half, C in the second half); a queue of
    // 48+ records (never on App. C data) starts one at once; the rest after the last step
    Emit E;
    E.o = 0;
    E.ein = 64u * (uint32_t)k0;
    E.qc = 0;
    E.last = k0;
    E.overflow = false;
    E.part = false;
    E.pend = 0;
    E.nv = false;
    E.o0 = E.tot = 0;
    E.bigm = 0;
    E.r = E.lit = E.mlm4 = E.off = E.ba = 0;
    __syncthreads();
    for (int s = k0; s < nsteps; s++) {
        // the walker's count as of its last publish before the previous barrier (kOneBar: its
        // publish in step s - 1, by parity -- a step without a publish leaves the parity two
        // steps old, smaller than what may be consumed already: clamped, so never negative)
        const uint32_t qr = (uint32_t)__builtin_amdgcn_readfirstlane(kOneBar ? S.qn[(s - 1) & 1] : S.qn[0]);
        const uint32_t avail = umax(qr, E.qc) - E.qc;
        if (E.pend == 0) {
            if (avail != 0u && (avail >= kFetchAt || s - E.last >= APE_EMIT_EVERY)) {
                // piece L runs in the second half of step s, when the ring holds input
                // [64 (s - 13), 64 (s + 3)) (chunk s + 2 was written over s - 14 at the
                // start of step s; s + 3 overwrites s - 13 at the start of step s + 1)
                emit_fetch(S, B, lane, E, avail, s >= 12 ? 64u * (uint32_t)(s - 12) : 0u);
                E.last = s;
            }
        } else if (avail >= kEmitAll) {   // rare: never on App. C data
            emit_all(S, B, lane, E);
        } else {
            emit_step(S, B, lane, E);
        }
        STAT(2);
        if constexpr (!kOneBar) __syncthreads();
        STAT(14);
        if (E.pend == 1 || E.pend == 3) emit_step(S, B, lane, E);   // L or C
        STAT(12);
        __syncthreads();
        STAT(15);
    }
    // every record is published now (the walker's last publish preceded the last barrier);
    // the ring holds the last 16 chunks
    emit_all(S, B, lane, E);
    {
        const uint32_t rlo = B.nch > 16 ? 64u * (uint32_t)(B.nch - 16) : 0u;
        // (counts only grow: the later of the two parities is the larger)
        for (uint32_t left = (uint32_t)__builtin_amdgcn_readfirstlane(umax(S.qn[0], S.qn[1])) - E.qc; left;) {
            const uint32_t qc0 = E.qc;
            emit_fetch(S, B, lane, E, left, rlo);
            emit_all(S, B, lane, E);
            left -= E.qc - qc0;
        }
    }
    if (!E.overflow) emit_tail(S, B, lane, E);
    // ---- last literals (:732-751), from the end of the last match ----
    if (!E.overflow) {
        const uint32_t anchor = E.ein;
        const uint32_t lit = B.un - anchor;
        const uint32_t hdr = 1u + ext_bytes(lit);
        const uint32_t total = E.o + hdr + lit;
        if (total > B.cap) {
            E.overflow = true;
        } else {
            if (lane == 0) {
                B.dst[E.o] = (uint8_t)((lit < 15u ? lit : 15u) << 4);
                put_len(B.dst + E.o + 1, lit);
            }
            wave_copy(B.in, B.dst, anchor, E.o + hdr, lit, lane);
            E.o = total;
        }
    }
    if (lane == 0) *result = E.overflow ? 0 : (int)E.o;
    STAT_ADD(13, 1);
    STATS_FLUSH_TID(g_enc_stats, 128);
}

}  // namespace

// ACC: compress_fast with acceleration > 1 (its own instantiation, so the default
// kernel carries none of the probe-pattern code)
template <bool ACC>
__global__ void __launch_bounds__(192) __attribute__((amdgpu_waves_per_eu(APE_LZ4_WAVES_PER_EU)))
lz4_encode_kernel(BlockArgs a) {
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
    // compress_fast's acceleration (:789-808): the reference's probe pattern (walk_chain)
    B.noL = ACC && !APE_LZ4_ACC_L;
    B.stride = ACC ? (a.accel < (1 << 20) ? (uint32_t)a.accel : 1u << 20) : 1u;
    B.cap = (uint32_t)icap;
    B.un = (uint32_t)B.n;
    B.mstart = B.un >= 12 ? B.un - 12 : 0;   // matches start at <= n-12 (:585)
    B.mlimit = B.un >= 5 ? B.un - 5 : 0;     // and end at <= n-5 (:633)
    B.nch = (B.n + 63) / 64;

    // table = 0 (the reference's memset state: position 0 for every hash)
    for (int i = tid; i < kHSize / 8; i += 192) ((uint4 *)S.tab)[i] = make_uint4(0, 0, 0, 0);
#if !APE_LZ4_NOL
    for (int i = tid; i < (int)kScr; i += 192) S.scr[i] = 0xFFFFFFFFu;
#endif
    for (int i = tid; i < (int)(kRingE / 16 + 4); i += 192) ((uint4 *)S.ring)[i] = make_uint4(0, 0, 0, 0);
    if (tid == 0) S.qn[0] = S.qn[1] = 0u;
    __syncthreads();
    if (B.n < kSmall) encode_block<true, ACC>(S, B, wave, lane, &a.result[b]);
    else encode_block<false, ACC>(S, B, wave, lane, &a.result[b]);
}

hipError_t launch_encode(const BlockArgs &a, hipStream_t s) {
    if (a.nblocks <= 0) return hipSuccess;
    if (a.accel > 1)
        hipLaunchKernelGGL(lz4_encode_kernel<true>, dim3(a.nblocks), dim3(192), 0, s, a);
    else
        hipLaunchKernelGGL(lz4_encode_kernel<false>, dim3(a.nblocks), dim3(192), 0, s, a);
    return hipGetLastError();
}

}  // namespace apelz4
