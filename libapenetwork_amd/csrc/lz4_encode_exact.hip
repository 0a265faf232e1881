// lz4_encode_exact.hip -- greedy-exact GPU encode mode ("reproduces
// LZ4_compress_generic byte-for-byte (slow, for debugging)").
//
// N x APE_LZ4_compress_fast (ref src/ape_lz4.c:789-808 -> :758-786 -> LZ4_compress_generic
// :530-755 with byU16 / noDict, the only table type a <= 64 KiB block takes, :766), byte for
// byte and with the same return value, limitedOutput's early exits included.  The parse is
// the reference's own sequential one, so the block is not parallelised: one wave per block,
// the block and the 8192-entry u16 position table in LDS (80 KiB: two blocks per CU), the
// wave walking the parse in lockstep with every value wave-uniform (scalar registers), and
// the lanes used only where the reference loops over bytes: LZ4_count (:359-385) as 64-byte
// compares + a ballot, literal copies, the table reset and the block load.
//
// Not the product path: APE_LZ4_compress_batch_dev's encoders parse in parallel and are
// 2-3 orders of magnitude faster; this mode exists to produce the reference's exact bytes
// on the device (debugging, diffing a GPU pipeline against a CPU one).
#include "lz4_gpu_internal.h"

namespace apelz4 {
namespace {

constexpr int kXHashLog = 13;                   // byU16: LZ4_HASHLOG + 1 (:393, :459)
constexpr int kXTable = 1 << kXHashLog;
constexpr int kXSkipTrigger = 6;                // LZ4_skipTrigger (:399)
constexpr uint64_t kXPrime5 = 889523592379ull;  // prime5bytes (:456)

struct ExactLds {
    uint8_t blk[kMaxBlock];
    uint16_t tbl[kXTable];
};
static_assert(2 * sizeof(ExactLds) <= 160 * 1024, "two blocks per CU");

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// LE32 of the block at byte p (any alignment; gfx950 LDS reads take unaligned addresses)
__device__ __forceinline__ uint32_t rd32(const ExactLds &S, uint32_t p) {
    return uni(*(const u32_u *)(S.blk + p));
}

// LZ4_hashPosition for byU16 on a 64-bit build (:457-462, :470-473): bits 27..39 of the
// 64-bit product of the 8 bytes at p and prime5bytes -- they depend on the first 5 bytes only
__device__ __forceinline__ uint32_t xhash(const ExactLds &S, uint32_t p) {
    const uint64_t v = (uint64_t)rd32(S, p) | ((uint64_t)uni(S.blk[p + 4]) << 32);
    return (uint32_t)((v * kXPrime5) >> (40 - kXHashLog)) & (uint32_t)(kXTable - 1);
}

}  // namespace

__global__ void __launch_bounds__(64) lz4_encode_exact_kernel(BlockArgs a) {
    __shared__ ExactLds S;
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const char *srcp = a.src ? a.src[b] : a.src_base + (size_t)b * a.src_stride;
    char *dstp = a.dst ? a.dst[b] : a.dst_base + (size_t)b * a.dst_stride;
    const int n = a.src_size[b];
    const int cap = a.dst_cap ? a.dst_cap[b] : (int)a.dst_stride;
    // (U32)inputSize > LZ4_MAX_INPUT_SIZE -> 0 (:564-565); a block over the GPU limit:
    // ERANGE as every batch encoder; a negative cap: 0 (the reference compares it as U32
    // in its last-literals check and writes an unbounded buffer there)
    if (n < 0 || n > kMaxBlock || cap < 0) {
        if (lane == 0) a.result[b] = n > kMaxBlock ? kErange : 0;
        return;
    }

    // ---- block -> LDS (16-byte loads, byte tail), table reset (APE_LZ4_resetStream, :760) ----
    {
        gcu8 *g = (gcu8 *)srcp;
        const int n16 = n >> 4;
        for (int i = lane; i < n16; i += 64) *(uint4 *)(S.blk + 16 * i) = gload16(g + 16 * i);
        for (int i = (n16 << 4) + lane; i < n; i += 64) S.blk[i] = g[i];
        for (int i = lane; i < kXTable / 2; i += 64) ((uint32_t *)S.tbl)[i] = 0u;
    }
    __syncthreads();

    gu8 *d = (gu8 *)dstp;
    auto put = [&](uint32_t o, uint32_t v) {   // one output byte (the wave's lane 0)
        if (lane == 0) d[o] = (uint8_t)v;
    };
    auto copy = [&](uint32_t o, uint32_t s, uint32_t len) {   // literals, lanes in parallel
        for (uint32_t j = (uint32_t)lane; j < len; j += 64u) d[o + j] = S.blk[s + j];
    };
    auto settbl = [&](uint32_t h, uint32_t p) {   // LZ4_putPositionOnHash (:485-497)
        if (lane == 0) S.tbl[h] = (uint16_t)p;   // one wave: its LDS ops stay in order
    };
    auto gettbl = [&](uint32_t h) -> uint32_t { return uni(S.tbl[h]); };
    auto byte = [&](uint32_t p) -> uint32_t { return uni(S.blk[p]); };

    const uint32_t un = (uint32_t)n;
    const uint32_t bound = un + un / 255u + 16u;     // APE_LZ4_compressBound (:768)
    const bool limited = (uint32_t)cap < bound;       // :764
    const uint32_t olimit = (uint32_t)cap;
    uint32_t op = 0, anchor = 0;
    bool fail = false;

    if (n >= kMinLength) {                            // else: all literals (:577-578)
        const uint32_t mflimit = un - (uint32_t)kMFLimit, matchlimit = un - (uint32_t)kLastLiterals;
        const uint32_t accel = a.accel < 1 ? 1u : (uint32_t)a.accel;   // :762

        // LZ4_count (:359-385): the matching bytes at p and m, stopping at lim
        auto count = [&](uint32_t p, uint32_t m, uint32_t lim) -> uint32_t {
            for (uint32_t c = 0;; c += 64u) {
                const uint32_t i = c + (uint32_t)lane;
                const bool out = p + i >= lim;
                const uint32_t pa = out ? p : p + i, ma = out ? m : m + i;
                const uint64_t mk = wave_ballot(out || S.blk[pa] != S.blk[ma]);
                if (mk) return c + (uint32_t)__builtin_ctzll(mk);
            }
        };

        settbl(xhash(S, 0), 0);                       // first byte (:581-583)
        uint32_t ip = 1, forwardH = xhash(S, 1);
        bool done = false;
        while (!done && !fail) {
            uint32_t match = 0;
            {   // find a match (:591-619)
                uint32_t forwardIp = ip, step = 1, searchMatchNb = accel << kXSkipTrigger;
                bool last = false;
                for (;;) {
                    const uint32_t h = forwardH;
                    ip = forwardIp;
                    forwardIp += step;
                    step = searchMatchNb++ >> kXSkipTrigger;
                    if (forwardIp > mflimit) { last = true; break; }
                    match = gettbl(h);
                    forwardH = xhash(S, forwardIp);
                    settbl(h, ip);
                    if (rd32(S, match) == rd32(S, ip)) break;
                }
                if (last) break;                      // -> last literals
            }
            // catch up (:623-627)
            while (ip > anchor && match > 0u && byte(ip - 1u) == byte(match - 1u)) {
                ip--;
                match--;
            }
            // literal length + literals (:630-651)
            const uint32_t lit = ip - anchor;
            uint32_t token = op++;
            if (limited && op + lit + (2u + 1u + (uint32_t)kLastLiterals) + lit / 255u > olimit) {
                fail = true;
                break;
            }
            uint32_t tokv;
            if (lit >= 15u) {
                tokv = 15u << 4;
                uint32_t len = lit - 15u;
                for (; len >= 255u; len -= 255u) put(op++, 255u);
                put(op++, len);
            } else {
                tokv = lit << 4;
            }
            copy(op, anchor, lit);
            op += lit;
            for (;;) {   // _next_match (:653-729)
                const uint32_t off = ip - match;
                put(op, off & 255u);
                put(op + 1u, off >> 8);
                op += 2u;
                uint32_t ml = count(ip + (uint32_t)kMinMatch, match + (uint32_t)kMinMatch, matchlimit);
                ip += (uint32_t)kMinMatch + ml;
                if (limited && op + (1u + (uint32_t)kLastLiterals) + (ml >> 8) > olimit) {
                    fail = true;
                    break;
                }
                if (ml >= 15u) {
                    tokv += 15u;
                    ml -= 15u;
                    for (; ml >= 510u; ml -= 510u) {
                        put(op++, 255u);
                        put(op++, 255u);
                    }
                    if (ml >= 255u) {
                        ml -= 255u;
                        put(op++, 255u);
                    }
                    put(op++, ml);
                } else {
                    tokv += ml;
                }
                put(token, tokv);
                anchor = ip;
                if (ip > mflimit) { done = true; break; }   // :704
                settbl(xhash(S, ip - 2u), ip - 2u);          // :707
                const uint32_t h = xhash(S, ip);             // :710-721
                match = gettbl(h);
                settbl(h, ip);
                if (rd32(S, match) == rd32(S, ip)) {
                    token = op++;
                    tokv = 0u;
                    continue;
                }
                forwardH = xhash(S, ++ip);                   // :728
                break;
            }
        }
    }
    int result = 0;
    if (!fail) {   // last literals (:732-751)
        const uint32_t lastRun = un - anchor;
        if (!(limited && op + lastRun + 1u + (lastRun + 255u - 15u) / 255u > olimit)) {
            if (lastRun >= 15u) {
                put(op++, 15u << 4);
                uint32_t acc = lastRun - 15u;
                for (; acc >= 255u; acc -= 255u) put(op++, 255u);
                put(op++, acc);
            } else {
                put(op++, lastRun << 4);
            }
            copy(op, anchor, lastRun);
            op += lastRun;
            result = (int)op;
        }
    }
    if (lane == 0) a.result[b] = result;
}

hipError_t launch_encode_exact(const BlockArgs &a, hipStream_t s) {
    if (a.nblocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(lz4_encode_exact_kernel, dim3(a.nblocks), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace apelz4
