// lz4_decode.hip -- MI355X (gfx950) batched LZ4 block decoder, bit-exact with
// APE_LZ4_decompress_safe / _safe_partial (ref src/ape_lz4.c:1275-1487).
//
// One wave (one 64-thread workgroup) decodes one independent block.  A batch
// holds ~1M blocks, so the parallelism comes from many blocks in flight, not
// from splitting a block; the kernel is instruction-issue bound, so the design
// minimises instructions per sequence and per output byte.
//
// Per block the wave alternates two phases over "batches" of <= 64 sequences:
//  PARSE  The compressed bytes of the batch are staged in LDS.  For a window of
//         64 candidate token positions P..P+63 every lane speculatively parses
//         "the sequence that would start at P+lane" (token, literal length,
//         offset, one match-length extension byte) and its successor position.
//         The true chain from P through those successors is found by binary
//         lifting (ds_bpermute rounds, no serial walk); a wave prefix-sum gives each
//         member its output position, and every member applies the reference's
//         checks (:1345-1444) in the reference's order, so the first failing
//         sequence returns the identical -(ip)-1.  Rare "complex" tokens
//         (a literal or match length needing more than one extension byte, or a
//         long literal run whose offset lies past the staged input)
//         are parsed by the scalar restatement of the reference loop instead.
//         Accepted sequences become descriptors {literal source, output
//         position, literal length, offset} in LDS.
//  COPY   One lane per sequence: the batch's output is assembled in an LDS window
//         of recent output.  Round 1: every lane writes its literal run (up to 64
//         bytes: four 16-byte units from the staged input, the last one ending
//         exactly) and its match when the match's sources precede the batch -- up to
//         four 16-byte units read from the window, or from dst history (flushed,
//         drained, read bypassing this CU's L1; issued before the literals are
//         written), or the external dictionary.  Matches whose sources lie inside the batch wait
//         for the rounds that follow: everything before the first pending sequence is
//         final, so each round copies every pending match whose sources end there.
//         Long runs, offsets < 16 inside their own output and sources straddling the
//         window start are copied by the whole wave.  The window is then flushed to
//         dst with coalesced 16-byte stores.
// Decoded blocks are not limited to 64 KiB: only the 64 KiB offset window is.
#include "lz4_gpu_internal.h"
#include <type_traits>

namespace apelz4 {

namespace {

// Output window (LDS): the batch's output is assembled in a linear window of recent
// output and flushed to dst with coalesced 16-byte stores.  When a batch would run past
// its end, the window slides: the last kKeep bytes move to its start, and everything
// older is read back from dst (flushed and drained by then).
#ifndef APE_LZ4_DWIN
#define APE_LZ4_DWIN 2048
#endif
#ifndef APE_LZ4_DKEEP
#define APE_LZ4_DKEEP 512
#endif
constexpr uint32_t kWinB = APE_LZ4_DWIN;   // output window bytes
constexpr uint32_t kKeep = APE_LZ4_DKEEP;  // history kept when the window slides
static_assert(kKeep >= 64 && kKeep % 16 == 0 && kWinB >= kKeep + 1024 && kWinB % 16 == 0,
              "output window");
#ifndef APE_LZ4_DSTAGE
#define APE_LZ4_DSTAGE 2304
#endif
constexpr int kStage = APE_LZ4_DSTAGE;   // staged compressed bytes (a multiple of 256)
constexpr int kWinNeed = 84;     // a parse window reads up to P + 63 + 21
constexpr int kBatch = 64;       // descriptors per copy batch (one per lane)
constexpr int kMaxDesc = kBatch + 44;   // held before a copy: <= 63 + 44 (two windows); a third only while nd stays <= kMaxDesc
constexpr uint32_t kLaneMax = 64;  // longest match one lane copies (4 x 16 bytes)

struct __attribute__((aligned(16))) WaveLds {
    // stage first: the parse's ds_read2_b32 (8-bit dword offsets) then needs no address add
    uint8_t stage[kStage + 16];  // src[s0 .. s0 + kStage), zero beyond the input
    uint8_t win[kWinB + 64];     // output [base, base + kWinB) (+ slack for 16-byte reads)
    uint4 desc[kMaxDesc];        // {lit_src, out, lit_len, offset}
};

// unaligned LDS accesses (gfx950 DS instructions take any byte address)
typedef uint32_t l32x4 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t l32x2 __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t l32 __attribute__((aligned(1)));
typedef uint16_t l16 __attribute__((aligned(1)));

__device__ __forceinline__ uint4 lds16(const uint8_t *p) {
    const l32x4 v = *(const l32x4 *)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void lds_st16(uint8_t *p, uint4 v) {
    l32x4 w;
    w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
    *(l32x4 *)p = w;
}
// dword k (0..3) of v
__device__ __forceinline__ uint32_t dw4(uint4 v, uint32_t k) {
    return (k & 2u) ? ((k & 1u) ? v.w : v.z) : ((k & 1u) ? v.y : v.x);
}
// Exactly n (1..15) bytes of v at p, as the pieces 8/4/2/1 of n.  A piece n lacks is
// written anyway at offset 0 (the same bytes are there) whenever n >= its size, so only
// pieces larger than n need a branch (none when MIN4 says n >= 4 and n >= 8).
template <bool MIN4>
__device__ __forceinline__ void lds_put_small(uint8_t *p, uint4 v, uint32_t n) {
    const uint32_t a4 = (n & 4u) ? (n & 8u) : 0u;
    const uint32_t a2 = (n & 2u) ? (n & 12u) : 0u;
    const uint32_t a1 = (n & 1u) ? (n & 14u) : 0u;
    if (n >= 8u) {
        l32x2 t;
        t.x = v.x; t.y = v.y;
        *(l32x2 *)p = t;
    }
    if (MIN4 || n >= 4u) *(l32 *)(p + a4) = dw4(v, a4 >> 2);
    if (MIN4 || n >= 2u) *(l16 *)(p + a2) = (uint16_t)(dw4(v, a2 >> 2) >> (8u * (a2 & 2u)));
    p[a1] = (uint8_t)(dw4(v, a1 >> 2) >> (8u * (a1 & 3u)));
}
// 16 bytes of dst history, bypassing this CU's L1 (stores of this wave reach L2 only)
__device__ __forceinline__ uint4 gload16_nt(gcu8 *p) {
    const u32x4_u v = __builtin_nontemporal_load((__attribute__((address_space(1))) const u32x4_u *)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// bytes sh..sh+3 of lo:hi (v_alignbyte; written as a 64-bit shift, the compiler kept later
// tests on the result in 64 bits)
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Compiler barrier for lane-to-lane communication through LDS inside one wave
// (the hardware executes a wave's LDS instructions in order).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Aligned dword of the compressed block at byte offset `off` (src + off is
// 4-aligned); bytes outside [0, csize) read as 0 and nothing beyond a dword that
// intersects [0, csize) is touched (a dword outside it loads the one at `first`, the
// aligned dword holding byte 0).  Loaded unconditionally and masked with selects, so
// a stage's loads are all in flight together (a branch around each load had made the
// compiler wait for every one before issuing the next).
__device__ __forceinline__ uint32_t src_dword(gcu8 *src, int csize, int off, int first) {
    const bool in = off < csize && off > -4;
    uint32_t v = *(__attribute__((address_space(1))) const uint32_t *)(src + (in ? off : first));
    const uint32_t lo = off < 0 ? 0xFFFFFFFFu << (8 * (umin((uint32_t)-off, 3u))) : 0xFFFFFFFFu;
    const uint32_t hi = off + 4 > csize ? 0xFFFFFFFFu >> (8 * umin((uint32_t)(off + 4 - csize), 3u))
                                        : 0xFFFFFFFFu;
    return in ? v & lo & hi : 0u;
}

// Stage src[s0 .. s0 + kStage) into LDS (src + s0 4-aligned; zero outside the input).
__device__ __forceinline__ void stage_load(WaveLds &L, gcu8 *src, int csize, int s0,
                                           int lane) {
    const int first = -(int)((uintptr_t)src & 3u);   // aligned dword holding byte 0
    uint32_t v[kStage / 256];
#pragma unroll
    for (int k = 0; k < kStage / 256; k++) v[k] = src_dword(src, csize, s0 + 4 * (lane + 64 * k), first);
#pragma unroll
    for (int k = 0; k < kStage / 256; k++) *(uint32_t *)&L.stage[4 * (lane + 64 * k)] = v[k];
}

// 4-aligned staging start at or below p
__device__ __forceinline__ int stage_base(gcu8 *src, int p) {
    return p - (int)((uintptr_t)(src + p) & 3u);
}

// byte p of the compressed block for the scalar path (wave-uniform p)
__device__ __forceinline__ uint32_t sbyte(const WaveLds &L, gcu8 *src, int csize, int s0,
                                          int p) {
    const uint32_t r = (uint32_t)(p - s0);
    if (r < (uint32_t)kStage) return L.stage[r];
    return p < csize ? (uint32_t)src[(uint32_t)p] : 0u;
}


}  // namespace

#ifdef APE_LZ4_STATS
__device__ unsigned long long g_dec_stats[16];
hipError_t dec_stats_read(unsigned long long *out, int reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dec_stats), sizeof(g_dec_stats));
    if (e == hipSuccess && reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_dec_stats), z, sizeof(z));
    }
    return e;
}
#endif

namespace {

struct Dec {
    gcu8 *src;
    gu8 *dst;
    gcu8 *dend;      // end of the external dictionary (DICT): history byte -k at dend - k
    uint32_t dsz;    // dictionary bytes the offset check admits: min(dictSize, 65536), 0 = none
    int csize, cap;
    int64_t oexit;
    int s0;          // staged window start
    int lane;
    uint32_t mk[5];  // mk[k]: all ones on lanes with bit k set (chain_at's lifting selects, VGPRs)
};

enum { ST_MORE = 0, ST_DONE = 1, ST_ERR = 2 };

// Scalar restatement of one iteration of the reference loop (:1324-1458) for a
// token at ip: appends its descriptor at desc[nd] (returns ST_MORE / ST_DONE) or
// reports the error (ST_ERR); `res` gets the block result when not ST_MORE.
// FASTD: decompress_fast (endOnOutputSize, :1489): the block ends where the output
// reaches cap exactly; no input-size tests (csize is only the readable bound of src);
// the result is the input consumed.
template <bool PARTIAL, bool FASTD = false>
__device__ int parse_scalar(WaveLds &L, const Dec &D, int &ip, uint32_t &op, int &nd, int &res) {
    const uint32_t tok = sbyte(L, D.src, D.csize, D.s0, ip);
    ip++;
    int64_t lit = tok >> 4;
    if (lit == 15) {  // :1331-1342
        uint32_t s;
        do {
            s = sbyte(L, D.src, D.csize, D.s0, ip);
            ip++;
            lit += s;
        } while ((FASTD || ip < D.csize - 15) && s == 255);
    }
    const int64_t cpy = (int64_t)op + lit;  // :1345-1370
    if (FASTD && (int64_t)ip + lit > D.csize) { res = -ip - 1; return ST_ERR; }  // bound
    const bool fin = FASTD ? (cpy > (int64_t)D.cap - 8)   // WILDCOPYLENGTH
                           : ((PARTIAL ? (cpy > D.oexit) : (cpy > (int64_t)D.cap - kMFLimit)) ||
                              ((int64_t)ip + lit > (int64_t)D.csize - 8));
    if (fin) {
        const bool bad = FASTD ? (cpy != D.cap)
                               : (PARTIAL ? (cpy > D.cap || (int64_t)ip + lit > D.csize)
                                          : ((int64_t)ip + lit != D.csize || cpy > D.cap));
        if (bad) { res = -ip - 1; return ST_ERR; }
        if (D.lane == 0) L.desc[nd] = make_uint4((uint32_t)ip, op, (uint32_t)lit, 0u);
        nd++;
        op = (uint32_t)cpy;
        res = FASTD ? ip + (int)lit : (int)cpy;
        return ST_DONE;
    }
    const int lit_src = ip;
    ip += (int)lit;
    if (FASTD && ip + 2 > D.csize) { res = -ip - 1; return ST_ERR; }   // bound
    const uint32_t off = sbyte(L, D.src, D.csize, D.s0, ip) |
                         (sbyte(L, D.src, D.csize, D.s0, ip + 1) << 8);  // :1373-1376
    ip += 2;
    // :1375-1376 (lowLimit = lowPrefix - dictSize; no check once dictSize >= 64 KiB)
    if (cpy + (int64_t)D.dsz - (int64_t)off < 0) { res = -ip - 1; return ST_ERR; }
    int64_t ml = tok & 15;  // :1379-1391
    if (ml == 15) {
        uint32_t s;
        do {
            if (!FASTD && ip > D.csize - kLastLiterals) { res = -ip - 1; return ST_ERR; }
            s = sbyte(L, D.src, D.csize, D.s0, ip);
            ip++;
            ml += s;
        } while (s == 255);
    }
    const int64_t mend = cpy + ml + kMinMatch;
    if (mend > (int64_t)D.cap - kLastLiterals) { res = -ip - 1; return ST_ERR; }  // :1444
    if (D.lane == 0) L.desc[nd] = make_uint4((uint32_t)lit_src, op, (uint32_t)lit, off);
    nd++;
    op = (uint32_t)mend;
    return ST_MORE;
}

// bitwise m ? a : b (v_bfi_b32)
__device__ __forceinline__ uint32_t vmux(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}

// lane l receives v of lane idx (0..63)
__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t idx) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(idx << 2), (int)v);
}

// The sequence that would start at window position rel (token at P + rel), parsed
// speculatively from the staged bytes: token, one literal-length extension byte (the
// reference's loop :1331-1342 reads exactly one when it is < 255), offset, one match-length
// extension byte, and where the next token would be.
struct Spec {
    uint32_t lit, off, ml;
    int ipl, ipo, q;                 // first literal byte, after the offset, next token
    bool fin_in, mlerr, cx;          // input ends in the literals / ml bytes run out / complex
    bool mlx;                        // match length nibble 15 (an extension byte follows)
    bool mlover;                     // ipo + kLastLiterals > csize (mlerr = mlx && mlover)
    uint32_t r1;                     // staged position after the literals (s0 + r1 = ipl + lit)
};

template <bool FASTD>
__device__ __forceinline__ Spec spec_at(const WaveLds &L, const Dec &D, int P, uint32_t rel) {
    Spec z;
    const uint32_t r = (uint32_t)(P - D.s0) + rel;
    // token and the byte after it as two byte reads (one unaligned ds_read_u16 per lane, at a
    // 1-byte lane stride, measured +7.8 % decode time; an aligned 8-byte read + funnel ties)
    const uint32_t tok = L.stage[r], e1 = L.stage[r + 1u];
    const bool litx = tok >= 0xF0u;             // literal length 15 + e1
    const uint32_t lit = litx ? 15u + e1 : tok >> 4, mn = tok & 15u;
    const uint32_t r1 = r + 1u + (litx ? 1u : 0u) + lit;   // offset bytes (then the ml byte)
    const uint32_t a1 = r1 & ~3u;
    const l32x2 w = *(const l32x2 *)&L.stage[a1];   // one ds_read_b64 (any byte address)
    const uint32_t x = funnel(w.y, w.x, r1 & 3u);
    const uint32_t e = (x >> 16) & 0xFFu;
    z.lit = lit;
    z.off = x & 0xFFFFu;
    z.ipl = P + (int)rel + 1 + (litx ? 1 : 0);
    z.ipo = z.ipl + (int)lit + 2;
    const bool mlx = mn == 15u;
    z.mlx = mlx;
    // on the staged position (s0 + r1 = ipl + lit) against a scalar limit: the same
    // compares (all values far below 2^31), without the absolute positions
    const int lim = D.csize - D.s0;   // scalar
    z.fin_in = !FASTD && (int)r1 > lim - 8;                      // ipl + lit + 8 > csize
    z.mlover = (int)r1 > lim - 2 - kLastLiterals;                  // ipo + 5 > csize
    z.mlerr = !FASTD && mlx && z.mlover;
    z.r1 = r1;
    // complex (the scalar restatement): a literal length with more than one extension byte,
    // a long literal run whose offset bytes lie past the staged input, or a match length with
    // more than one extension byte
    z.cx = (litx && (e1 == 255u || r1 + 3u > (uint32_t)kStage)) || (mlx && e == 255u && !z.mlerr);
    z.ml = mlx ? 15u + e : mn;
    z.q = z.ipo + (mlx ? 1 : 0);
    return z;
}

// The hop alone of the sequence at window position rel (chain_at): as spec_at, but the offset
// is not needed -- only the match-length extension byte, one byte read (every lane reads it,
// only a nibble-15 lane uses it; no further than spec_at's 8-byte read, and a position past the
// staged input only ever belongs to a complex lane, whose bytes do not matter).  Against the full spec_at here: -0.5 % decode time
// (profiles/r5_decoder_hop_ab.txt).
constexpr uint32_t kHopTerm = 0x200u, kHopCplx = 0x300u;   // chain_at's exit codes (below)
template <bool FASTD>
__device__ __forceinline__ uint32_t hop_at(const WaveLds &L, const Dec &D, int P, uint32_t rel) {
    const uint32_t r = (uint32_t)(P - D.s0) + rel;
    const uint32_t tok = L.stage[r], e1 = L.stage[r + 1u];
    const bool litx = tok >= 0xF0u;
    const uint32_t lit = litx ? 15u + e1 : tok >> 4;
    const bool mlx = (tok & 15u) == 15u;
    const uint32_t r1 = r + 1u + (litx ? 1u : 0u) + lit;
    const int lim = D.csize - D.s0;
    const bool fin_in = !FASTD && (int)r1 > lim - 8;
    const bool mlerr = !FASTD && mlx && (int)r1 > lim - 2 - kLastLiterals;
    const uint32_t e = L.stage[r1 + 2u];
    const bool cx = (litx && (e1 == 255u || r1 + 3u > (uint32_t)kStage)) || (mlx && e == 255u && !mlerr);
    const uint32_t qr = r1 - (uint32_t)(P - D.s0) + (mlx ? 3u : 2u);
    return cx ? kHopCplx : (fin_in ? kHopTerm : qr);
}

// The chain of sequences from window position 0 of a window at P: every lane parses
// "the sequence at P + lane" and its successor (hop).  The true chain is found by binary
// lifting instead of a serial walk: J_k = hop^(2^k) (four ds_bpermute rounds), and lane t
// composes them by the bits of t into pos = the window position of the chain's t-th
// sequence (a window holds <= 22: each sequence takes >= 3 input bytes).  cnt members
// (lanes [0, cnt)); X = the chain's exit (next token position >= 64, or kHopTerm after a
// final / failing sequence, kHopCplx before a complex token); lastp = the last member.
// A real hop is < 0x200 (63 + 1 + 1 + 269 + 2 + 1); the codes are above it.
template <bool FASTD>
__device__ __forceinline__ void chain_at(const WaveLds &L, const Dec &D, int P, uint32_t &pos,
                                         int &cnt, uint32_t &X, uint32_t &lastp) {
    // hop and the J_k hold window positions x 4: ds_bpermute's byte address (it uses
    // address bits [7:2] only), so an exit (>= 64, i.e. >= 256 here) needs no mask
    uint32_t hop;
    {
        // the hop alone: mlerr implies fin_in (ipo + 5 = ipl + lit + 7), and the successor
        // relative to P is the staged position after the literals + 2 (+1 with the ml byte)
        hop = 4u * hop_at<FASTD>(L, D, P, (uint32_t)D.lane);
    }
    // Exits absorb as a max: a real hop moves forward (J[a] > a), and an exit (>= 256) reads
    // some lane's J through the address wrap but max keeps it >= 256.  A jump from a real
    // position whose chain reaches its first exit exactly at the jump's end returns that exit
    // exactly (by induction over k: both halves of J_k are then exact), so lanes up to the
    // first exit -- the members and the exit X -- are exact; lanes past it hold some value
    // >= 256 (no member).  One v_max_u32 instead of v_cmp + v_cndmask per jump.
    auto jump = [](uint32_t J, uint32_t a) {
        const uint32_t g = (uint32_t)__builtin_amdgcn_ds_bpermute((int)a, (int)J);
        return umax(g, a);
    };
    const uint32_t J1 = jump(hop, hop);
    const uint32_t J2 = jump(J1, J1);
    const uint32_t J3 = jump(J2, J2);
    const uint32_t t = (uint32_t)D.lane;
    // lane t takes J_k where bit k of t is set: a v_bfi on a per-lane VGPR mask each (the
    // lane masks had been hoisted into SGPR pairs, and the SGPR file spilled them to VGPR
    // lanes: two v_readlane to reload one, inside the parse loop)
    uint32_t p = vmux(D.mk[0], lane_val(hop, 0), 0u);
    p = vmux(D.mk[1], jump(J1, p), p);
    p = vmux(D.mk[2], jump(J2, p), p);
    p = vmux(D.mk[3], jump(J3, p), p);
    const uint32_t p15 = lane_val(p, 15);
    // lanes 16..31 take J^16, or the exit p15 when the chain has no member 15 (lanes >= 32
    // are no members); J^16 and its two dependent rounds only when needed (wave-uniform)
    uint32_t sel = p15;
    if (p15 < 256u) {
        const uint32_t J4 = jump(J3, J3);
        sel = jump(J4, p);
    }
    p = vmux(D.mk[4], sel, p);
    p >>= 2;
    pos = t < 32u ? p : kHopTerm;
    cnt = __popcll(wave_ballot(pos < 64u));
    X = lane_val(pos, cnt);
    lastp = lane_val(pos, cnt - 1);
}

// Up to three speculative windows (P, then where each chain leaves the last, if that is
// staged and the members fit) and one pass over their members: appends the descriptors
// (<= 63, and nd stays <= kMaxDesc).  Returns
// ST_MORE with P advanced (to the next token, or to a complex token when `cplx`), or
// ST_DONE / ST_ERR with `res`.  Members are lanes [0, nm) in chain order: lane t re-reads
// its sequence from the staged bytes.
template <bool PARTIAL, bool DICT, bool FASTD = false>
__device__ int parse_window(WaveLds &L, const Dec &D, int &P, uint32_t &op, int &nd, int &res,
                            bool &cplx) {
    const int lane = D.lane;
    const uint32_t t = (uint32_t)lane;
    uint32_t posA, XA, lastA;
    int cntA;
    chain_at<FASTD>(L, D, P, posA, cntA, XA, lastA);
    const bool cplxA = XA == kHopCplx;
    // the complex token is not a member.  (XA is wave-uniform and is 64..0x1FF, kHopTerm
    // 0x200 or kHopCplx 0x300: bits 9 and 8 both set only for kHopCplx -- scalar arithmetic,
    // where a select on the bool was materialised in a VGPR)
    static_assert(kHopCplx == 0x300u && kHopTerm == 0x200u, "hop exit codes");
    const int nmA = cntA - (int)((XA >> 9) & (XA >> 8) & 1u);
    const int PB = P + (int)XA;
    const bool two = XA < kHopTerm && PB - D.s0 + kWinNeed <= kStage;
    int nmB = 0, nmC = 0, Pn, PC = PB;
    uint32_t posB = 0, posC = 0;
    if (two) {
        uint32_t XB, lastB;
        int cntB;
        chain_at<FASTD>(L, D, PB, posB, cntB, XB, lastB);
        nmB = cntB - (int)((XB >> 9) & (XB >> 8) & 1u);   // (as nmA)
        PC = PB + (int)XB;
        // a third window while the members still fit the wave (<= 41 + 22 lanes) and the
        // descriptors the array (nd + nm <= kMaxDesc), and its bytes are staged
        const bool three = XB < kHopTerm && nmA + nmB <= 41 && nd + nmA + nmB <= kMaxDesc - 22 &&
                           PC - D.s0 + kWinNeed <= kStage;
        if (three) {
            uint32_t XC, lastC;
            int cntC;
            chain_at<FASTD>(L, D, PC, posC, cntC, XC, lastC);
            cplx = XC == kHopCplx;
            nmC = cntC - (int)((XC >> 9) & (XC >> 8) & 1u);
            Pn = PC + (int)(XC >= kHopTerm ? lastC : XC);
        } else {
            cplx = XB == kHopCplx;
            Pn = PB + (int)(XB >= kHopTerm ? lastB : XB);   // (not past a final token)
        }
    } else {
        cplx = cplxA;
        Pn = P + (int)(XA >= kHopTerm ? lastA : XA);
    }
    const uint32_t pB = bperm(posB, (t - (uint32_t)nmA) & 63u);
    const int nmAB = nmA + nmB;
    const int nm = nmAB + nmC;
    const uint64_t M = (1ull << nm) - 1ull;   // nm <= 63
    const bool mem = (int)t < nm;
    uint32_t pos = (int)t < nmA ? posA : (uint32_t)(PB - P) + pB;   // relative to P
    if (nmC) {
        const uint32_t pC = bperm(posC, (t - (uint32_t)nmAB) & 63u);
        pos = (int)t < nmAB ? pos : (uint32_t)(PC - P) + pC;
    }

    // member t = the sequence at P + pos, re-read from the staged bytes
    const Spec z = spec_at<FASTD>(L, D, P, mem ? pos : 0u);
    const uint32_t lit = z.lit, ml = z.ml, off = z.off;
    const int ipl = z.ipl, ipo = z.ipo, q = z.q;
    const bool fin_in = z.fin_in;
    // output positions, checks in the reference's order
    const uint32_t ob = mem ? (fin_in ? lit : lit + ml + kMinMatch) : 0u;
    const uint32_t ex = wave_excl_scan(ob);
    const uint32_t opl = op + ex;
    // The checks of :1345-1447 in the reference's order, as selects (no divergent
    // branches).  32-bit unsigned arithmetic is exact here: cap, csize > 0, a window
    // token has lit < 270 and ml < 274, and op + ex stays far below 2^32.
    const uint32_t cpy = opl + lit, ucap = (uint32_t)D.cap;
    const uint32_t iend = (uint32_t)ipl + lit;  // input position after the literals
    // FASTD (:1346-1366 with endOnOutputSize): final once the literals pass cap - 8,
    // valid only when they end exactly at cap; the result is the input consumed
    // (every condition is a wave mask of single compares: a ballot of an OR / AND of
    // compares, or a bool kept across a select, was materialised as 0/1 and compared again)
    uint64_t fm, badfm;   // final sequence; a final one that fails
    if (FASTD) {
        fm = wave_ballot(cpy + 8u > ucap);
        badfm = wave_ballot(cpy != ucap);
    } else if (PARTIAL) {
        fm = wave_ballot(fin_in) | wave_ballot((int64_t)cpy > D.oexit);
        badfm = wave_ballot(cpy > ucap) | wave_ballot(iend > (uint32_t)D.csize);
    } else {
        // cpy + 12 > cap as cpy >= a scalar bound; iend != csize on the staged position
        const uint32_t capA = ucap > (uint32_t)kMFLimit - 1u ? ucap - ((uint32_t)kMFLimit - 1u) : 0u;
        fm = wave_ballot(fin_in) | wave_ballot(cpy >= capA);
        badfm = wave_ballot(z.r1 != (uint32_t)(D.csize - D.s0)) | wave_ballot(cpy > ucap);
    }
    const bool fin = lane_in(fm);
    const uint64_t mlm = FASTD ? 0ull : wave_ballot(z.mlx) & wave_ballot(z.mlover);
    const bool e_off = (DICT ? cpy + D.dsz : cpy) < off;               // :1375-1376
    // FASTD: the bytes a sequence needs must lie inside the readable bound (the reference
    // has no bound and reads on; here that is an error, never a read past the buffer)
    const bool e_in = FASTD && (fin ? iend > (uint32_t)D.csize
                                    : (uint32_t)q > (uint32_t)D.csize);
    const bool e_cap = cpy + ml + (uint32_t)(kMinMatch + kLastLiterals) > ucap;   // :1444
    // stop = fin || e_off || mlerr || e_cap || e_in; bad = fin ? badfin || e_in : stop
    // (ballots of the single conditions, combined as wave masks: no per-lane 0/1)
    const uint64_t om = wave_ballot(e_off) | mlm;   // stops at the offset / ml bytes
    const uint64_t inm = FASTD ? wave_ballot(e_in) : 0ull;
    const uint64_t stm = fm | om | wave_ballot(e_cap) | inm;
    const uint64_t badm = (fm & (badfm | inm)) | (~fm & stm);
    const uint64_t sm = M & stm;
    uint64_t emit = M;
    int st = ST_MORE;
    if (sm) {
        const int T = __ffsll((long long)sm) - 1;
        const bool tbad = (badm >> T) & 1ull;
        // the result of the stopping sequence T, formed only here (a per-lane select chain
        // on every pass had become a divergent branch that re-materialised the masks):
        // final: bad ? -(ip)-1 : output size (FASTD: input consumed); otherwise -(ip)-1 at
        // the offset / ml bytes or after the sequence
        if ((fm >> T) & 1ull)
            res = tbad ? -(int)lane_val((uint32_t)ipl, T) - 1
                       : (int)lane_val(FASTD ? iend : cpy, T);
        else
            res = ((om >> T) & 1ull) ? -(int)lane_val((uint32_t)ipo, T) - 1
                                     : -(int)lane_val((uint32_t)q, T) - 1;
        // members before T (error) or up to T (final literals)
        emit = tbad ? ((1ull << T) - 1ull) : ((2ull << T) - 1ull);   // T <= 62
        st = tbad ? ST_ERR : ST_DONE;
        cplx = false;
    }
    if (st != ST_ERR) {
        const int ne = __popcll(emit);
        if ((int)t < ne) L.desc[nd + lane] = make_uint4((uint32_t)ipl, opl, lit, fin ? 0u : off);
        nd += ne;
        if (ne) {
            // a final sequence's size is its literals (ob assumed a match unless the
            // input ended: a PARTIAL or FASTD stop by output size ends the block too)
            op = lane_val(opl + (fin ? lit : ob), ne - 1);
        }
    }
    if (st == ST_MORE) P = Pn;
    return st;
}

// ---------------- copy: descriptors -> output window -> dst ----------------
// The window holds output positions [base, base + kWinB); dst[0, fl) is flushed and
// dst[0, gdone) flushed and drained (readable as history; gdone >= base + kKeep - 15
// once the window has slid, so every position below base is readable from dst).
struct Win {
    uint32_t base, fl, gdone;
};

// Literal run of one sequence, copied by the whole wave: n bytes from input position
// src to output position at (16-byte units; the last unit ends exactly at n and
// overlaps its neighbour with the same bytes, so nothing outside [at, at + n) is written).
__device__ __forceinline__ void coop_literal(WaveLds &L, const Dec &D, uint32_t base, uint32_t at,
                                             uint32_t n, uint32_t src) {
    const int lane = D.lane;
    uint8_t *w = L.win + (at - base);
    const uint32_t rs = src - (uint32_t)D.s0;
    const bool staged = rs < (uint32_t)kStage && rs + n <= (uint32_t)kStage;   // wave-uniform
    if (n >= 16u) {
        for (uint32_t t = 16u * (uint32_t)lane; t < n; t += 1024u) {
            const uint32_t tt = umin(t, n - 16u);
            const uint4 v = staged ? lds16(L.stage + rs + tt) : gload16(D.src + (src + tt));
            lds_st16(w + tt, v);
        }
    } else if ((uint32_t)lane < n) {
        w[lane] = staged ? L.stage[rs + lane] : D.src[src + (uint32_t)lane];
    }
}

// Match of one sequence copied by the whole wave, 64 bytes per pass in order (every
// source precedes its byte: offset >= 64 reads earlier passes, a shorter offset reads
// the match's first period).  Sources: the window (>= base), dst history (< base) or
// the external dictionary (< 0).  Used for what the lane path does not take: long
// matches, offsets < 16 inside their own output, sources straddling the window start.
template <bool DICT>
__device__ __forceinline__ void coop_match(WaveLds &L, const Dec &D, uint32_t base, uint32_t ma,
                                        uint32_t n, uint32_t off) {
    const int lane = D.lane;
    uint8_t *w = L.win + (ma - base);
    if (off == 0u) {   // offset 0 decodes as zero bytes
        for (uint32_t t = (uint32_t)lane; t < n; t += 64u) w[t] = 0;
        return;
    }
    const bool per = off < 64u;                     // wave-uniform
    uint32_t r = per ? (uint32_t)lane % off : 0u;   // (t - ma) mod off for t = lane
    const uint32_t inc = per ? 64u % off : 0u;
    for (uint32_t t0 = 0; t0 < n; t0 += 64u) {
        const uint32_t t = t0 + (uint32_t)lane;
        if (t < n) {
            const int sp = per ? (int)ma - (int)off + (int)r : (int)(ma + t) - (int)off;
            uint32_t v;
            if (sp >= (int)base) v = L.win[(uint32_t)sp - base];
            else if (DICT && sp < 0) v = D.dend[sp];
            else v = __builtin_nontemporal_load(D.dst + sp);
            w[t] = (uint8_t)v;
        }
        r += inc;
        r = r >= off ? r - off : r;
        wave_sync();
    }
}

// Match of this lane's sequence (n <= 64 bytes at output ma, offset off), for the
// lanes with `go`: up to four 16-byte units (the last one ends exactly at n), read
// first and then written when the sources precede ma, unit after unit when the match
// overlaps itself (offset 16..n-1), or exactly n bytes when n < 16.  `glb`: the source
// is dst history / the dictionary instead of the window.
template <bool DICT>
__device__ __forceinline__ void lane_match(WaveLds &L, const Dec &D, uint32_t base, bool go,
                                           uint32_t ma, uint32_t n, uint32_t off, bool glb) {
    if (!go) return;
    uint8_t *w = L.win + (ma - base);
    const int ps = (int)ma - (int)off;
    const bool big = n >= 16u;
    // Only the units a lane needs: unit k (k = 1..3) exists when n > 16 k.  Lanes whose
    // match is shorter issue no load for it, so a gather instruction touches only the lines
    // its active lanes need (the texture path's cost is per line: tools/ubench/gather_rate).
    // The units a lane does not need stay unset (never stored): no v_mov per unit and call,
    // and no unit waits for another's load.
    const uint32_t t1 = umin(16u, n - 16u), t2 = umin(32u, n - 16u), t3 = n - 16u;
    const bool u1 = n > 16u, u2 = n > 32u, u3 = n > 48u;
    uint4 v0, v1, v2, v3;
    if (off != 0u && off < n) {   // overlaps itself (off >= 16, n > 16): unit after unit
        const uint8_t *s = L.win + ((uint32_t)ps - base);
        lds_st16(w, lds16(s));
        if (u1) lds_st16(w + t1, lds16(s + t1));
        if (u2) lds_st16(w + t2, lds16(s + t2));
        if (u3) lds_st16(w + t3, lds16(s + t3));
        return;
    }
    if (!glb) {   // (offset 0: in-window bytes, zeroed below)
        const uint8_t *s = L.win + ((uint32_t)ps - base);
        v0 = lds16(s);
        if (u1) v1 = lds16(s + t1);
        if (u2) v2 = lds16(s + t2);
        if (u3) v3 = lds16(s + t3);
    } else if (!DICT) {
        // dst history (ps >= 0): 32-bit offsets from the scalar base (global_load's SGPR-base
        // form), no 64-bit address adds
        gcu8 *d = (gcu8 *)D.dst;
        const uint32_t o0 = (uint32_t)ps;
        v0 = gload16_nt(d + o0);
        if (u1) v1 = gload16_nt(d + (o0 + t1));
        if (u2) v2 = gload16_nt(d + (o0 + t2));
        if (u3) v3 = gload16_nt(d + (o0 + t3));
    } else {
        gcu8 *s = ps < 0 ? D.dend + ps : (gcu8 *)D.dst + ps;
        v0 = gload16_nt(s);
        if (u1) v1 = gload16_nt(s + t1);
        if (u2) v2 = gload16_nt(s + t2);
        if (u3) v3 = gload16_nt(s + t3);
    }
    if (off == 0u) v0 = v1 = v2 = v3 = make_uint4(0, 0, 0, 0);
    if (big) {
        lds_st16(w, v0);
        if (u1) lds_st16(w + t1, v1);
        if (u2) lds_st16(w + t2, v2);
        if (u3) lds_st16(w + t3, v3);
    } else {
        lds_put_small<true>(w, v0, n);
    }
}

// Round 1 in two halves: the sources are read (window or dst history / dictionary) before the
// segment's literals are written, and stored after them, so the history loads' latency overlaps
// the literal copies.  (A round-1 source lies before the segment: no literal overwrites it.)
// Measured -1.1 % decode time (131072 blocks, medians of 9).
struct MLoad {
    uint4 v0, v1, v2, v3;
};
template <bool DICT>
__device__ __forceinline__ void lane_match_load(WaveLds &L, const Dec &D, uint32_t base, bool go,
                                                uint32_t ma, uint32_t n, uint32_t off, bool glb,
                                                MLoad &u) {
    if (!go || (off != 0u && off < n)) return;   // (self-overlap: all in the store half)
    const int ps = (int)ma - (int)off;
    const uint32_t t1 = umin(16u, n - 16u), t2 = umin(32u, n - 16u), t3 = n - 16u;
    const bool u1 = n > 16u, u2 = n > 32u, u3 = n > 48u;
    if (!glb) {
        const uint8_t *s = L.win + ((uint32_t)ps - base);
        u.v0 = lds16(s);
        if (u1) u.v1 = lds16(s + t1);
        if (u2) u.v2 = lds16(s + t2);
        if (u3) u.v3 = lds16(s + t3);
    } else if (!DICT) {
        gcu8 *d = (gcu8 *)D.dst;
        const uint32_t o0 = (uint32_t)ps;
        u.v0 = gload16_nt(d + o0);
        if (u1) u.v1 = gload16_nt(d + (o0 + t1));
        if (u2) u.v2 = gload16_nt(d + (o0 + t2));
        if (u3) u.v3 = gload16_nt(d + (o0 + t3));
    } else {
        gcu8 *s = ps < 0 ? D.dend + ps : (gcu8 *)D.dst + ps;
        u.v0 = gload16_nt(s);
        if (u1) u.v1 = gload16_nt(s + t1);
        if (u2) u.v2 = gload16_nt(s + t2);
        if (u3) u.v3 = gload16_nt(s + t3);
    }
}
__device__ __forceinline__ void lane_match_store(WaveLds &L, uint32_t base, bool go, uint32_t ma,
                                                 uint32_t n, uint32_t off, MLoad &u) {
    if (!go) return;
    uint8_t *w = L.win + (ma - base);
    const int ps = (int)ma - (int)off;
    const uint32_t t1 = umin(16u, n - 16u), t2 = umin(32u, n - 16u), t3 = n - 16u;
    const bool u1 = n > 16u, u2 = n > 32u, u3 = n > 48u;
    if (off != 0u && off < n) {   // overlaps itself (off >= 16, n > 16): unit after unit
        const uint8_t *s = L.win + ((uint32_t)ps - base);
        lds_st16(w, lds16(s));
        if (u1) lds_st16(w + t1, lds16(s + t1));
        if (u2) lds_st16(w + t2, lds16(s + t2));
        if (u3) lds_st16(w + t3, lds16(s + t3));
        return;
    }
    if (off == 0u) u.v0 = u.v1 = u.v2 = u.v3 = make_uint4(0, 0, 0, 0);
    if (n >= 16u) {
        lds_st16(w, u.v0);
        if (u1) lds_st16(w + t1, u.v1);
        if (u2) lds_st16(w + t2, u.v2);
        if (u3) lds_st16(w + t3, u.v3);
    } else {
        lds_put_small<true>(w, u.v0, n);
    }
}

// Copy sub-phase timers (diagnostic stats build only): cycles of the slides, the segment's
// ballots + literals, round 1, the dependent passes and the flushes.
#ifdef APE_LZ4_STATS
#define SUB_P , uint64_t *sub_
#define SUB_A , sub_
#define SUB_START uint64_t sub_t_ = clock64();
#define SUB_MARK(i) do { const uint64_t t_ = clock64(); sub_[i] += t_ - sub_t_; sub_t_ = t_; } while (0)
#else
#define SUB_P
#define SUB_A
#define SUB_START
#define SUB_MARK(i) do {} while (0)
#endif

// Per-lane sequence of the batch: literal [o, m) from input ls, match [m, me) at offset off.
struct Seq {
    uint32_t o, m, me, ls, off;
};

// Produce output [S0, S1) of the batch in the window.  Literals first (a lane each when
// short and staged, the whole wave for the others), then round 1: every match whose
// sources lie before S0.  The remaining matches read output of this segment: each finds
// the sequences owning its source range (binary search over the sequence starts) and runs
// in the first pass after all of them are done.  A pass with nothing ready means the first
// pending sequence is a whole-wave item (everything before it is done): it runs then.
template <bool DICT>
__device__ __forceinline__ void copy_segment(WaveLds &L, const Dec &D, const Win &W, const Seq &q,
                                             uint32_t S0, uint32_t S1, uint32_t &diag SUB_P) {
    SUB_START
    const int lane = D.lane;
    const uint32_t base = W.base;
    const uint32_t la = umax(q.o, S0), lb = umin(q.m, S1);
    const uint32_t nl = lb > la ? lb - la : 0u;
    const uint32_t lsrc = q.ls + (la - q.o);
    const uint32_t ma = umax(q.m, S0), mb = umin(q.me, S1);
    const uint32_t nm = mb > ma ? mb - ma : 0u;
    uint32_t off = q.off;
    // opaque per segment: compares on it stay here (the loop-invariant ones, hoisted out of
    // the segment loop, were kept as per-lane bools and re-materialised as 0/1 + v_cmp)
    asm volatile("" : "+v"(off));
    const int ps = (int)ma - (int)off;
    // Every condition below is a wave mask of single compares (a ballot of an AND / OR of
    // compares, or a bool kept across a select, was materialised as 0/1 and compared again).
    // literal: lane path when short and staged
    const uint32_t rs = lsrc - (uint32_t)D.s0;
    const uint64_t nlm = wave_ballot(nl != 0u);
    // (literal runs up to 64 bytes: a lane each, as a match; 16 had been the limit -- runs of
    // 17..64 then took a whole-wave copy each: -3.1 % decode time with 64, -2.6 % with 32)
    const uint64_t litm = nlm & wave_ballot(nl <= 64u) & wave_ballot(rs < (uint32_t)kStage) &
                          wave_ballot(rs + nl <= (uint32_t)kStage);
    // match: lane path (window / dst history / dictionary sources, or a self-overlap with
    // offset >= 16 inside the window; a match cut by a segment edge can be shorter than 4)
    // or the whole wave; pe = end of the sources it needs from this segment
    const uint64_t off0m = wave_ballot(off == 0u);
    const uint64_t ovlm = ~off0m & wave_ballot(off < nm);
    const int pe0 = ps + (int)nm;
    const uint64_t inwm = wave_ballot(ps >= (int)base);
    uint64_t ingm = wave_ballot(pe0 <= (int)W.gdone) &
                    (wave_ballot(nm >= 16u) | wave_ballot(ps + 16 <= D.cap));
    if (DICT) ingm &= wave_ballot(ps >= 0);
    const uint64_t indm = DICT ? wave_ballot(ps + (int)umax(nm, 16u) <= 0) : 0ull;
    const uint64_t lpnm = inwm | ingm | indm;
    const uint64_t lpom = wave_ballot(off >= 16u) & inwm;
    const uint64_t lenm = wave_ballot(nm >= 4u) & wave_ballot(nm <= kLaneMax);
    const uint64_t lpm = lenm & (off0m | (ovlm & lpom) | (~ovlm & lpnm));
    const bool glb = lane_in(~off0m & ~inwm);
    const int pe = lane_in(off0m) ? -0x7FFFFFFF : (lane_in(ovlm) ? (int)ma : pe0);
    const uint64_t mpm = wave_ballot(nm != 0u);
    const uint64_t r1m = mpm & lpm & wave_ballot(pe <= (int)S0);
    MLoad r1u;
    lane_match_load<DICT>(L, D, base, lane_in(r1m), ma, nm, off, glb, r1u);

    // literals
    for (uint64_t lc = nlm & ~litm; lc; lc &= lc - 1ull) {
        const int f = __builtin_ctzll(lc);
        coop_literal(L, D, base, lane_val(la, f), lane_val(nl, f), lane_val(lsrc, f));
    }
    wave_sync();
    if (lane_in(litm)) {   // up to four 16-byte units, the last one ending exactly at nl
        uint8_t *w = L.win + (la - base);
        const uint8_t *sp = L.stage + rs;
        const uint4 v = lds16(sp);
        if (nl >= 16u) {
            const uint32_t t1 = umin(16u, nl - 16u), t2 = umin(32u, nl - 16u), t3 = nl - 16u;
            uint4 v1, v2, v3;
            if (nl > 16u) v1 = lds16(sp + t1);
            if (nl > 32u) v2 = lds16(sp + t2);
            if (nl > 48u) v3 = lds16(sp + t3);
            lds_st16(w, v);
            if (nl > 16u) lds_st16(w + t1, v1);
            if (nl > 32u) lds_st16(w + t2, v2);
            if (nl > 48u) lds_st16(w + t3, v3);
        } else {
            lds_put_small<false>(w, v, nl);
        }
    }
    // round 1
    SUB_MARK(1);
    lane_match_store(L, base, lane_in(r1m), ma, nm, off, r1u);
    uint64_t pm = mpm & ~r1m;
    SUB_MARK(2);
    if (!pm) return;
    // sequences owning [max(ps, S0), pe): k0 = owner(first byte), k1 = owner(last byte),
    // by binary search over the sequence starts (lanes past the batch hold B1)
    const uint32_t x0 = (uint32_t)(ps > (int)S0 ? ps : (int)S0), x1 = (uint32_t)(pe - 1);
    uint32_t k0 = 0, k1 = 0;
#pragma unroll
    for (uint32_t st = 32; st >= 1; st >>= 1) {
        const uint32_t c0 = k0 + st, c1 = k1 + st;
        const uint32_t v0 = bperm(q.o, c0), v1 = bperm(q.o, c1);
        k0 = v0 <= x0 ? c0 : k0;
        k1 = v1 <= x1 ? c1 : k1;
    }
    k1 = umin(k1, (uint32_t)lane - 1u);   // (its own literal is written; lane 0 has no needs)
    const uint64_t need = (lane_in(pm) && lane > 0 && k0 <= k1)
                              ? (((2ull << k1) - 1ull) & ~((1ull << k0) - 1ull)) : 0ull;
    uint64_t done = ~pm;   // lanes still pending = pm & ~done
    wave_sync();
    for (;;) {
        diag += 1u;
        const uint64_t gm = pm & ~done & lpm & wave_ballot((need & ~done) == 0ull);
        if (gm) {
            lane_match<DICT>(L, D, base, lane_in(gm), ma, nm, off, glb);
            done |= gm;
        } else {   // the first pending sequence is a whole-wave item, and its sources are done
            const int f = __builtin_ctzll(pm & ~done);
            diag += 0x10000u;
            coop_match<DICT>(L, D, base, lane_val(ma, f), lane_val(nm, f), lane_val(off, f));
            done |= 1ull << f;
        }
        if (!(pm & ~done)) break;
        wave_sync();
    }
    SUB_MARK(3);
}

// Write window bytes [fl, F1) to dst: F1 = S1 rounded down to a 16-byte dst address
// (the rest waits for the next flush), or S1 itself at the end of the block.
__device__ __forceinline__ void flush(WaveLds &L, const Dec &D, Win &W, uint32_t S1, bool fin) {
    const int lane = D.lane;
    const uint32_t da = (uint32_t)(uintptr_t)D.dst & 15u;
    const uint32_t F0 = W.fl;
    const uint32_t sa = (S1 + da) & ~15u;
    const uint32_t F1 = fin ? S1 : (sa > da ? sa - da : 0u);
    if ((int)F1 <= (int)F0) return;
    const uint32_t h = umin(((F0 + da + 15u) & ~15u) - da, F1);   // first 16-byte dst address
    const uint32_t ta = (F1 + da) & ~15u;                          // last one
    const uint32_t t = umax(ta > da ? ta - da : 0u, h);
    const uint32_t base = W.base;
    wave_sync();
    if (lane < 16) {
        const uint32_t x = F0 + (uint32_t)lane;
        if (x < h) D.dst[x] = L.win[x - base];
    } else if (lane < 32) {
        const uint32_t x = t + (uint32_t)lane - 16u;
        if (x < F1) D.dst[x] = L.win[x - base];
    }
    for (uint32_t c = h + 16u * (uint32_t)lane; c < t; c += 1024u)
        gstore16(D.dst + c, lds16(L.win + (c - base)));
    W.fl = F1;
}

// Slide the window to start at nb (a multiple of 16, <= S0 - kKeep): output [nb, S0)
// moves to the window start; dst is drained, so everything below nb reads from dst.
__device__ __forceinline__ void slide(WaveLds &L, const Dec &D, Win &W, uint32_t nb, uint32_t S0) {
    const uint32_t from = nb - W.base, len = S0 - nb;   // len <= kKeep + 15
    constexpr int kU = (int)((kKeep + 16u + 1023u) / 1024u);
    uint4 v[kU];
    wave_sync();
#pragma unroll
    for (int k = 0; k < kU; k++) {
        const uint32_t x = 16u * (uint32_t)D.lane + 1024u * (uint32_t)k;
        if (x < len) v[k] = lds16(L.win + from + x);
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < kU; k++) {
        const uint32_t x = 16u * (uint32_t)D.lane + 1024u * (uint32_t)k;
        if (x < len) lds_st16(L.win + x, v[k]);
    }
    wave_sync();
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    W.gdone = W.fl;
    W.base = nb;
}

// Copy the batch's output [B0, B1) (nd descriptors) through the window to dst.
template <bool DICT>
__device__ __forceinline__ void copy_batch(WaveLds &L, const Dec &D, Win &W, int nd, uint32_t B0,
                                           uint32_t B1, bool last, uint32_t &diag SUB_P) {
    const int lane = D.lane;
    wave_sync();
    const bool has = lane < nd;
    const uint4 d = L.desc[has ? lane : 0];
    const uint32_t nxt = lane + 1 < nd ? L.desc[lane + 1].y : B1;
    Seq q;
    q.o = has ? d.y : B1;
    q.m = has ? d.y + d.z : B1;
    q.me = has ? nxt : B1;
    q.ls = d.x;
    q.off = d.w;
    for (uint32_t S0 = B0; S0 < B1;) {
        if (B1 > W.base + kWinB && S0 >= W.base + kKeep + 16u) {
            SUB_START
            slide(L, D, W, (S0 - kKeep) & ~15u, S0);
            SUB_MARK(0);
            diag += 1u << 24;
        }
        const uint32_t S1 = umin(B1, W.base + kWinB);
        copy_segment<DICT>(L, D, W, q, S0, S1, diag SUB_A);
        {
            SUB_START
            flush(L, D, W, S1, last && S1 == B1);
            SUB_MARK(4);
        }
        S0 = S1;
    }
    if (last) flush(L, D, W, B1, true);
}

}  // namespace

// One block (block index b of the batch) decoded by the calling wave.
template <bool PARTIAL, bool DICT, bool FASTD>
__device__ __forceinline__ void decode_block(WaveLds &L, const BlockArgs &a, const int b,
                                             const int lane) {
    Dec D;
    D.dst = (gu8 *)(a.dst ? a.dst[b] : a.dst_base + (size_t)b * a.dst_stride);
    if (a.frame_off) {   // framed stream: [le32 size][block] (lz4_frame.hip)
        // The header is untrusted: it must fit the frame the offsets give (ref
        // src/ape_socket.c:1382-1384 rejects a size above the data it has).  A frame
        // shorter than its header, or a size < 0 or past the next frame, is malformed:
        // -1, nothing read beyond the frame, nothing written.
        const long long f0 = a.frame_off[b], avail = a.frame_off[b + 1] - f0 - 4;
        int hdr = -1;
        gcu8 *f = (gcu8 *)(a.src_base + f0);
        if (avail >= 0)
            hdr = (int)((uint32_t)f[0] | ((uint32_t)f[1] << 8) | ((uint32_t)f[2] << 16) |
                        ((uint32_t)f[3] << 24));
        if (hdr < 0 || (long long)hdr > avail) {
            if (lane == 0) a.result[b] = -1;
            return;
        }
        D.csize = hdr;
        D.src = f + 4;
    } else {
        D.src = (gcu8 *)(a.src ? a.src[b] : a.src_base + (size_t)b * a.src_stride);
        D.csize = a.src_size[b];
    }
    D.cap = a.dst_cap ? a.dst_cap[b] : (int)a.dst_stride;
    D.oexit = PARTIAL ? a.target[b] : 0;
    if (PARTIAL && D.oexit > (int64_t)D.cap - kMFLimit) D.oexit = (int64_t)D.cap - kMFLimit;
    D.lane = lane;
    for (int k = 0; k < 5; ++k) {
        uint32_t m = 0u - (((uint32_t)lane >> k) & 1u);
        asm volatile("" : "+v"(m));   // opaque: stays a VGPR mask, not turned back into a select
        D.mk[k] = m;
    }
    D.dend = nullptr;
    D.dsz = 0;
    if (DICT) {   // usingDict (:1625-1647): any placement, adjacent or not, reads the same
        const int ds = a.dict_size[b] > 0 ? a.dict_size[b] : 0;
        D.dend = (gcu8 *)a.dict[b] + ds;
        D.dsz = ds < 65536 ? (uint32_t)ds : 65536u;
    }

    // Special cases of :1316-1318 and the empty-input quirk (the reference reads
    // src[0] even when compressedSize <= 0).
    if (FASTD && (D.cap == 0 || D.csize <= 0)) {   // :1321-1322 (and no readable input)
        if (lane == 0) a.result[b] = (D.cap == 0 && D.csize > 0 && D.src[0] == 0) ? 1 : -1;
        return;
    }
    if (D.cap == 0 || D.csize <= 0) {
        if (lane == 0) {
            int r;
            if (D.cap == 0) r = (D.csize == 1 && D.src[0] == 0) ? 0 : -1;
            else r = ((D.src ? D.src[0] : 0u) >= 0xF0) ? -3 : -2;
            a.result[b] = r;
        }
        return;
    }

    // One literal run holding the whole block (incompressible input, e.g. SURVEY config 2):
    // the reference reads the token and its length bytes (:1329-1342), then takes the final-
    // literals branch (:1346-1366): ret = the run if it ends exactly at csize and fits cap,
    // else -(ip)-1.  Here the length bytes are scanned 64 at a time and the run is copied
    // global -> global, 16 bytes per lane, without the LDS staging or the output window.
    if (!PARTIAL && !FASTD && !DICT && D.csize >= 32 && D.cap > 0 && D.src[0] >= 0xF0u) {
        // bytes 1.. while 255 and ip < csize - 15 after the read (:1334-1337): J = the last
        // one read; all before it are 255
        int J = 0;
        for (int base = 1;; base += 64) {
            const int i = base + lane;
            const uint32_t byte = D.src[i < D.csize ? i : D.csize - 1];   // (never past src)
            const bool stop = i + 1 >= D.csize - 15 || byte != 255u;
            const uint64_t m = wave_ballot(stop);
            if (m) {
                J = base + __builtin_ctzll(m);
                break;
            }
        }
        const long long L = 15ll + 255ll * (J - 1) + (long long)D.src[J];
        if ((long long)J + 1 + L == (long long)D.csize) {
            if (L > (long long)D.cap) {
                if (lane == 0) a.result[b] = -(J + 1) - 1;
                return;
            }
            gcu8 *s = D.src + J + 1;
            gu8 *d = D.dst;
            const int n16 = (int)(L >> 4);
            int k = lane;
            for (; k + 192 < n16; k += 256) {   // four 16-byte loads in flight per lane
                const uint4 v0 = gload16(s + 16 * k), v1 = gload16(s + 16 * (k + 64));
                const uint4 v2 = gload16(s + 16 * (k + 128)), v3 = gload16(s + 16 * (k + 192));
                gstore16(d + 16 * k, v0);
                gstore16(d + 16 * (k + 64), v1);
                gstore16(d + 16 * (k + 128), v2);
                gstore16(d + 16 * (k + 192), v3);
            }
            for (; k < n16; k += 64) gstore16(d + 16 * k, gload16(s + 16 * k));
            for (int i = 16 * n16 + lane; i < (int)L; i += 64) d[i] = s[i];
            if (lane == 0) a.result[b] = (int)L;
            return;
        }
    }

    STATS_DECL
#ifdef APE_LZ4_STATS
    uint64_t sub_[5] = {0, 0, 0, 0, 0};
#endif
    int P = 0;               // next token (wave-uniform)
    uint32_t op = 0;         // its output position
    int result = 0;
    int st = ST_MORE;
    if (lane < 4) *(uint32_t *)&L.stage[kStage + 4 * lane] = 0u;  // over-read pad
    D.s0 = stage_base(D.src, 0);
    stage_load(L, D.src, D.csize, D.s0, lane);
    wave_sync();
    if (D.cap < 0) {
        // oend < dest in the reference: the first sequence's literals already pass it,
        // so its final-literals test fails (:1345-1366) -> -(ip)-1 after the token and
        // its length bytes.  The scalar restatement computes exactly that (64-bit
        // compares) and writes nothing; the window parser's unsigned cap would not.
        int ip = 0, nd = 0;
        uint32_t op0 = 0;
        (void)parse_scalar<PARTIAL, FASTD>(L, D, ip, op0, nd, result);
        if (lane == 0) a.result[b] = result;
        return;
    }

    // Per batch: parse until >= 64 descriptors are held (nd <= kMaxDesc after a step), then
    // produce the output of the first 64 through the LDS window (copy_batch) and carry
    // the rest.  A failing sequence ends the block without copying its batch (the result
    // is the error; dst bytes are unspecified then).
    Win W;
    W.base = 0;
    W.fl = 0;
    W.gdone = 0;
    int nd = 0;              // descriptors held (carried ones first)
    uint32_t cst = 0;        // output position of desc[0]
    for (;;) {
        // ---- PARSE ----
        // one exit (a loop with several breaks was structurised into flag phis: s_mov /
        // s_cselect of 64-bit masks per pass); a complex token may jump far past the staged
        // bytes, which the loop condition then sees.  (restage may now also hold with nd >= 64:
        // every descriptor is copied before the restage, as at any restage)
        while (st == ST_MORE && nd < kBatch && P - D.s0 + kWinNeed <= kStage) {
            bool cplx;
            st = parse_window<PARTIAL, DICT, FASTD>(L, D, P, op, nd, result, cplx);
            if (st == ST_MORE && cplx) st = parse_scalar<PARTIAL, FASTD>(L, D, P, op, nd, result);
        }
        const bool restage = st == ST_MORE && P - D.s0 + kWinNeed > kStage;
        STAT(0);
        if (st == ST_ERR) break;
        // ---- COPY: batches of <= 64 descriptors; all of them before a restage (their
        // literals are staged) or at the end ----
        do {
            const int nc = nd < kBatch ? nd : kBatch;
            wave_sync();
            const uint32_t B1 = nc < nd ? (uint32_t)__builtin_amdgcn_readfirstlane(L.desc[nc].y) : op;
            const bool last = st == ST_DONE && nc == nd;
            uint32_t diag = 0;
            copy_batch<DICT>(L, D, W, nc, cst, B1, last, diag SUB_A);
            STAT_ADD(3, diag & 0xFFFFu);          // wave passes after round 1
            STAT_ADD(5, (diag >> 16) & 0xFFu);    // coop matches
            STAT_ADD(6, diag >> 24);              // window slides
            STAT_ADD(2, 1);
            cst = B1;
            if (nc < nd) {   // carry desc[nc, nd) -> desc[0, nd - nc)
                wave_sync();
                const uint4 dv = L.desc[nc + (lane < nd - nc ? lane : 0)];
                wave_sync();
                if (lane < nd - nc) L.desc[lane] = dv;
            }
            nd -= nc;
        } while (nd > 0 && (restage || st != ST_MORE));
        STAT(1);
        if (st != ST_MORE) break;
        if (restage) {
            wave_sync();
            D.s0 = stage_base(D.src, P);
            stage_load(L, D.src, D.csize, D.s0, lane);
            wave_sync();
            STAT_ADD(4, 1);
        }
    }
    if (lane == 0) a.result[b] = result;
    STAT_ADD(10, 1);
#ifdef APE_LZ4_STATS
    STAT_ADD(7, sub_[0]);    // slides
    STAT_ADD(8, sub_[1]);    // segment ballots + literals
    STAT_ADD(9, sub_[2]);    // round 1
    STAT_ADD(11, sub_[3]);   // dependent passes
    STAT_ADD(12, sub_[4]);   // flushes
#endif
    STATS_FLUSH(g_dec_stats);
}

template <bool PARTIAL, bool DICT, bool FASTD>
__global__ void __launch_bounds__(64)
lz4_decode_kernel(BlockArgs a) {
    __shared__ WaveLds L;
    decode_block<PARTIAL, DICT, FASTD>(L, a, (int)blockIdx.x, (int)threadIdx.x);
}

// Chained streams (lz4_sock.hip): workgroup i decodes chunks i, i + nconn, i + 2 nconn, ...
// in order -- chunk q + 1 of a connection takes the output of chunks <= q as its dictionary
// -- so a round of nq chunk positions is one launch instead of nq.  Between chunks, the
// wave's stores are made visible to its own loads (release, then acquire with the L1
// invalidated).
__global__ void __launch_bounds__(64)
lz4_decode_chain_kernel(BlockArgs a, int nconn, int nq) {
    __shared__ WaveLds L;
    for (int q = 0; q < nq; q++) {
        decode_block<false, true, false>(L, a, q * nconn + (int)blockIdx.x, (int)threadIdx.x);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
}


hipError_t launch_decode_chain(const BlockArgs &a, int nconn, int nq, hipStream_t s) {
    if (nconn <= 0 || nq <= 0) return hipSuccess;
    hipLaunchKernelGGL(lz4_decode_chain_kernel, dim3(nconn), dim3(64), 0, s, a, nconn, nq);
    return hipGetLastError();
}

hipError_t launch_decode(const BlockArgs &a, bool partial, hipStream_t s) {
    if (a.nblocks <= 0) return hipSuccess;
    if (a.fast)   // decompress_fast (ref :1489)
        hipLaunchKernelGGL((lz4_decode_kernel<false, false, true>), dim3(a.nblocks), dim3(64), 0, s, a);
    else if (a.dict)   // usingDict decodes are full decodes (ref :1625-1647)
        hipLaunchKernelGGL((lz4_decode_kernel<false, true, false>), dim3(a.nblocks), dim3(64), 0, s, a);
    else if (partial)
        hipLaunchKernelGGL((lz4_decode_kernel<true, false, false>), dim3(a.nblocks), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL((lz4_decode_kernel<false, false, false>), dim3(a.nblocks), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace apelz4
