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
//         The scalar unit then follows the true chain from P through those
//         successors (one v_readlane per sequence); a wave prefix-sum gives each
//         member its output position, and every member applies the reference's
//         checks (:1345-1444) in the reference's order, so the first failing
//         sequence returns the identical -(ip)-1.  Rare "complex" tokens
//         (literal length >= 15, or a match length needing > 1 extension byte)
//         are parsed by the scalar restatement of the reference loop instead.
//         Accepted sequences become descriptors {literal source, output
//         position, literal length, offset} in LDS.
//  COPY   The batch's output is produced in 256-byte steps, 4 bytes per lane.
//         A byte is a literal (staged compressed bytes, or the block in HBM for
//         long literal runs), or a match byte whose source -- reduced modulo the
//         offset to lie before the match -- is older than `gdone` (stored to dst
//         and drained by vmcnt(0): read back bypassing this CU's L1), newer (the
//         LDS history ring), or inside this step (resolved through the step's
//         owner map).  Output goes to the ring and straight to dst.
// Decoded blocks are not limited to 64 KiB: only the 64 KiB offset window is.
#include "lz4_gpu_internal.h"
#include <type_traits>

namespace apelz4 {

namespace {

#ifndef APE_LZ4_DRING
#define APE_LZ4_DRING 1024
#endif
constexpr int kRing = APE_LZ4_DRING;  // per-wave history ring (bytes, power of two)
constexpr int kStage = 2304;     // staged compressed bytes per batch (9 dwords/lane)
constexpr int kWinNeed = 84;     // a parse window reads up to P + 63 + 21
constexpr int kStep = 256;       // output bytes per copy step (4 per lane)
constexpr int kMaxDesc = 64;     // descriptors per batch
constexpr int kFlushAt = 40;     // copy once a batch holds more than this (window adds <= 22)
constexpr int kMaxCarry = 24;    // descriptors carried into the next batch (< kFlushAt)

struct __attribute__((aligned(16))) WaveLds {
    uint8_t ring[kRing];
    uint8_t stage[kStage + 16];  // src[s0 .. s0 + kStage), zero beyond the input
    uint4 desc[kMaxDesc];        // {lit_src, out, lit_len, offset}
    uint32_t own[kStep / 4];     // owner map of the current step (u8 per byte)
};



__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * sh));
}

// Compiler barrier for lane-to-lane communication through LDS inside one wave
// (the hardware executes a wave's LDS instructions in order).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Aligned dword of the compressed block at byte offset `off` (src + off is
// 4-aligned); bytes outside [0, csize) read as 0 and nothing beyond that dword
// (which cannot cross a page) is touched.
__device__ __forceinline__ uint32_t src_dword(gcu8 *src, int csize, int off) {
    if (off >= csize || off <= -4) return 0u;
    uint32_t v = *(__attribute__((address_space(1))) const uint32_t *)(src + off);
    if (off < 0) v &= 0xFFFFFFFFu << (8 * (-off));
    if (off + 4 > csize) v &= 0xFFFFFFFFu >> (8 * (off + 4 - csize));
    return v;
}

// Stage src[s0 .. s0 + kStage) into LDS (src + s0 4-aligned; zero outside the input).
__device__ __forceinline__ void stage_load(WaveLds &L, gcu8 *src, int csize, int s0,
                                           int lane) {
    uint32_t v[kStage / 256];
#pragma unroll
    for (int k = 0; k < kStage / 256; k++) v[k] = src_dword(src, csize, s0 + 4 * (lane + 64 * k));
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

// One speculative window at P (P - s0 + kWinNeed <= kStage): appends the
// chain's descriptors.  Returns ST_MORE with P advanced (to the next token, or
// to a complex token when `cplx`), or ST_DONE / ST_ERR with `res`.
template <bool PARTIAL, bool DICT, bool FASTD = false>
__device__ int parse_window(WaveLds &L, const Dec &D, int &P, uint32_t &op, int &nd, int &res,
                            bool &cplx) {
    const int lane = D.lane;
    const uint32_t r = (uint32_t)(P - D.s0 + lane);
    const uint32_t tok = L.stage[r];
    const uint32_t lit = tok >> 4, mn = tok & 15u;
    const uint32_t r1 = r + 1u + lit;           // offset bytes (then the ml byte)
    const uint32_t a1 = r1 & ~3u;
    const uint32_t x = funnel(*(const uint32_t *)&L.stage[a1 + 4], *(const uint32_t *)&L.stage[a1],
                              r1 & 3u);
    const uint32_t off = x & 0xFFFFu, e = (x >> 16) & 0xFFu;
    const int p = P + lane;
    const int ipl = p + 1;                       // first literal byte
    const int ipo = ipl + (int)lit + 2;          // after the offset
    const bool fin_in = !FASTD && (uint32_t)ipl + lit + 8u > (uint32_t)D.csize;   // ipl >= 1
    const bool mlx = mn == 15u;
    const bool mlerr = !FASTD && mlx && ipo + kLastLiterals > D.csize;
    const bool cx = lit == 15u || (mlx && e == 255u && !mlerr);
    const uint32_t ml = mlx ? 15u + e : mn;
    const int q = ipo + (mlx ? 1 : 0);           // next token
    // hop to the next token (relative to P); a final / failing sequence ends the
    // chain (kHopTerm), a complex token ends it before itself (kHopCplx)
    constexpr uint32_t kHopTerm = 0x80u, kHopCplx = 0xC0u;
    const uint32_t hop = cx ? kHopCplx : ((fin_in || mlerr) ? kHopTerm : (uint32_t)(q - P));

    // follow the chain from P (scalar: one v_readlane per sequence, 4 instructions)
    uint32_t c = 0, last = 0;
    uint64_t M = 0;
    do {
        last = c;
        M |= 1ull << c;
        c = (uint32_t)__builtin_amdgcn_readlane((int)hop, (int)c);
    } while (c < 64u);
    cplx = c == kHopCplx;
    if (cplx) M &= ~(1ull << last);           // the complex token is not a member
    if (c >= kHopTerm) c = last;              // (P is not advanced past a final token)
    // output positions, checks in the reference's order
    const bool mem = (M >> lane) & 1ull;
    const uint32_t ob = mem ? (fin_in ? lit : lit + ml + kMinMatch) : 0u;
    const uint32_t ex = wave_excl_scan(ob);
    const uint32_t opl = op + ex;
    // The checks of :1345-1447 in the reference's order, as selects (no divergent
    // branches).  32-bit unsigned arithmetic is exact here: cap, csize > 0, a window
    // token has lit < 15 and ml < 274, and op + ex stays far below 2^32.
    const uint32_t cpy = opl + lit, ucap = (uint32_t)D.cap;
    const uint32_t iend = (uint32_t)ipl + lit;  // input position after the literals
    // FASTD (:1346-1366 with endOnOutputSize): final once the literals pass cap - 8,
    // valid only when they end exactly at cap; the result is the input consumed
    const bool fin = FASTD ? (cpy + 8u > ucap)
                           : (fin_in || (PARTIAL ? ((int64_t)cpy > D.oexit)
                                                 : (cpy + (uint32_t)kMFLimit > ucap)));
    const bool badfin = FASTD ? (cpy != ucap)
                              : (PARTIAL ? (cpy > ucap || iend > (uint32_t)D.csize)
                                         : (iend != (uint32_t)D.csize || cpy > ucap));
    const bool e_off = (DICT ? cpy + D.dsz : cpy) < off;               // :1375-1376
    // FASTD: the bytes a sequence needs must lie inside the readable bound (the reference
    // has no bound and reads on; here that is an error, never a read past the buffer)
    const bool e_in = FASTD && (fin ? iend > (uint32_t)D.csize
                                    : (uint32_t)q > (uint32_t)D.csize);
    const bool e_cap = cpy + ml + (uint32_t)(kMinMatch + kLastLiterals) > ucap;   // :1444
    const bool stop = fin || e_off || mlerr || e_cap || e_in;
    const bool bad = fin ? (badfin || e_in) : stop;
    const int rv = fin ? ((badfin || e_in) ? -ipl - 1 : (int)(FASTD ? iend : cpy))
                       : ((e_off || mlerr) ? -ipo - 1 : -q - 1);
    const uint64_t sm = wave_ballot(mem && stop) & M;
    uint64_t emit = M;
    int st = ST_MORE;
    if (sm) {
        const int T = __ffsll((long long)sm) - 1;
        res = (int)lane_val((uint32_t)rv, T);
        const bool tbad = lane_val(bad ? 1u : 0u, T) != 0u;
        // members before T (error) or up to T (final literals)
        if (tbad) emit = M & ((1ull << T) - 1ull);
        else emit = M & (T == 63 ? ~0ull : ((2ull << T) - 1ull));
        st = tbad ? ST_ERR : ST_DONE;
        cplx = false;
    }
    if (st != ST_ERR) {
        if ((emit >> lane) & 1ull) {
            const uint32_t idx = (uint32_t)nd + __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(emit >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)emit, 0u));
            L.desc[idx] = make_uint4((uint32_t)ipl, opl, lit, fin ? 0u : off);
        }
        nd += __popcll(emit);
        if (emit) {
            const int last = 63 - __clzll((long long)emit);
            // a final sequence's size is its literals (ob assumed a match unless the
            // input ended: a PARTIAL or FASTD stop by output size ends the block too)
            op = lane_val(opl + (fin ? lit : ob), last);
        }
    }
    if (st == ST_MORE) P += (int)c;
    return st;
}

// x mod off for x < off + 3 (three conditional subtractions cover off = 1)
__device__ __forceinline__ uint32_t reduce3(uint32_t x, uint32_t off) {
    x = x >= off ? x - off : x;
    x = x >= off ? x - off : x;
    return x >= off ? x - off : x;
}

// Produce output [lo, hi) of the step at `base` from the batch's descriptors.
// Branch-light: every byte gets an LDS address and (rarely) an HBM pointer; loads
// are guarded by wave-uniform tests only, so the wave does not juggle exec masks.
template <bool DICT>
__device__ __forceinline__ void copy_step(WaveLds &L, const Dec &D, uint32_t base, uint32_t lo,
                                          uint32_t hi, uint32_t gdone, int nd, uint32_t d_out,
                                          uint32_t &diag) {
    const int lane = D.lane;
    // owner map: mark descriptor starts inside (lo, hi); the one covering lo carries in
    const uint32_t cur = (uint32_t)__popcll(wave_ballot(d_out <= lo)) - 1u;   // d_out = ~0 past nd
    L.own[lane] = 0u;
    wave_sync();
    if (d_out - lo - 1u < hi - lo - 1u) ((uint8_t *)L.own)[d_out - base] = (uint8_t)(lane + 1);  // lo < d_out < hi
    wave_sync();
    const uint32_t m = L.own[lane];
    const uint32_t run = umax(umax(m & 0xFFu, (m >> 8) & 0xFFu), umax((m >> 16) & 0xFFu, m >> 24));
    const uint32_t pre = umax(wave_shr1(wave_incl_max(run), 0u), cur + 1u);
    const uint32_t A = pre - 1u;
    const bool hasB = A + 1u < (uint32_t)nd;
    const uint4 dA = L.desc[A];
    const uint4 dB = L.desc[hasB ? A + 1u : A];
    const uint32_t outB = hasB ? dB.y : 0xFFFFFFFFu;
    const uint32_t leA = dA.y + dA.z, leB = dB.y + dB.z;
    const uint32_t xlA = dA.x - dA.y, xlB = dB.x - dB.y;   // literal source - output
    const uint32_t offA = dA.w, offB = dB.w;
    const uint32_t s0 = (uint32_t)D.s0;
    const uint32_t q0 = base + 4u * (uint32_t)lane;

    // offset of byte 0 inside A's match period (one division, only if some lane needs it)
    uint32_t rA = q0 - leA;                       // valid when q0 >= leA
    const bool needmod = q0 >= leA && offA != 0u && rA >= offA;
    if (wave_any(needmod)) {
        diag |= 1u;
        if (needmod) rA %= offA;
    }

    // per byte: source position, LDS address (kNone = a zero byte), HBM kind (1 src,
    // 2 dst, 3 dictionary).  Two wave-uniform specialisations: FULL (the step is
    // produced whole: no range test) and SO (some lane's offset is 1..3: its period
    // needs up to three reductions; otherwise one conditional subtraction covers
    // rA + j < off + 3 and q - le <= 2).
    constexpr uint32_t kNone = (uint32_t)offsetof(WaveLds, stage) + (uint32_t)kStage;
    uint32_t pos[4], lad[4], gk[4];
    uint32_t pendm = 0;
    bool anyg = false;
    auto bytes = [&](auto so_t, auto full_t) {
        constexpr bool SO = decltype(so_t)::value, FU = decltype(full_t)::value;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            // Every arm is computed into a variable first and the ternaries only pick
            // between plain values: the compiler then emits v_cndmask selects, not the
            // divergent branches (exec-mask juggling on the scalar unit) that nested
            // ternaries with arithmetic in their arms become.
            const uint32_t q = q0 + j;
            const bool inB = q >= outB;
            const uint32_t le = inB ? leB : leA, off = inB ? offB : offA, xl = inB ? xlB : xlA;
            const bool lit = q < le;
            const uint32_t mbB = q - leB, mbA0 = rA + j, mbA1 = q - leA;
            const uint32_t mbA = q0 >= leA ? mbA0 : mbA1;
            const uint32_t mb = inB ? mbB : mbA;
            const uint32_t red = SO ? reduce3(mb, off) : umin(mb, mb - off);
            const uint32_t mpos = le - off + red;
            const uint32_t lpos = q + xl;
            const uint32_t ps = lit ? lpos : mpos;
            const bool live = (FU || (q >= lo && q < hi)) && (lit || off != 0u);  // offset 0 -> 0
            const bool inst = ps - s0 < (uint32_t)kStage;
            // DICT: a match source before the block start ("negative" ps) is in the dictionary
            const bool hist = DICT && ps >= 0x80000000u;
            const bool ring = !lit && !hist && ps >= gdone && ps < lo;
            const bool pend = live && !lit && !hist && ps >= lo;
            const uint32_t a_st = ps - s0 + (uint32_t)offsetof(WaveLds, stage), a_rg = ps & (kRing - 1);
            const uint32_t a_lit = inst ? a_st : kNone, a_mat = ring ? a_rg : kNone;
            const uint32_t a_live = lit ? a_lit : a_mat;
            pos[j] = ps;
            lad[j] = live ? a_live : kNone;
            const uint32_t g_old = ps < gdone ? 2u : 0u;
            const uint32_t g_lit = inst ? 0u : 1u, g_mat = hist ? 3u : g_old;
            const uint32_t g_live = lit ? g_lit : g_mat;
            gk[j] = (live && !pend) ? g_live : 0u;
            anyg |= gk[j] != 0u;
            pendm |= pend ? 1u << j : 0u;
        }
    };
    const bool so = offA - 1u < 3u || offB - 1u < 3u;
    const bool full = lo == base && hi == base + kStep;
    if (wave_any(so)) {
        if (full) bytes(std::true_type{}, std::true_type{});
        else bytes(std::true_type{}, std::false_type{});
    } else {
        if (full) bytes(std::false_type{}, std::true_type{});
        else bytes(std::false_type{}, std::false_type{});
    }
    // fetch: LDS for every byte, HBM only if a lane needs it (an in-step source
    // reads 0 here and is filled in below)
    const uint8_t *lds = (const uint8_t *)&L;
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) v[j] = lds[lad[j]];   // kNone reads 0
    if (wave_any(anyg)) {
        diag |= 0x10000u;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            // one nontemporal byte load for both sources (history in dst must bypass
            // this CU's L1; the literal in src does not care); idle lanes read src[0].
            // A/B (tools/dec_variants.sh, 65536 blocks): device-scope loads that allocate
            // in L2 fetch as much (the history misses L2 either way: ~1000 blocks per XCD
            // stream their output through its 4 MB) and take 12% longer.
            gcu8 *bp = gk[j] == 2u ? (gcu8 *)D.dst : D.src;
            const uint32_t o = gk[j] != 0u ? pos[j] : 0u;
            if (DICT && gk[j] == 3u) bp = D.dend - 0x100000000ll;   // dend + (int32)o
            const uint32_t g = __builtin_nontemporal_load(bp + o);
            v[j] = gk[j] != 0u ? g : v[j];
        }
    }
    // In-step sources.  A pending byte's source (already reduced into the match's first
    // period) is an earlier byte of this step.  The step's resolved bytes go to the
    // ring, with a done flag per byte in the (no longer needed) owner map; each pass
    // then copies every pending byte whose source is done.  Sources strictly precede
    // their bytes, so each pass resolves at least the lowest pending byte of the step,
    // and one pass usually resolves all.  No byte of this step reads the ring slots it
    // overwrites (ring sources lie in [gdone, lo), and lo - gdone <= 512).
#ifdef APE_DEXP_NOPEND
    if (false) {   // diagnostic: instruction count without in-step sources (wrong bytes)
#else
    if (wave_any(pendm != 0)) {
#endif
        diag |= 2u;
        uint8_t *ring = L.ring;
        uint8_t *done = (uint8_t *)L.own;
        wave_sync();
        uint32_t dw = 0;
        if (lo == base && hi == base + kStep) {   // whole step: one dword (pending bytes 0)
            *(uint32_t *)&ring[q0 & (kRing - 1)] = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t q = q0 + j;
                if (q >= lo && q < hi) ring[q & (kRing - 1)] = (uint8_t)v[j];
            }
        }
#pragma unroll
        for (int j = 0; j < 4; j++) dw |= ((pendm >> j) & 1u) ? 0u : 1u << (8 * j);
        L.own[lane] = dw;
        wave_sync();
        while (wave_any(pendm != 0)) {
            diag += 4u;
            uint32_t now = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t src = pos[j];
                const bool pj = (pendm >> j) & 1u;
                const uint32_t dn = done[pj ? src - base : 0u];
                const uint32_t val = ring[src & (kRing - 1)];
                const bool ok = pj && dn != 0u;
                v[j] = ok ? val : v[j];
                now |= ok ? 1u << j : 0u;
            }
            wave_sync();
#pragma unroll
            for (int j = 0; j < 4; j++) {
                if ((now >> j) & 1u) {
                    const uint32_t q = q0 + j;
                    ring[q & (kRing - 1)] = (uint8_t)v[j];
                    done[q - base] = 1u;
                }
            }
            pendm &= ~now;
            wave_sync();
        }
    }
    const uint32_t word = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
    wave_sync();
    // store: ring and dst (the whole-step case is uniform)
    gu8 *o8 = D.dst + q0;
    if (lo == base && hi == base + kStep) {
        *(uint32_t *)&L.ring[q0 & (kRing - 1)] = word;
        if ((((uintptr_t)(D.dst + base)) & 3u) == 0) {
            *(__attribute__((address_space(1))) uint32_t *)o8 = word;
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) o8[j] = (uint8_t)(word >> (8 * j));
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t q = q0 + j;
            if (q >= lo && q < hi) {
                L.ring[q & (kRing - 1)] = (uint8_t)(word >> (8 * j));
                o8[j] = (uint8_t)(word >> (8 * j));
            }
        }
    }
}

}  // namespace

template <bool PARTIAL, bool DICT, bool FASTD>
__global__ void __launch_bounds__(64)
lz4_decode_kernel(BlockArgs a) {
    __shared__ WaveLds L;
    const int b = blockIdx.x;
    const int lane = threadIdx.x;

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

    STATS_DECL
    int P = 0;               // next token (wave-uniform)
    uint32_t op = 0;         // its output position
    uint32_t gdone = 0;      // dst[0, gdone) stored and drained
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

    // Output is copied in whole 256-byte steps: a batch copies up to the last step
    // boundary its sequences reach and carries the descriptors of the unfinished
    // step into the next batch (the last batch copies everything), so each step is
    // produced once instead of once per batch that touches it.
    uint32_t cstart = 0;     // output [0, cstart) copied
    int nd = 0;              // descriptors in L.desc (carried ones first)
    while (st == ST_MORE) {
        // ---- PARSE one batch ----
        bool restage = false;
        while (st == ST_MORE && nd <= kFlushAt) {
            if (P - D.s0 + kWinNeed > kStage) { restage = true; break; }
            bool cplx;
            st = parse_window<PARTIAL, DICT, FASTD>(L, D, P, op, nd, result, cplx);
            if (st == ST_MORE && cplx) {
                st = parse_scalar<PARTIAL, FASTD>(L, D, P, op, nd, result);
                // a complex token may jump far past the staged bytes
                if (st == ST_MORE && P - D.s0 + kWinNeed > kStage) { restage = true; break; }
            }
        }
        STAT(0);
        if (st == ST_ERR) break;
        // ---- COPY the batch's output [cstart, cend) ----
        wave_sync();
        const uint32_t bend = op;
        const uint32_t d_out = lane < nd ? L.desc[lane].y : 0xFFFFFFFFu;   // ~0 past nd
        // Copy through the last step boundary and carry the descriptors from the
        // owner of that boundary on; with no new boundary, carry them all.  The
        // last batch, or one that would carry too many, copies through its end.
        uint32_t cend = bend & ~(uint32_t)(kStep - 1);
        int keep = 0;
        if (cend > cstart) keep = __popcll(wave_ballot(d_out <= cend)) - 1;
        else cend = cstart;
        const bool carry = st == ST_MORE && cend < bend && nd - keep <= kMaxCarry;
        if (!carry) cend = bend;
#ifdef APE_DEXP_NOCOPY
        for (uint32_t base = cend; base < cend; base += kStep) {
#else
        for (uint32_t base = cstart & ~(uint32_t)(kStep - 1); base < cend; base += kStep) {
#endif
            const uint32_t lo = base > cstart ? base : cstart;
            const uint32_t hi = base + kStep < cend ? base + kStep : cend;
            if (lo - gdone > (uint32_t)(kRing / 2)) {
                __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
                gdone = lo;
            }
            wave_sync();
            uint32_t diag = 0;
            copy_step<DICT>(L, D, base, lo, hi, gdone, nd, d_out, diag);
            STAT_ADD(5, diag & 1u);          // steps with a period division
            STAT_ADD(6, (diag >> 1) & 1u);   // steps with in-step sources
            STAT_ADD(7, (diag >> 2) & 0x3FFFu);   // their resolution passes
            STAT_ADD(8, diag >> 16);         // steps reading HBM history / literals
            (void)diag;
            STAT_ADD(3, 1);
        }
        cstart = cend;
        if (carry) {   // desc[keep, nd) -> desc[0, nd - keep)
            wave_sync();
            const uint4 dv = L.desc[keep + (lane < nd - keep ? lane : 0)];
            wave_sync();
            if (lane < nd - keep) L.desc[lane] = dv;
            nd -= keep;
        } else {
            nd = 0;
        }
        STAT(1);
        STAT_ADD(2, 1);
        if (restage && st == ST_MORE) {
            wave_sync();
            D.s0 = stage_base(D.src, P);
            stage_load(L, D.src, D.csize, D.s0, lane);
            wave_sync();
            STAT_ADD(4, 1);
        }
    }
    if (lane == 0) a.result[b] = result;
    STAT_ADD(10, 1);
    STATS_FLUSH(g_dec_stats);
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
