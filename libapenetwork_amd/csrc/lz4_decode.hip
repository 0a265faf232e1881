// lz4_decode.hip -- MI355X (gfx950) batched LZ4 block decoder, bit-exact with
// APE_LZ4_decompress_safe / _safe_partial (ref src/ape_lz4.c:1275-1487).
//
// One 256-thread workgroup decodes one independent block; the whole decoded
// block lives in LDS (64 KiB) so match back-references are LDS reads, and it is
// written to HBM once, with 16-byte stores, at the end.  ~79 KiB LDS per
// workgroup -> two blocks resident per CU.
//
// The compressed stream is processed in chunks of kChunk bytes:
//  1. stage the chunk (+ margin) into LDS;
//  2. TOKEN CHAIN: wave 0's 64 lanes each own a 32-byte segment of the chunk and
//     walk LZ4 tokens from a guessed start.  A walker's entry is the max of the
//     earlier walkers' exits (chain positions only grow); lanes re-walk until no
//     entry changes -- a fixpoint equal to the sequential token chain.  Walks
//     from different starts coalesce quickly ("Kruskal count"), and a re-walk
//     stops as soon as it reaches a token the previous walk visited;
//  3. VALIDATE: lanes re-walk their sequences with exact output positions from a
//     wave prefix-sum, applying the reference's checks in the reference's order,
//     so errors return the identical -(ip - src) - 1, and emit one descriptor per
//     sequence;
//  4. COPY: the 4 waves take 128-byte output steps round-robin.  A byte whose
//     source lies below the published frontier reads it directly; a source inside
//     the same step resolves through the step's descriptors (lane shuffles); only
//     a source in the few steps still in flight waits for the frontier.  The
//     lowest unfinished step never waits, so the scheme cannot deadlock.
#include "lz4_gpu_internal.h"

namespace apelz4 {

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 2048;                 // compressed bytes walked per round
constexpr int kMargin = 320;                 // staged beyond the chunk
constexpr int kStage = kChunk + kMargin;     // multiple of 4
constexpr int kWalkers = 64;                 // wave 0
constexpr int kSeg = kChunk / kWalkers;      // 32 compressed bytes per walker
constexpr int kMaxSeq = kChunk / 3 + 4;      // each non-final sequence >= 3 bytes
constexpr int kStep = 256;                   // output bytes per copy step (4 per lane)
constexpr uint32_t kEnd = 0xFFFFFFFFu;       // "chain ended" exit marker

enum { T_NONE = 0, T_DONE = 1, T_ERR = 2 };

struct SeqDesc {
    uint32_t lit_src;  // compressed position of the literals
    uint32_t out;      // output position of the literals
    uint32_t lit_len;
    uint32_t mo;       // match offset (low 16) | match length (high 16); 0 = none
};

struct __attribute__((aligned(16))) DecShared {
    uint8_t out[kMaxBlock + 16];
    uint32_t comp[kStage / 4 + 2];  // staged compressed bytes, zero beyond the input
    SeqDesc desc[kMaxSeq];
    uint32_t cbase, out0, nseq, carry, out_next, front;
    int state, result;
};

struct DecCtx {
    const uint8_t *src;
    int csize;    // iend
    int cap;      // oend
    int oexit;    // partial target (already clamped)
    bool partial;
};

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * sh));
}

__device__ __forceinline__ uint32_t rb(const DecShared &S, const DecCtx &c, uint32_t cbase,
                                       uint32_t pos) {
    uint32_t r = pos - cbase;
    if (r < (uint32_t)kStage) return (S.comp[r >> 2] >> (8u * (r & 3u))) & 0xFFu;
    return ((int)pos < c.csize) ? (uint32_t)c.src[pos] : 0u;
}

// 8 bytes at pos, little-endian (three aligned LDS dwords in the staged window).
__device__ __forceinline__ uint64_t rd8(const DecShared &S, const DecCtx &c, uint32_t cbase,
                                        uint32_t pos) {
    const uint32_t r = pos - cbase;
    if (r + 8u <= (uint32_t)kStage) {
        const uint32_t *w = &S.comp[r >> 2];
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], sh = r & 3u;
        return (uint64_t)funnel(w1, w0, sh) | ((uint64_t)funnel(w2, w1, sh) << 32);
    }
    uint64_t x = 0;
    for (int k = 0; k < 8; k++) x |= (uint64_t)rb(S, c, cbase, pos + k) << (8 * k);
    return x;
}

// One parsed sequence, input side only (what :1330-1391 read, in that order).
struct Tok {
    uint32_t tok;
    uint32_t ip;    // first literal byte
    uint32_t lit;   // literal length
    uint32_t off;   // match offset (read at ip + lit)
    uint32_t q;     // position after the match-length bytes (next token)
    uint32_t ml;    // match length - 4
    uint32_t qerr;  // where the match-length loop hit the input end (mlerr)
    bool mlerr;
};

// Usually one LDS round trip: the 8-byte window at the token covers the token,
// short literal-length bytes, and for short literal runs the offset too.
__device__ __forceinline__ Tok parse_seq(const DecShared &S, const DecCtx &c, uint32_t cbase,
                                         uint32_t t) {
    Tok r;
    uint64_t w = rd8(S, c, cbase, t);
    uint32_t base = t;
#define WB(pos) ((uint32_t)((pos) - base) < 8u ? (uint32_t)(w >> (8u * ((pos) - base))) & 0xFFu \
                                                 : rb(S, c, cbase, (pos)))
    r.tok = (uint32_t)w & 0xFFu;
    uint32_t ip = t + 1, lit = r.tok >> 4;
    if (lit == 15) {
        uint32_t s;
        do {
            s = WB(ip);
            ip++;
            lit += s;
        } while ((int)ip < c.csize - 15 && s == 255);
    }
    r.ip = ip;
    r.lit = lit;
    const uint32_t qo = ip + lit;
    if ((uint32_t)(qo - t) > 4u) {  // offset (+2 length bytes) not in the first window
        w = rd8(S, c, cbase, qo);
        base = qo;
    }
    r.off = WB(qo) | (WB(qo + 1) << 8);
    uint32_t q = qo + 2, ml = r.tok & 15;
    r.mlerr = false;
    r.qerr = 0;
    if (ml == 15) {
        uint32_t s;
        do {
            if ((int)q > c.csize - kLastLiterals) {
                r.mlerr = true;
                r.qerr = q;
                break;
            }
            s = WB(q);
            q++;
            ml += s;
        } while (s == 255);
    }
#undef WB
    r.q = q;
    r.ml = ml;
    return r;
}

// Exit-only walk used by the fixpoint iterations.  `vis` collects the token
// positions visited (bit t - seg_lo); when a re-walk from a new entry reaches a
// position the previous walk visited, the rest is identical, so it stops there.
// Returns kEnd when the chain terminates (final literals / input-side error).
__device__ uint32_t walk_exit(const DecShared &S, const DecCtx &c, uint32_t cbase, uint32_t t,
                              uint32_t seg_lo, uint32_t seg_hi, uint32_t prev_vis,
                              uint32_t prev_ex, uint32_t &vis) {
    vis = 0;
    while (t < seg_hi) {
        const uint32_t bit = 1u << (t - seg_lo);
        if (prev_vis & bit) {
            vis |= prev_vis & ~(bit - 1u);
            return prev_ex;
        }
        vis |= bit;
        if ((int)t >= c.csize) return kEnd;
        const Tok r = parse_seq(S, c, cbase, t);
        if ((int64_t)r.ip + r.lit > (int64_t)c.csize - 8 || r.mlerr) return kEnd;
        t = r.q;
    }
    return t;
}

// Counting walk: number of sequences and decoded bytes from t to the segment end.
__device__ uint32_t walk_count(const DecShared &S, const DecCtx &c, uint32_t cbase, uint32_t t,
                               uint32_t seg_hi, uint32_t &nseq, uint32_t &nbytes) {
    nseq = 0;
    nbytes = 0;
    while (t < seg_hi) {
        if ((int)t >= c.csize) return kEnd;
        const Tok r = parse_seq(S, c, cbase, t);
        nseq++;
        if ((int64_t)r.ip + r.lit > (int64_t)c.csize - 8 || r.mlerr) return kEnd;
        nbytes += r.lit + r.ml + kMinMatch;
        t = r.q;
    }
    return t;
}

// Validation walk: the reference's sequence loop (:1324-1458) with exact `op`,
// checks in the reference's order, emitting descriptors.  Returns T_NONE /
// T_DONE / T_ERR with `tv` the block result (decoded size, -(ip)-1, or kErange).
__device__ int validate(DecShared &S, const DecCtx &c, uint32_t cbase, uint32_t t,
                        uint32_t seg_hi, int64_t op, uint32_t di, uint32_t &cnt, int &tv) {
    cnt = 0;
    while (t < seg_hi) {
        const Tok r = parse_seq(S, c, cbase, t);
        const int64_t cpy = op + r.lit;
        bool fin = c.partial ? (cpy > c.oexit) : (cpy > (int64_t)c.cap - kMFLimit);
        fin = fin || ((int64_t)r.ip + r.lit > (int64_t)c.csize - 8);
        if (fin) {  // :1346-1366
            const bool err = c.partial ? (cpy > c.cap || (int64_t)r.ip + r.lit > c.csize)
                                       : ((int64_t)r.ip + r.lit != c.csize || cpy > c.cap);
            if (err) { tv = -(int)r.ip - 1; return T_ERR; }
            if (cpy > kMaxBlock) { tv = kErange; return T_ERR; }
            if (di + cnt < (uint32_t)kMaxSeq) {
                S.desc[di + cnt] = SeqDesc{r.ip, (uint32_t)op, r.lit, 0u};
                cnt++;
            }
            tv = (int)cpy;
            return T_DONE;
        }
        const uint32_t ip_off = r.ip + r.lit + 2;
        if (cpy - (int64_t)r.off < 0) { tv = -(int)ip_off - 1; return T_ERR; }  // :1375
        if (r.mlerr) { tv = -(int)r.qerr - 1; return T_ERR; }                   // :1383
        const uint32_t ml = r.ml + kMinMatch;
        const int64_t mend = cpy + ml;
        if (mend > (int64_t)c.cap - kLastLiterals) { tv = -(int)r.q - 1; return T_ERR; }  // :1444
        if (mend > kMaxBlock) { tv = kErange; return T_ERR; }
        if (di + cnt < (uint32_t)kMaxSeq) {
            S.desc[di + cnt] = SeqDesc{r.ip, (uint32_t)op, r.lit, r.off | (ml << 16)};
            cnt++;
        } else {
            tv = kErange;  // cannot happen for a converged chain (>= 3 bytes/sequence)
            return T_ERR;
        }
        op = mend;
        t = r.q;
    }
    return T_NONE;
}

__device__ __forceinline__ uint32_t front_load(const DecShared &S) {
    return __hip_atomic_load(&S.front, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}


// Last descriptor with out <= pos, searching forward from si0 (wave-uniform).
__device__ __forceinline__ uint32_t seek(const DecShared &S, uint32_t nseq, uint32_t si0,
                                         uint32_t pos, int lane) {
    for (;;) {
        const uint32_t idx = si0 + lane;
        const uint32_t o = idx < nseq ? S.desc[idx].out : 0xFFFFFFFFu;
        const unsigned long long m = __ballot(o <= pos);
        if (m == ~0ull) { si0 += 64; continue; }
        return si0 + (uint32_t)__popcll(m) - 1u;
    }
}

// Copy output bytes [lo, hi) of the step at `base` (BPL bytes per lane); the 64
// lanes hold the descriptors si0 .. si0+63, which cover the whole step.
template <int BPL>
__device__ __forceinline__ void copy_step(DecShared &S, const DecCtx &c, uint32_t cbase,
                                          uint32_t nseq, uint32_t si0, uint32_t base,
                                          uint32_t lo, uint32_t hi, uint8_t *out, int lane) {
    const uint32_t idx = si0 + lane;
    const SeqDesc dl = idx < nseq ? S.desc[idx] : SeqDesc{0u, 0xFFFFFFFFu, 0u, 0u};
    uint32_t pos[BPL], val[BPL], rsrc[BPL];
    bool live[BPL], rd[BPL], pend[BPL];
#pragma unroll
    for (int j = 0; j < BPL; j++) {
        const uint32_t q = base + BPL * (uint32_t)lane + j;
        pos[j] = q;
        val[j] = 0;
        rsrc[j] = 0;
        rd[j] = false;
        live[j] = q >= lo && q < hi;
        pend[j] = live[j];
    }
    // Resolve byte p inside descriptor d: literal -> value, match -> its source;
    // a source inside this step stays pending (pos = source) for the next hop.
    auto resolve = [&](int j, uint32_t p, uint32_t d_out, uint32_t d_src, uint32_t d_lit,
                       uint32_t d_mo) {
        const uint32_t le = d_out + d_lit;
        const uint32_t off = d_mo & 0xFFFFu;
        if (p < le) {
            val[j] = rb(S, c, cbase, d_src + (p - d_out));
            pend[j] = false;
        } else if (off == 0) {
            pend[j] = false;  // offset 0: stale dst bytes in the reference (App. B)
        } else {
            uint32_t k = p - le;
            if (k >= off) k %= off;
            const uint32_t src = le - off + k;
            if (src < lo) {
                rsrc[j] = src;
                rd[j] = true;
                pend[j] = false;
            } else {
                pos[j] = src;
            }
        }
    };
    auto owner = [&](uint32_t p) {
        int ol = 0;
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) {
            const uint32_t o = __shfl(dl.out, ol + s, 64);
            if (ol + s < 64 && o <= p) ol += s;
        }
        return ol;
    };
    {   // first pass: the lane's BPL consecutive bytes lie in the owner A of the
        // first one or in its successor B (every non-final sequence is >= 4 bytes)
        const int ol = owner(base + BPL * (uint32_t)lane);
        const int ob = ol + 1 < 64 ? ol + 1 : 63;
        const uint32_t a_out = __shfl(dl.out, ol, 64), a_src = __shfl(dl.lit_src, ol, 64);
        const uint32_t a_lit = __shfl(dl.lit_len, ol, 64), a_mo = __shfl(dl.mo, ol, 64);
        const uint32_t b_out = __shfl(dl.out, ob, 64), b_src = __shfl(dl.lit_src, ob, 64);
        const uint32_t b_lit = __shfl(dl.lit_len, ob, 64), b_mo = __shfl(dl.mo, ob, 64);
#pragma unroll
        for (int j = 0; j < BPL; j++) {
            if (!pend[j]) continue;
            const uint32_t p = pos[j];
            if (p < b_out) resolve(j, p, a_out, a_src, a_lit, a_mo);
            else resolve(j, p, b_out, b_src, b_lit, b_mo);
        }
    }
    // in-step sources (rare): one pending byte per lane per hop
    for (int hop = 0; hop < BPL * kStep; hop++) {
        bool any = false;
        int jj = 0;
        uint32_t p = 0;
#pragma unroll
        for (int j = BPL - 1; j >= 0; j--)
            if (pend[j]) { any = true; jj = j; p = pos[j]; }
        if (!__any(any)) break;
        const int ol = owner(p);
        const uint32_t d_out = __shfl(dl.out, ol, 64), d_src = __shfl(dl.lit_src, ol, 64);
        const uint32_t d_lit = __shfl(dl.lit_len, ol, 64), d_mo = __shfl(dl.mo, ol, 64);
        if (any) {
#pragma unroll
            for (int j = 0; j < BPL; j++)
                if (j == jj) resolve(j, p, d_out, d_src, d_lit, d_mo);
        }
    }
    // sources in steps still in flight: wait for the frontier
    uint32_t f = front_load(S);
    for (;;) {
        bool w = false;
#pragma unroll
        for (int j = 0; j < BPL; j++) w |= rd[j] && rsrc[j] >= f;
        if (!__any(w)) break;
        __builtin_amdgcn_s_sleep(1);
        f = front_load(S);
    }
    uint32_t word = 0;
    bool all_live = true;
#pragma unroll
    for (int j = 0; j < BPL; j++) {
        if (rd[j]) val[j] = out[rsrc[j]];
        word |= (val[j] & 0xFFu) << (8 * j);
        all_live &= live[j];
    }
    uint8_t *o = out + base + BPL * (uint32_t)lane;
    if (BPL == 4 && all_live && (((uintptr_t)o) & 3) == 0) {
        *(uint32_t *)o = word;
    } else {
#pragma unroll
        for (int j = 0; j < BPL; j++)
            if (live[j]) o[j] = (uint8_t)val[j];
    }
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

template <bool PARTIAL>
__global__ void __launch_bounds__(kThreads)
lz4_decode_kernel(BlockArgs a) {
    __shared__ DecShared S;
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    DecCtx c;
    c.src = (const uint8_t *)(a.src ? a.src[b] : a.src_base + (size_t)b * a.src_stride);
    uint8_t *dst = (uint8_t *)(a.dst ? a.dst[b] : a.dst_base + (size_t)b * a.dst_stride);
    c.csize = a.src_size[b];
    c.cap = a.dst_cap ? a.dst_cap[b] : (int)a.dst_stride;
    c.partial = PARTIAL;
    c.oexit = PARTIAL ? a.target[b] : 0;
    if (PARTIAL && (int64_t)c.oexit > (int64_t)c.cap - kMFLimit) c.oexit = c.cap - kMFLimit;

    // Special cases of :1316-1318 and the empty-input quirk (the reference reads
    // src[0] even when compressedSize <= 0).
    if (c.cap == 0 || c.csize <= 0) {
        if (tid == 0) {
            int r;
            if (c.cap == 0) r = (c.csize == 1 && c.src[0] == 0) ? 0 : -1;
            else r = ((c.src ? c.src[0] : 0u) >= 0xF0) ? -3 : -2;
            a.result[b] = r;
        }
        return;
    }

    uint8_t *out = S.out + ((uintptr_t)dst & 15);
    STATS_DECL
    if (tid == 0) {
        S.cbase = 0;
        S.out0 = 0;
        S.state = 0;
        S.result = 0;
    }
    __syncthreads();
    STAT(0);

    for (;;) {
        const uint32_t cbase = S.cbase;
        const uint32_t out0 = S.out0;
        // 1. stage (byte loads, all in flight together)
        {
            constexpr int kPer = (kStage + 8 + 4 * kThreads - 1) / (4 * kThreads);
            uint32_t v[kPer];
#pragma unroll
            for (int j = 0; j < kPer; j++) {
                const uint32_t i = 4u * (tid + j * kThreads);
                uint32_t x = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t p = cbase + i + k;
                    if (i + k < (uint32_t)kStage + 8 && (int)p < c.csize)
                        x |= (uint32_t)c.src[p] << (8 * k);
                }
                v[j] = x;
            }
#pragma unroll
            for (int j = 0; j < kPer; j++) {
                const uint32_t i = tid + j * kThreads;
                if (i < (uint32_t)(kStage / 4 + 2)) S.comp[i] = v[j];
            }
        }
        if (tid == 0) S.front = out0;
        __syncthreads();
        STAT(1);
        STAT_ADD(8, 1);

        // 2+3. token chain + validation (wave 0)
        if (wave == 0) {
            const uint32_t seg_lo = cbase + lane * kSeg;
            const uint32_t seg_hi = seg_lo + kSeg;
            const uint32_t floor_e = seg_lo > cbase ? seg_lo : cbase;
            uint32_t entry = floor_e, ex = 0, vis = 0, pvis = 0, pex = 0;
            int it = 0;
            for (; it < 2 * kWalkers + 2; it++) {
                if (entry < seg_hi) ex = walk_exit(S, c, cbase, entry, seg_lo, seg_hi, pvis, pex, vis);
                else { ex = entry; vis = 0; }
                pvis = vis;
                pex = ex;
                const uint32_t prev = wave_shr1(wave_incl_max(ex), 0u);
                const uint32_t ne = prev < floor_e ? floor_e : prev;
                bool ch = ne != entry;
                entry = ne;
                if (!__any(ch)) break;
            }
            STAT(2);
            STAT_ADD(5, it + 1);
            uint32_t nseq = 0, nbytes = 0;
            if (entry < seg_hi) ex = walk_count(S, c, cbase, entry, seg_hi, nseq, nbytes);
            else ex = entry;
            const uint32_t seq0 = wave_excl_scan(nseq);
            const uint32_t byt0 = wave_excl_scan(nbytes);
            STAT(3);
            uint32_t cnt = 0;
            int tv = 0, term = T_NONE;
            if (entry < seg_hi)
                term = validate(S, c, cbase, entry, seg_hi, (int64_t)out0 + byt0, seq0, cnt, tv);
            STAT(4);
            unsigned long long tm = __ballot(term != T_NONE);
            if (tm) {
                int first = __ffsll((long long)tm) - 1;
                uint32_t s0 = lane_val(seq0 + cnt, first);
                int ftv = (int)lane_val((uint32_t)tv, first);
                int fterm = (int)lane_val((uint32_t)term, first);
                if (lane == 0) {
                    S.nseq = s0;
                    S.state = fterm;
                    S.result = ftv;
                    S.out_next = (fterm == T_DONE) ? (uint32_t)ftv : out0;
                }
            } else {
                uint32_t tot = lane_val(seq0 + nseq, 63);
                uint32_t last_ex = lane_val(ex, 63);
                uint32_t tb = lane_val(byt0 + nbytes, 63);
                if (lane == 0) {
                    S.nseq = tot;
                    S.carry = last_ex;
                    S.out_next = out0 + tb;
                }
            }
        }
        __syncthreads();
        STAT(6);
        if (S.state == T_ERR) break;
        const uint32_t nseq = S.nseq;

        // 4. COPY: round-robin steps behind a published frontier.
        {
            const uint32_t out_end = S.out_next;
            const uint32_t first = out0 / kStep, last = (out_end + kStep - 1) / kStep;
            uint32_t si0 = 0;  // wave-uniform: last descriptor with out <= step start
            for (uint32_t st = first + wave; st < last; st += kThreads / 64) {
                const uint32_t base = st * kStep;
                const uint32_t lo = base > out0 ? base : out0;
                const uint32_t hi = base + kStep < out_end ? base + kStep : out_end;
                si0 = seek(S, nseq, si0, lo, lane);
                // 4 bytes per lane; a step that overlaps more than 64 sequences
                // (all of them ~4 bytes long) is done as two 2-byte-per-lane halves
                const uint32_t i63 = si0 + 63;
                if (i63 >= nseq || S.desc[i63].out >= hi) {
                    copy_step<4>(S, c, cbase, nseq, si0, base, lo, hi, out, lane);
                } else {
                    const uint32_t mid = base + kStep / 2;
                    copy_step<2>(S, c, cbase, nseq, si0, base, lo, mid < hi ? mid : hi, out, lane);
                    if (mid < hi) {
                        si0 = seek(S, nseq, si0, mid, lane);
                        copy_step<2>(S, c, cbase, nseq, si0, mid, mid, hi, out, lane);
                    }
                }
                // publish this step once every earlier step has been published
                if (lane == 0) {
                    while (front_load(S) < lo) __builtin_amdgcn_s_sleep(1);
                    __hip_atomic_store(&S.front, hi, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        }
        __syncthreads();
        STAT(7);
        if (S.state == T_DONE) break;
        if (tid == 0) {
            // the chain always advances (>= 3 bytes per sequence); anything else is
            // an internal error, reported rather than looped on
            if (S.carry <= cbase || S.carry >= (uint32_t)c.csize) {
                S.state = T_ERR;
                S.result = kErange;
            }
            S.cbase = S.carry;
            S.out0 = S.out_next;
        }
        __syncthreads();
        if (S.state == T_ERR) break;
    }

    // 5. result + flush dst[0:result) with 16-byte stores
    const int res = S.result;
    if (tid == 0) a.result[b] = res;
    if (S.state == T_DONE && res > 0) {
        const uint32_t n = (uint32_t)res;
        const uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15);
        const uint32_t h = head < n ? head : n;
        if ((uint32_t)tid < h) dst[tid] = out[tid];
        const uint32_t body = (n - h) & ~15u;
        for (uint32_t k = h + 16 * tid; k < h + body; k += 16 * kThreads)
            *(uint4 *)(dst + k) = *(const uint4 *)(out + k);
        for (uint32_t k = h + body + tid; k < n; k += kThreads) dst[k] = out[k];
    }
    STAT(9);
    STAT_ADD(10, 1);
    STATS_FLUSH(g_dec_stats);
}

hipError_t launch_decode(const BlockArgs &a, bool partial, hipStream_t s) {
    if (a.nblocks <= 0) return hipSuccess;
    if (partial)
        hipLaunchKernelGGL(lz4_decode_kernel<true>, dim3(a.nblocks), dim3(kThreads), 0, s, a);
    else
        hipLaunchKernelGGL(lz4_decode_kernel<false>, dim3(a.nblocks), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace apelz4
