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
//     walk LZ4 tokens from a guessed start (segment start; lane 0 starts at the
//     exact carried position).  Each lane's exit becomes the next lane's entry
//     and lanes re-walk until no entry changes -- a fixpoint that equals the
//     sequential token chain (walks from different starts coalesce quickly, the
//     "Kruskal count" effect, so this converges in a few rounds);
//  3. VALIDATE: lanes re-walk their sequences with exact output positions from
//     a wave prefix-sum, applying the reference's checks in the reference's
//     order, so errors return the identical -(ip - src) - 1, and emit one
//     descriptor per sequence;
//  4. COPY: all 256 threads copy literals, then matches whose source lies in
//     already-final output; wave 0 then does the remaining (dependent or long)
//     copies in sequence order.
#include "lz4_gpu_internal.h"

namespace apelz4 {

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 2048;                 // compressed bytes walked per round
constexpr int kMargin = 320;                 // staged beyond the chunk
constexpr int kStage = kChunk + kMargin;
constexpr int kWalkers = 64;                 // wave 0
constexpr int kSeg = kChunk / kWalkers;      // 32 compressed bytes per walker
constexpr int kMaxSeq = kChunk / 3 + 4;      // each non-final sequence >= 3 bytes
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
    uint8_t comp[kStage];
    SeqDesc desc[kMaxSeq];
    uint32_t cbase, out0, nseq, carry, out_next;
    int state, result;
};

struct DecCtx {
    const uint8_t *src;
    int csize;    // iend
    int cap;      // oend
    int oexit;    // partial target (already clamped)
    bool partial;
};

__device__ __forceinline__ uint32_t rb(const DecShared &S, const DecCtx &c, uint32_t cbase,
                                       uint32_t pos) {
    uint32_t r = pos - cbase;
    if (r < (uint32_t)kStage) return S.comp[r];
    return ((int)pos < c.csize) ? (uint32_t)c.src[pos] : 0u;
}

// Token-chain walk (input side only): from token position t, walk until the
// next token position is >= seg_hi.  Returns the exit; kEnd when the chain
// terminates (final literal run or an input-side error) inside this segment.
__device__ uint32_t walk(const DecShared &S, const DecCtx &c, uint32_t cbase, uint32_t t,
                         uint32_t seg_hi, uint32_t &nseq, uint32_t &nbytes) {
    nseq = 0;
    nbytes = 0;
    while (t < seg_hi) {
        if ((int)t >= c.csize) return kEnd;
        uint32_t tok = rb(S, c, cbase, t);
        uint32_t ip = t + 1;
        uint32_t lit = tok >> 4;
        if (lit == 15) {
            uint32_t s;
            do {
                s = rb(S, c, cbase, ip);
                ip++;
                lit += s;
            } while ((int)ip < c.csize - 15 && s == 255);
        }
        nseq++;
        if ((int64_t)ip + lit > (int64_t)c.csize - 8) return kEnd;
        uint32_t q = ip + lit + 2;
        uint32_t ml = tok & 15;
        if (ml == 15) {
            uint32_t s;
            do {
                if ((int)q > c.csize - kLastLiterals) return kEnd;
                s = rb(S, c, cbase, q);
                q++;
                ml += s;
            } while (s == 255);
        }
        nbytes += lit + ml + kMinMatch;
        t = q;
    }
    return t;
}

// Exit-only walk used by the fixpoint iterations.  `vis` collects the token
// positions visited (bit t - seg_lo); when a re-walk from a new entry reaches a
// position the previous walk visited, the rest is identical, so it stops there.
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
        uint32_t tok = rb(S, c, cbase, t);
        uint32_t ip = t + 1;
        uint32_t lit = tok >> 4;
        if (lit == 15) {
            uint32_t s;
            do {
                s = rb(S, c, cbase, ip);
                ip++;
                lit += s;
            } while ((int)ip < c.csize - 15 && s == 255);
        }
        if ((int64_t)ip + lit > (int64_t)c.csize - 8) return kEnd;
        uint32_t q = ip + lit + 2;
        if ((tok & 15) == 15) {
            uint32_t s;
            do {
                if ((int)q > c.csize - kLastLiterals) return kEnd;
                s = rb(S, c, cbase, q);
                q++;
            } while (s == 255);
        }
        t = q;
    }
    return t;
}

// Validation walk: the reference's sequence loop (:1324-1458) with exact `op`,
// emitting descriptors.  Returns T_NONE / T_DONE / T_ERR with `tv` the block
// result (decoded size, or -(ip)-1, or kErange).
__device__ int validate(DecShared &S, const DecCtx &c, uint32_t cbase, uint32_t t,
                        uint32_t seg_hi, int64_t op, uint32_t di, uint32_t &cnt, int &tv) {
    cnt = 0;
    while (t < seg_hi) {
        uint32_t tok = rb(S, c, cbase, t);
        uint32_t ip = t + 1;
        uint32_t lit = tok >> 4;
        if (lit == 15) {
            uint32_t s;
            do {
                s = rb(S, c, cbase, ip);
                ip++;
                lit += s;
            } while ((int)ip < c.csize - 15 && s == 255);
        }
        int64_t cpy = op + lit;
        bool fin = c.partial ? (cpy > c.oexit) : (cpy > (int64_t)c.cap - kMFLimit);
        fin = fin || ((int64_t)ip + lit > (int64_t)c.csize - 8);
        if (fin) {  // :1346-1366
            bool err = c.partial ? (cpy > c.cap || (int64_t)ip + lit > c.csize)
                                 : ((int64_t)ip + lit != c.csize || cpy > c.cap);
            if (err) { tv = -(int)ip - 1; return T_ERR; }
            if (cpy > kMaxBlock) { tv = kErange; return T_ERR; }
            if (di + cnt < (uint32_t)kMaxSeq) {
                S.desc[di + cnt] = SeqDesc{ip, (uint32_t)op, lit, 0u};
                cnt++;
            }
            tv = (int)cpy;
            return T_DONE;
        }
        uint32_t lit_src = ip;
        ip += lit;
        uint32_t off = rb(S, c, cbase, ip) | (rb(S, c, cbase, ip + 1) << 8);
        ip += 2;
        if (cpy - (int64_t)off < 0) { tv = -(int)ip - 1; return T_ERR; }  // :1375
        uint32_t ml = tok & 15;
        if (ml == 15) {  // :1380-1390
            uint32_t s;
            do {
                if ((int)ip > c.csize - kLastLiterals) { tv = -(int)ip - 1; return T_ERR; }
                s = rb(S, c, cbase, ip);
                ip++;
                ml += s;
            } while (s == 255);
        }
        ml += kMinMatch;
        int64_t mend = cpy + ml;
        if (mend > (int64_t)c.cap - kLastLiterals) { tv = -(int)ip - 1; return T_ERR; }  // :1444
        if (mend > kMaxBlock) { tv = kErange; return T_ERR; }
        if (di + cnt < (uint32_t)kMaxSeq) {
            S.desc[di + cnt] = SeqDesc{lit_src, (uint32_t)op, lit, off | (ml << 16)};
            cnt++;
        } else {
            tv = kErange;  // cannot happen for a converged chain (>= 3 bytes/sequence)
            return T_ERR;
        }
        op = mend;
        t = ip;
    }
    return T_NONE;
}

// Largest i with desc[i].out <= pos (descriptors are in output order).
__device__ __forceinline__ uint32_t find_seq(const DecShared &S, uint32_t nseq, uint32_t pos) {
    uint32_t lo = 0, hi = nseq - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi + 1) >> 1;
        if (S.desc[mid].out <= pos) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Value of output byte `s` (>= out0, inside this chunk) by walking its source
// chain back to a literal or to output before the chunk.  Each hop moves to
// before the current sequence's match start, so it terminates.
__device__ uint32_t resolve(const DecShared &S, const DecCtx &c, uint32_t cbase, uint32_t nseq,
                            uint32_t out0, uint32_t s, const uint8_t *out) {
    for (;;) {
        const SeqDesc d = S.desc[find_seq(S, nseq, s)];
        const uint32_t lit_end = d.out + d.lit_len;
        if (s < lit_end) return rb(S, c, cbase, d.lit_src + (s - d.out));
        const uint32_t off = d.mo & 0xFFFFu;
        if (off == 0) return 0;
        uint32_t k = s - lit_end;
        if (k >= off) k %= off;
        s = lit_end - off + k;
        if (s < out0) return out[s];
    }
}

}  // namespace

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

    // Special cases of :1316-1318 and the empty-input quirk (reads src[0]).
    if (c.cap == 0 || c.csize <= 0) {
        if (tid == 0) {
            int r;
            if (c.csize < 0) r = -1;  // reference: negative size -> iend < ip (garbage); see DESIGN
            else if (c.cap == 0) r = (c.csize == 1 && c.src[0] == 0) ? 0 : -1;
            else {
                uint32_t t0 = c.src ? c.src[0] : 0u;
                r = (t0 >= 0xF0) ? -3 : -2;
            }
            a.result[b] = r;
        }
        return;
    }
    if (c.cap < 0) c.cap = -1;  // every size check then fails like the reference

    uint8_t *out = S.out + ((uintptr_t)dst & 15);
    if (tid == 0) {
        S.cbase = 0;
        S.out0 = 0;
        S.state = 0;
        S.result = 0;
    }
    __syncthreads();

    for (;;) {
        const uint32_t cbase = S.cbase;
        const uint32_t out0 = S.out0;
        // 1. stage
        {
            uint8_t v[(kStage + kThreads - 1) / kThreads];
#pragma unroll
            for (int j = 0; j < (kStage + kThreads - 1) / kThreads; j++) {
                uint32_t i = tid + j * kThreads, p = cbase + i;
                v[j] = (i < (uint32_t)kStage && (int)p < c.csize) ? c.src[p] : 0;
            }
#pragma unroll
            for (int j = 0; j < (kStage + kThreads - 1) / kThreads; j++) {
                uint32_t i = tid + j * kThreads;
                if (i < (uint32_t)kStage) S.comp[i] = v[j];
            }
        }
        __syncthreads();

        // 2+3. token chain + validation (wave 0)
        if (wave == 0) {
            const uint32_t seg_lo = cbase + lane * kSeg;
            const uint32_t seg_hi = seg_lo + kSeg;
            // On the true chain a walker's entry is the max of all earlier walkers'
            // exits (chain positions only grow) and never below its segment start.
            const uint32_t floor_e = seg_lo > cbase ? seg_lo : cbase;
            uint32_t entry = floor_e, ex = 0, vis = 0, pvis = 0, pex = 0;
            for (int it = 0; it < 2 * kWalkers + 2; it++) {
                if (entry < seg_hi) ex = walk_exit(S, c, cbase, entry, seg_lo, seg_hi, pvis, pex, vis);
                else { ex = entry; vis = 0; }
                pvis = vis;
                pex = ex;
                uint32_t mx = ex;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    uint32_t y = __shfl_up(mx, d, 64);
                    if (lane >= d) mx = mx > y ? mx : y;
                }
                uint32_t prev = __shfl_up(mx, 1, 64);
                uint32_t ne = (lane == 0 || prev < floor_e) ? floor_e : prev;
                bool ch = ne != entry;
                entry = ne;
                if (!__any(ch)) break;
            }
            uint32_t nseq = 0, nbytes = 0;
            if (entry < seg_hi) ex = walk(S, c, cbase, entry, seg_hi, nseq, nbytes);
            else ex = entry;
            const uint32_t seq0 = wave_excl_scan(nseq);
            const uint32_t byt0 = wave_excl_scan(nbytes);
            uint32_t cnt = 0;
            int tv = 0, term = T_NONE;
            if (entry < seg_hi)
                term = validate(S, c, cbase, entry, seg_hi, (int64_t)out0 + byt0, seq0, cnt, tv);
            unsigned long long tm = __ballot(term != T_NONE);
            if (tm) {
                int first = __ffsll((long long)tm) - 1;
                uint32_t s0 = __shfl(seq0 + cnt, first, 64);
                int ftv = __shfl(tv, first, 64);
                int fterm = __shfl(term, first, 64);
                if (lane == 0) {
                    S.nseq = s0;
                    S.state = fterm;
                    S.result = ftv;
                    S.out_next = (fterm == T_DONE) ? (uint32_t)ftv : out0;
                }
            } else {
                uint32_t tot = __shfl(seq0 + nseq, 63, 64);
                uint32_t last_ex = __shfl(ex, 63, 64);
                uint32_t tb = __shfl(byt0 + nbytes, 63, 64);
                if (lane == 0) {
                    S.nseq = tot;
                    S.carry = last_ex;
                    S.out_next = out0 + tb;
                }
            }
        }
        __syncthreads();
        if (S.state == T_ERR) break;
        const uint32_t nseq = S.nseq;

        // 4. COPY.  Every output byte of this chunk resolves on its own: a literal
        // byte comes from the compressed stream, a match byte from out[src] when
        // src precedes the chunk, else by following src's own sequence backwards
        // until it lands on a literal or on pre-chunk output.  Only final data is
        // ever read, so there is no ordering and no barrier inside a chunk.
        {
            const uint32_t out_end = S.out_next;
            for (uint32_t base = (out0 & ~15u) + 16u * tid; base < out_end; base += 16u * kThreads) {
                uint32_t q = base < out0 ? out0 : base;
                const uint32_t qe = base + 16u < out_end ? base + 16u : out_end;
                if (q >= qe) continue;
                uint32_t si = find_seq(S, nseq, q);
                SeqDesc d = S.desc[si];
                uint32_t lit_end = d.out + d.lit_len;
                uint32_t off = d.mo & 0xFFFFu, mend = lit_end + (d.mo >> 16);
                uint32_t k = 0;
                bool kvalid = false;
                for (; q < qe; q++) {
                    while (q >= mend && si + 1 < nseq) {
                        d = S.desc[++si];
                        lit_end = d.out + d.lit_len;
                        off = d.mo & 0xFFFFu;
                        mend = lit_end + (d.mo >> 16);
                        kvalid = false;
                    }
                    uint32_t v;
                    if (q < lit_end) {
                        v = rb(S, c, cbase, d.lit_src + (q - d.out));
                    } else if (off == 0) {
                        v = 0;  // offset 0: the reference copies stale dst bytes (App. B)
                    } else {
                        if (!kvalid) {
                            k = q - lit_end;
                            if (k >= off) k %= off;
                            kvalid = true;
                        }
                        const uint32_t src = lit_end - off + k;
                        v = (src < out0) ? out[src] : resolve(S, c, cbase, nseq, out0, src, out);
                        if (++k == off) k = 0;
                    }
                    out[q] = (uint8_t)v;
                }
            }
        }
        __syncthreads();
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
    if (S.state != T_DONE || res <= 0) return;
    const uint32_t n = (uint32_t)res;
    const uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15);
    const uint32_t h = head < n ? head : n;
    if ((uint32_t)tid < h) dst[tid] = out[tid];
    const uint32_t body = (n - h) & ~15u;
    for (uint32_t k = h + 16 * tid; k < h + body; k += 16 * kThreads)
        *(uint4 *)(dst + k) = *(const uint4 *)(out + k);
    for (uint32_t k = h + body + tid; k < n; k += kThreads) dst[k] = out[k];
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
