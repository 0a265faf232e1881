/* seg_model.c -- DESIGN TOOL (not product, not oracle): CPU model of a two-phase LZ4 block
 * encoder for the GPU, to choose its parameters before writing kernels.
 *
 *   gcc -O2 -o /tmp/seg_model tools/seg_model.c oracle/synth.c && /tmp/seg_model
 *
 * Phase A (chain): positions q = 0, stride, 2*stride, ... are inserted into a head table of
 *   2^hlog entries in order; prev[q] = the latest inserted position p < q with hash(p) ==
 *   hash(q) (what an in-order LDS exchange per position gives), for EVERY q.  This is
 *   parse-independent, so it is computed for the whole block before any parsing.
 * Phase B (parse): the block is cut into nseg segments; each is parsed greedily on its own
 *   (the reference's search loop, ref src/ape_lz4.c:591-619, with its skip acceleration)
 *   from the chain: candidates prev[q], prev[prev[q]], ... (depth), verified (4 bytes) and
 *   measured; the longest wins; catch-up backwards (ref :623-627) within the segment's
 *   literals.  A match may run past the segment end.
 * Splice: segment k's sequences that lie inside the previous segment's last match are dropped,
 *   a straddling one is cut to start at that match end (kept if >= 4 bytes), and the literal
 *   runs join across segment boundaries.  The output size is exact LZ4 block size.
 *
 * Reports ratio vs the reference encoder, and per segment the number of loop iterations
 * (positions probed + 16-byte extension steps), whose max over a wave's segments prices the
 * lock-step parse.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void synth_blocks(uint8_t *out, int n, long long stride, long long first, int nb, int kind);

static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static int ext(int v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }

typedef struct { int lit0, m, len, off; } seq_t;

static int g_hlog = 13, g_stride = 1, g_depth = 1, g_nseg = 64, g_skip = 1, g_ext16 = 16;
static long g_iter_sum, g_iter_max_sum, g_blocks, g_wave_sum;

static int g_ways = 0, g_fpbits = 16, g_cap = 0, g_capx = 0, g_meas = 0;   /* ways > 0: bucket scheme with fingerprints */
static uint64_t hprod(const uint8_t *p) { return (rd64(p) << 24) * 0x9E3779B185EBCA87ULL; }
static uint32_t hsh(const uint8_t *p) {
    if (g_ways) return (uint32_t)(hprod(p) >> (64 - g_hlog));
    return (uint32_t)((rd64(p) * 889523592379ULL) >> (40 - g_hlog)) & ((1u << g_hlog) - 1);
}
static uint32_t fpr(const uint8_t *p) {
    return (uint32_t)(hprod(p) >> (64 - g_hlog - g_fpbits)) & ((1u << g_fpbits) - 1);
}

static long encode(const uint8_t *in, int n, int *prev, int *head, seq_t *seqs, int *nseqs_out)
{
    const int H = 1 << g_hlog, mflimit = n - 12, mlimit = n - 5;
    /* phase A */
    if (!g_ways) {
        for (int i = 0; i < H; i++) head[i] = -1;
        for (int q = 0; q < n; q++) {
            if (q + 8 > n) { prev[q] = -1; continue; }
            uint32_t h = hsh(in + q);
            prev[q] = head[h];
            if (q % g_stride == 0) head[h] = q;
        }
    } else {   /* W-way buckets of (position, fingerprint); prev[q] = newest fp match */
        int *bp = head, *bf = head + H * 8;
        for (int i = 0; i < H * g_ways; i++) bp[i] = -1, bf[i] = -1;
        for (int q = 0; q < n; q++) {
            if (q + 8 > n) { prev[q] = -1; continue; }
            uint32_t h = hsh(in + q), f = fpr(in + q);
            prev[q] = -1;
            for (int w = 0; w < g_ways; w++)
                if (bp[h * g_ways + w] >= 0 && (uint32_t)bf[h * g_ways + w] == f) { prev[q] = bp[h * g_ways + w]; break; }
            for (int w = g_ways - 1; w > 0; w--) {
                bp[h * g_ways + w] = bp[h * g_ways + w - 1];
                bf[h * g_ways + w] = bf[h * g_ways + w - 1];
            }
            bp[h * g_ways] = q;
            bf[h * g_ways] = (int)f;
        }
    }
    /* phase B: per segment */
    const int S = (n + g_nseg - 1) / g_nseg;
    int nq = 0;
    int *segfirst = calloc(g_nseg + 1, sizeof(int));
    long itmax = 0, wmax = 0;
    for (int k = 0; k < g_nseg; k++) {
        int s0 = k * S, s1 = s0 + S < n ? s0 + S : n;
        int anchor = s0, p = s0 < 1 ? 1 : s0;
        long it = 0;
        int misses = 0;
        segfirst[k] = nq;
        while (p < s1 && p <= mflimit) {
            int best = 0, bc = -1, c = prev[p];
            it++;
            for (int d = 0; d < g_depth && c >= 0; d++, c = prev[c]) {
                if (p - c > 65535) break;
                if (rd32(in + c) != rd32(in + p)) continue;
                int l = 4;
                const int lim = g_cap ? (s1 + g_capx < mlimit ? s1 + g_capx : mlimit) : mlimit;
                const int mcap = g_meas ? (p + g_meas < lim ? p + g_meas : lim) : lim;
                while (p + l < mcap && in[p + l] == in[c + l]) l++;
                if (l > best) { best = l; bc = c; }
            }
            if (best < 4) {
                /* reference skip: step = searchMatchNb++ >> 6 from 1 << 6 (ref :593-600) */
                int step = g_skip ? (64 + misses++) >> 6 : 1;
                p += step;
                continue;
            }
            misses = 0;
            if (g_meas) {   /* extend the chosen candidate past the first measure */
                const int lim = g_cap ? (s1 + g_capx < mlimit ? s1 + g_capx : mlimit) : mlimit;
                while (p + best < lim && in[p + best] == in[bc + best]) best++;
            }
            int m = p, cc = bc, len = best;
            while (m > anchor && cc > 0 && in[m - 1] == in[cc - 1]) { m--; cc--; len++; }
            it += (best - 4 + g_ext16 - 1) / g_ext16;   /* extension steps past the first */
            seqs[nq].lit0 = anchor;
            seqs[nq].m = m;
            seqs[nq].len = len;
            seqs[nq].off = m - cc;
            nq++;
            anchor = m + len;
            p = anchor;
        }
        if (it > itmax) itmax = it;
        if (it > wmax) wmax = it;
        if ((k & 63) == 63 || k == g_nseg - 1) { g_wave_sum += wmax; wmax = 0; }
        g_iter_sum += it;
    }
    segfirst[g_nseg] = nq;
    g_iter_max_sum += itmax;
    /* splice */
    long out = 0;
    int cover = 0, anchor = 0, nk = 0, lastlit = 0, lastlen = 0, lastoff = -1;
    for (int i = 0; i < nq; i++) {
        seq_t s = seqs[i];
        if (s.m + s.len <= cover) continue;
        if (s.m < cover) { s.len -= cover - s.m; s.m = cover; if (s.len < 4) continue; }
        if (s.m > mflimit || s.m + s.len > mlimit) {   /* never past the block limits */
            if (s.m > mflimit) continue;
            s.len = mlimit - s.m;
            if (s.len < 4) continue;
        }
        if (nk > 0 && s.m == anchor && s.off == lastoff && s.m == cover) {
            /* a match cut at a segment end continued by the next segment at the same offset */
            out -= 1 + ext(lastlit) + lastlit + 2 + ext(lastlen - 4);
            lastlen += s.len;
            out += 1 + ext(lastlit) + lastlit + 2 + ext(lastlen - 4);
            anchor = cover = s.m + s.len;
            continue;
        }
        int lit = s.m - anchor;
        out += 1 + ext(lit) + lit + 2 + ext(s.len - 4);
        lastlit = lit; lastlen = s.len; lastoff = s.off;
        anchor = cover = s.m + s.len;
        nk++;
    }
    int last = n - anchor;
    out += 1 + ext(last) + last;
    *nseqs_out = nk;
    free(segfirst);
    return out;
}

/* the reference's own encoder (greedy, walked-only insertion, 8192 x u16 table), for the ratio */
int APE_LZ4_compress_default(const char *src, char *dst, int n, int cap);

int main(int argc, char **argv)
{
    const int n = 65536, nb = argc > 1 ? atoi(argv[1]) : 64;
    const int kind = argc > 2 ? atoi(argv[2]) : 1;   /* synth kind: 1 = App. C compressible */
    uint8_t *in = malloc((size_t)n * nb);
    int *prev = malloc(sizeof(int) * n), *head = malloc(sizeof(int) * (1 << 24));
    seq_t *seqs = malloc(sizeof(seq_t) * n);
    synth_blocks(in, n, n, 0, nb, kind == 2 ? 0 : kind);
    if (kind == 2) {   /* random bytes + back-copies of 11..86 bytes (tests' _boundary_copies) */
        static const int lens[] = {11, 12, 13, 15, 16, 17, 19, 20, 21, 75, 76, 77, 79, 80, 81, 83, 84, 85, 86};
        uint64_t r = 88172645463325252ULL;
        for (int b = 0; b < nb; b++) {
            uint8_t *o = in + (size_t)b * n;
            int i = 2048;
            while (i < n) {
                r ^= r << 13; r ^= r >> 7; r ^= r << 17;
                int ln = lens[r % 19], off = 1 + (int)((r >> 8) % (uint64_t)(i < 65535 ? i - 1 : 65534));
                for (int k = 0; k < ln && i < n; k++, i++) o[i] = o[i - off];
                if (i < n) o[i++] = (uint8_t)(r >> 40);
            }
        }
    }
    struct { int hlog, stride, depth, nseg, ways, cap, meas; } cfg[] = {
        {11, 4, 4, 1024, 0, 64, 16}, {11, 4, 4, 4096, 0, 64, 16}, {11, 4, 3, 4096, 0, 64, 16},
        {11, 4, 2, 4096, 0, 64, 16}, {11, 4, 4, 2048, 0, 64, 16}};
    struct { int hlog, stride, depth, nseg; } cfg_old[] = {
        {13, 1, 1, 64}, {13, 1, 2, 64}, {13, 1, 4, 64}, {13, 2, 1, 64}, {13, 4, 1, 64},
        {13, 4, 2, 64}, {14, 1, 1, 64}, {14, 1, 2, 64}, {14, 2, 2, 64}, {14, 4, 2, 64},
        {15, 1, 1, 64}, {15, 1, 2, 64}, {15, 2, 2, 64}, {16, 1, 1, 64}, {16, 1, 2, 64},
        {13, 1, 2, 32}, {13, 1, 2, 16}, {13, 1, 2, 1}, {16, 1, 4, 64}, {12, 1, 2, 64},
        {12, 2, 2, 64}, {12, 1, 4, 64}};
    for (size_t c = 0; c < sizeof cfg / sizeof cfg[0]; c++) {
        g_hlog = cfg[c].hlog; g_stride = cfg[c].stride; g_depth = cfg[c].depth; g_nseg = cfg[c].nseg;
        g_meas = cfg[c].meas; g_ways = cfg[c].ways; g_cap = cfg[c].cap > 0; g_capx = cfg[c].cap > 16 ? cfg[c].cap : cfg[c].cap > 0 ? (cfg[c].cap - 1) * ((n + cfg[c].nseg - 1) / cfg[c].nseg) : 0;
        g_iter_sum = g_iter_max_sum = g_wave_sum = 0;
        long tot = 0, nseq = 0;
        for (int b = 0; b < nb; b++) {
            int ns;
            tot += encode(in + (size_t)b * n, n, prev, head, seqs, &ns);
            nseq += ns;
        }
        printf("meas %2d cap %d ways %d hlog %2d stride %d depth %d nseg %4d: ratio %.4f  seq/blk %6.0f  iter/seg %5.1f  "
               "max-iter/blk %6.1f  sum-wave-max/blk %7.0f\n", g_meas, g_cap, g_ways, g_hlog, g_stride, g_depth, g_nseg, (double)n * nb / tot,
               (double)nseq / nb, (double)g_iter_sum / nb / g_nseg, (double)g_iter_max_sum / nb, (double)g_wave_sum / nb);
    }
    return 0;
}
