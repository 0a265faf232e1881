/* seg_emul.c -- DESIGN TOOL (not product, not oracle): a sequential C restatement of
 * lz4_encode_seg.hip's algorithm (index, parse, splice, emit), lane by lane, to check its
 * output decodes with the reference and to count its work without a GPU.
 *
 *   gcc -O2 -o /tmp/seg_emul tools/seg_emul.c oracle/synth.c -ldl && /tmp/seg_emul [nblocks]
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void synth_blocks(uint8_t *out, int n, long long stride, long long first, int nb, int kind);

enum { THREADS = 1024, SEG = 64, STRIDE = 4, HLOG = 11, NB = 1 << HLOG, CAPX = 64, NREC = 13,
       DEPTH = 4 };

static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint32_t shash(uint32_t x, uint32_t b4) {
    uint32_t lo = x & 0xFFFFFF, hi = (x >> 24) | ((b4 & 0xFF) << 8);
    return (lo * 0x9E3779u + hi * 0xC2B2AEu) >> (32 - HLOG);
}
static int extlen(int v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }
static int prefix16(const uint8_t *a, const uint8_t *b) {
    int l = 0;
    while (l < 16 && a[l] == b[l]) l++;
    return l;
}

static long g_probes, g_wave_iters;

/* returns the compressed size written to out */
static int encode(const uint8_t *src, int n, uint8_t *out)
{
    static uint8_t blk[65536 + 64];
    static uint16_t pos[16384];
    static uint32_t offs[NB + 1];
    static uint32_t rec[THREADS][NREC];
    static int nrec[THREADS];
    memset(blk, 0, sizeof blk);
    memcpy(blk, src, n);
    /* index: positions 4i <= n-13, stable by position within bucket */
    int nidx = n >= 13 ? (n - 13) / STRIDE + 1 : 0;
    uint32_t cnt[NB] = {0};
    for (int i = 0; i < nidx; i++) cnt[shash(rd32(blk + 4 * i), blk[4 * i + 4])]++;
    uint32_t run = 0;
    for (int h = 0; h < NB; h++) { offs[h] = run; run += cnt[h]; }
    offs[NB] = run;
    uint32_t cur[NB];
    memcpy(cur, offs, sizeof cur);
    for (int i = 0; i < nidx; i++) pos[cur[shash(rd32(blk + 4 * i), blk[4 * i + 4])]++] = (uint16_t)(4 * i);
    /* parse */
    const int mfl = n - 12, mlim = n - 5;
    long wmax = 0;
    for (int t = 0; t < THREADS; t++) {
        int s0 = t * SEG, k = 0;
        long it = 0;
        nrec[t] = 0;
        if (s0 < n) {
            int s1 = s0 + SEG < n ? s0 + SEG : n, capE = s1 + CAPX < mfl ? s1 + CAPX : mfl;
            int q = s0 > 1 ? s0 : 1, anchor = s0;
            while (q < s1 && q <= mfl && k < NREC) {
                it++;
                uint32_t h = shash(rd32(blk + q), blk[q + 4]);
                int lo = offs[h], hi = offs[h + 1], blo = lo;
                while (lo < hi) { int mid = (lo + hi) >> 1; if (pos[mid] < q) lo = mid + 1; else hi = mid; }
                int room = capE - q, best = 0, bestc = 0;
                for (int d = 0; d < DEPTH; d++) {
                    int j = lo - 1 - d;
                    if (j >= blo) {
                        int c = pos[j], l = prefix16(blk + q, blk + c);
                        if (l > room) l = room;
                        if (l > best) { best = l; bestc = c; }
                    }
                }
                if (best < 4) { q++; continue; }
                int len = best;
                if (best == 16) {
                    while (len < room) {
                        int l = prefix16(blk + q + len, blk + bestc + len);
                        len += l;
                        it++;
                        if (l < 16) break;
                    }
                    if (len > room) len = room;
                }
                int m = q, c = bestc;
                while (m > anchor && c > 0 && blk[m - 1] == blk[c - 1]) { m--; c--; len++; }
                rec[t][k++] = (uint32_t)(m - s0) | ((uint32_t)len << 6) | ((uint32_t)(m - c) << 16);
                anchor = m + len;
                q = anchor;
            }
        }
        nrec[t] = k;
        g_probes += it;
        if (it > wmax) wmax = it;
        if ((t & 63) == 63) { g_wave_iters += wmax; wmax = 0; }
    }
    /* splice (sequential over lanes: the kernel's rules) -> sequences, then emit */
    static uint32_t sq_m[65536], sq_len[65536], sq_off[65536], sq_lit0[65536];
    int ns = 0;
    uint32_t cover = 0;
    for (int t = 0; t < THREADS; t++) {
        uint32_t pe = cover;
        int s0 = t * SEG, k = 0;
        for (int r = 0; r < nrec[t]; r++) {
            uint32_t w = rec[t][r], m = s0 + (w & 63), len = (w >> 6) & 1023, off = w >> 16, e = m + len;
            if (e <= pe) continue;
            if (m < pe) { len = e - pe; m = pe; if (len < 4) continue; }
            k++;
            if (k == 1 && ns > 0 && m == cover && sq_m[ns - 1] + sq_len[ns - 1] == cover && off == sq_off[ns - 1]) {
                sq_len[ns - 1] += len;   /* continuation of the covering match */
            } else {
                sq_lit0[ns] = pe; sq_m[ns] = m; sq_len[ns] = len; sq_off[ns] = off; ns++;
            }
            pe = e;
        }
        if (nrec[t]) {   /* coverage after this segment: f(c) = c + 4 <= e ? e : c */
            uint32_t w = rec[t][nrec[t] - 1], e = s0 + (w & 63) + ((w >> 6) & 1023);
            if (cover + 4 <= e) cover = e;
        }
    }
    int o = 0;
    for (int i = 0; i < ns; i++) {
        int lit = sq_m[i] - sq_lit0[i], ml = sq_len[i] - 4;
        out[o++] = (uint8_t)(((lit < 15 ? lit : 15) << 4) | (ml < 15 ? ml : 15));
        if (lit >= 15) { int v = lit - 15; for (; v >= 255; v -= 255) out[o++] = 255; out[o++] = v; }
        memcpy(out + o, blk + sq_lit0[i], lit);
        o += lit;
        out[o++] = sq_off[i] & 255;
        out[o++] = sq_off[i] >> 8;
        if (ml >= 15) { int v = ml - 15; for (; v >= 255; v -= 255) out[o++] = 255; out[o++] = v; }
    }
    int last = n - cover;
    out[o++] = (uint8_t)((last < 15 ? last : 15) << 4);
    if (last >= 15) { int v = last - 15; for (; v >= 255; v -= 255) out[o++] = 255; out[o++] = v; }
    memcpy(out + o, blk + cover, last);
    o += last;
    int litonly = 1 + extlen(n) + n;
    if (o >= litonly) {
        int h = 0;
        out[h++] = n >= 15 ? 0xF0 : n << 4;
        if (n >= 15) { int v = n - 15; for (; v >= 255; v -= 255) out[h++] = 255; out[h++] = v; }
        memcpy(out + h, src, n);
        return litonly;
    }
    return o;
}

int main(int argc, char **argv)
{
    int nb = argc > 1 ? atoi(argv[1]) : 64;
    void *ref = dlopen("oracle/_ref/libape_lz4_ref.so", RTLD_NOW);
    int (*dec)(const char *, char *, int, int) = ref ? dlsym(ref, "APE_LZ4_decompress_safe") : NULL;
    int (*cmp)(const char *, char *, int, int) = ref ? dlsym(ref, "APE_LZ4_compress_default") : NULL;
    if (!dec) { fprintf(stderr, "need oracle/_ref\n"); return 2; }
    const int n = 65536;
    uint8_t *in = malloc((size_t)n * nb), *out = malloc(70000), *back = malloc(n), *rout = malloc(70000);
    for (int kind = 1; kind >= 0; kind--) {
        synth_blocks(in, n, n, 0, nb, kind);
        long tot = 0, rtot = 0, bad = 0;
        g_probes = g_wave_iters = 0;
        for (int b = 0; b < nb; b++) {
            const uint8_t *s = in + (size_t)b * n;
            int c = encode(s, n, out);
            if (b < 4) printf("block %d: %d\n", b, c);
            tot += c;
            rtot += cmp((const char *)s, (char *)rout, n, 70000);
            int r = dec((const char *)out, (char *)back, c, n);
            if (r != n || memcmp(back, s, n)) bad++;
            r = dec((const char *)out, (char *)back, c, n - 1);
            if (r >= 0) bad++;
        }
        printf("kind %d: ratio %.4f (reference %.4f), bad %ld, probes/blk %.0f, wave-iters/blk %.0f\n",
               kind, (double)n * nb / tot, (double)n * nb / rtot, bad, (double)g_probes / nb,
               (double)g_wave_iters / nb);
    }
    /* odd sizes and contents */
    long bad = 0;
    for (int k = 0; k < 400; k++) {
        int m = k < 40 ? k : (int)((k * 7919u) % 65537);
        uint8_t *s = in;
        for (int i = 0; i < m; i++) s[i] = (k % 3 == 0) ? 0 : (k % 3 == 1) ? (uint8_t)(i % 7) : in[i];
        int c = encode(s, m, out);
        if (k == 3 || k == 6) printf("size %d content %d: %d bytes\n", m, k % 3, c);
        int r = dec((const char *)out, (char *)back, c, m);
        if (r != m || memcmp(back, s, m)) { bad++; if (bad < 5) printf("bad size %d r %d c %d\n", m, r, c); }
    }
    printf("odd sizes: bad %ld\n", bad);
    return 0;
}
