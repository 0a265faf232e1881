/* enc_model.c -- DESIGN TOOL (not product, not oracle): CPU model of candidate
 * policies for a round-parallel LZ4 match finder, to compare compression ratio
 * against the reference encoder before committing a GPU design.
 *
 *   gcc -O2 -o /tmp/enc_model tools/enc_model.c oracle/synth.c && /tmp/enc_model
 *
 * Policies (all greedy parses, valid LZ4 limits: match start <= n-12, end <= n-5):
 *   insert = 0: every position inserted (hash -> latest earlier position)
 *   insert = 1: only walked positions (literal positions + match starts) and
 *               match_end - 2, as the reference does
 *   rounds R:   lookups during round [R0, R0+R) see only insertions of earlier rounds
 *   inround:    also try the earliest same-hash position inside the round
 *   back:       backward match extension into pending literals (reference catch-up)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void synth_blocks(uint8_t *out, int n, long long stride, long long first, int nb, int kind);

static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

static int ext(int v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }

/* hash variants for model2: 0 = reference 5-byte multiplicative, 1 = two 24-bit
 * multiplies (full-rate on CDNA: v_mul_u32_u24) */
static int g_hash = 0;
static uint32_t hsh(const uint8_t *p, int hlog) {
    if (g_hash == 0) return (uint32_t)((rd64(p) * 889523592379ULL) >> (40 - hlog)) & ((1u << hlog) - 1);
    uint32_t x = rd32(p), b4 = p[4];
    uint32_t lo = x & 0xFFFFFF, hi = (x >> 24) | (b4 << 8);
    uint32_t v = lo * 0x9E3779u + hi * 0xC2B2AEu;   /* 24-bit x 24-bit, low 32 bits */
    return v >> (32 - hlog);
}

static long model(const uint8_t *in, int n, int hlog, int insert, int R, int inround, int back)
{
    const int H = 1 << hlog;
    int *tab = malloc(sizeof(int) * H);
    for (int i = 0; i < H; i++) tab[i] = -1;
    int *cand = malloc(sizeof(int) * n), *cand2 = malloc(sizeof(int) * n);
    uint32_t *hh = malloc(sizeof(uint32_t) * n);
    const int mstart = n - 12, mlimit = n - 5;
    long out = 0;
    int anchor = 0, p = 0;
    for (int r0 = 0; r0 < n; r0 += R) {
        int r1 = r0 + R < n ? r0 + R : n;
        for (int q = r0; q < r1; q++) {
            if (q + 8 <= n) hh[q] = (uint32_t)((rd64(in + q) * 889523592379ULL) >> (40 - hlog)) & (H - 1);
            else hh[q] = 0;
            cand[q] = (q <= n - 5) ? tab[hh[q]] : -1;
            cand2[q] = -1;
        }
        if (inround) {
            for (int q = r0; q < r1 && q <= n - 5; q++) {
                for (int j = r0; j < q; j++)
                    if (hh[j] == hh[q]) { cand2[q] = j; break; }
            }
        }
        if (insert == 0)
            for (int q = r0; q < r1 && q <= n - 5; q++) tab[hh[q]] = q;
        /* walk this round */
        while (p < r1) {
            int best = 0, bc = -1;
            if (p >= 1 && p <= mstart) {
                int cs[2] = {cand[p], cand2[p]};
                for (int k = 0; k < 2; k++) {
                    int c = cs[k];
                    if (c < 0 || c >= p || p - c > 65535) continue;
                    if (rd32(in + c) != rd32(in + p)) continue;
                    int l = 4;
                    while (p + l < mlimit && in[p + l] == in[c + l]) l++;
                    if (l > best || (l == best && c > bc)) { best = l; bc = c; }
                }
            }
            if (insert == 1 && p <= n - 5) tab[hh[p]] = p; /* walked position */
            if (best >= 4) {
                int m = p, c = bc, len = best;
                if (back)
                    while (m > anchor && c > 0 && in[m - 1] == in[c - 1]) { m--; c--; len++; }
                int lit = m - anchor;
                out += 1 + ext(lit) + lit + 2 + ext(len - 4);
                p = m + len;
                anchor = p;
                if (insert == 1 && p - 2 <= n - 5) tab[hh[p - 2] = (uint32_t)((rd64(in + p - 2) * 889523592379ULL) >> (40 - hlog)) & (H - 1)] = p - 2;
            } else {
                p++;
            }
        }
    }
    int lit = n - anchor;
    out += 1 + ext(lit) + lit;
    free(tab); free(cand); free(cand2); free(hh);
    return out;
}


/* Wave-per-block policy: rounds of R positions start at the walk position P;
 * lookups see the table as of the round start (walked positions + end-2 of
 * earlier rounds); in-round candidate = earliest lane with the same low `sb`
 * hash bits; backward extension capped at `bcap` bytes. */
static long model2(const uint8_t *in, int n, int hlog, int R, int sb, int bcap, int end2)
{
    const int H = 1 << hlog;
    int *tab = calloc(H, sizeof(int));
    int *cand = malloc(sizeof(int) * (R + 1)), *cand2 = malloc(sizeof(int) * (R + 1));
    uint32_t *hh = malloc(sizeof(uint32_t) * (R + 1));
    int *scr = malloc(sizeof(int) * (1 << sb));
    const int mstart = n - 12, mlimit = n - 5;
    long out = 0;
    int anchor = 0, p = 0;
    while (p < n) {
        const int P = p, r1 = P + R < n ? P + R : n;
        for (int i = 0; i < (1 << sb); i++) scr[i] = -1;
        for (int q = P; q < r1; q++) {
            hh[q - P] = (q + 8 <= n) ? hsh(in + q, hlog) : 0;
            cand[q - P] = tab[hh[q - P]];
            int k = hh[q - P] & ((1 << sb) - 1);
            cand2[q - P] = -1;
            if (scr[k] < 0) scr[k] = q; else cand2[q - P] = scr[k];
        }
        int walked[4096]; int nw = 0; int ends[4096]; int ne = 0;
        while (p < r1) {
            int best = 0, bc = -1;
            if (p >= 1 && p <= mstart) {
                int cs[2] = {cand[p - P], cand2[p - P]};
                for (int k = 0; k < 2; k++) {
                    int c = cs[k];
                    if (c < 0 || c >= p || p - c > 65535) continue;
                    if (rd32(in + c) != rd32(in + p)) continue;
                    int l = 4;
                    while (p + l < mlimit && in[p + l] == in[c + l]) l++;
                    if (l > best || (l == best && c > bc)) { best = l; bc = c; }
                }
            }
            walked[nw++] = p;
            if (best >= 4) {
                int m = p, c = bc, len = best, b = 0;
                while (b < bcap && m > anchor && c > 0 && in[m - 1] == in[c - 1]) { m--; c--; len++; b++; }
                int lit = m - anchor;
                out += 1 + ext(lit) + lit + 2 + ext(len - 4);
                p = m + len;
                anchor = p;
                ends[ne++] = p - 2;
            } else {
                p++;
            }
        }
        for (int i = 0; i < nw; i++) if (walked[i] <= n - 5 && walked[i] < r1) tab[hh[walked[i] - P]] = walked[i];
        if (end2) for (int i = 0; i < ne; i++) if (ends[i] + 8 <= n) tab[hsh(in + ends[i], hlog)] = ends[i];
    }
    int lit = n - anchor;
    out += 1 + ext(lit) + lit;
    free(tab); free(cand); free(cand2); free(hh); free(scr);
    return out;
}

/* Producer/consumer policy: every position inserted (latest earlier position
 * with the same hash), chunks of R positions see the table as of the chunk
 * start (plus `lag` chunks of staleness for parallel producers), in-round
 * candidate = earliest lane with the same low `sb` hash bits, back-ext cap. */
static long model3(const uint8_t *in, int n, int hlog, int R, int lag, int sb, int bcap)
{
    const int H = 1 << hlog;
    int *tab = calloc(H, sizeof(int));
    int *cand = malloc(sizeof(int) * n), *cand2 = malloc(sizeof(int) * n);
    uint32_t *hh = malloc(sizeof(uint32_t) * n);
    int *scr = malloc(sizeof(int) * (1 << sb));
    for (int q = 0; q < n; q++)
        hh[q] = (q + 8 <= n) ? (uint32_t)((rd64(in + q) * 889523592379ULL) >> (40 - hlog)) & (H - 1) : 0;
    /* candidates per chunk: table state after chunks < k - lag */
    int done = 0;  /* positions inserted so far */
    for (int r0 = 0; r0 < n; r0 += R) {
        int lim = r0 - lag * R;
        for (; done < lim; done++) if (done <= n - 5) tab[hh[done]] = done;
        int r1 = r0 + R < n ? r0 + R : n;
        for (int i = 0; i < (1 << sb); i++) scr[i] = -1;
        for (int q = r0; q < r1; q++) {
            cand[q] = (q <= n - 5) ? tab[hh[q]] : -1;
            int k = hh[q] & ((1 << sb) - 1);
            cand2[q] = -1;
            if (scr[k] < 0) scr[k] = q; else cand2[q] = scr[k];
        }
    }
    const int mstart = n - 12, mlimit = n - 5;
    long out = 0;
    int anchor = 0, p = 0;
    while (p < n) {
        int best = 0, bc = -1;
        if (p >= 1 && p <= mstart) {
            int cs[2] = {cand[p], cand2[p]};
            for (int k = 0; k < 2; k++) {
                int c = cs[k];
                if (c < 0 || c >= p || p - c > 65535) continue;
                if (rd32(in + c) != rd32(in + p)) continue;
                int l = 4;
                while (p + l < mlimit && in[p + l] == in[c + l]) l++;
                if (l > best || (l == best && c > bc)) { best = l; bc = c; }
            }
        }
        if (best >= 4) {
            int m = p, c = bc, len = best, b = 0;
            while (b < bcap && m > anchor && c > 0 && in[m - 1] == in[c - 1]) { m--; c--; len++; b++; }
            int lit = m - anchor;
            out += 1 + ext(lit) + lit + 2 + ext(len - 4);
            p = m + len;
            anchor = p;
        } else p++;
    }
    int lit = n - anchor;
    out += 1 + ext(lit) + lit;
    free(tab); free(cand); free(cand2); free(hh); free(scr);
    return out;
}


/* Kernel policy (lz4_encode.hip): fixed 64-position chunks; the table lags `lag`
 * chunks (walked positions + match_end - 2); L = earliest lane of the chunk with the
 * same low `sb` hash bits; catch-up <= 4.  pol 0: T and L measured in full, longer
 * wins (tie: closer); pol 7: L measured to 12 bytes only, taken when T is shorter
 * than 12 and L at least as long (the product since the L-12 change). */
static int g_tsize = 8192;   /* model4 table entries (hash scaled onto [0, g_tsize)) */
static uint32_t hslot(const uint8_t *p) {
    if (g_tsize == 8192) return hsh(p, 13);
    uint32_t x = rd32(p), b4 = p[4];
    uint32_t lo = x & 0xFFFFFF, hi = (x >> 24) | (b4 << 8);
    uint32_t v = lo * 0x9E3779u + hi * 0xC2B2AEu;
    return (uint32_t)(((uint64_t)(v >> 16) * (uint32_t)g_tsize) >> 16);
}
static long model4(const uint8_t *in, int n, int lag, int pol, int sb, int lmax)
{
    int tab[8192];
    for (int i = 0; i < 8192; i++) tab[i] = -1;
    int *cT = malloc(4 * n), *cL = malloc(4 * n), scr[256];
    int *ins = malloc(8 * n), *insc = malloc(8 * n), nins = 0, done = 0;
    const int mstart = n - 12, mlimit = n - 5, nch = (n + 63) / 64;
    long out = 0;
    int anchor = 0, p = 0;
    g_hash = 1;
    for (int k = 0; k < nch; k++) {
        while (done < nins && insc[done] <= k - lag - 1) {
            int q = ins[done++];
            if (q + 8 <= n) tab[hslot(in + q)] = q;
        }
        int r0 = 64 * k, r1 = r0 + 64 < n ? r0 + 64 : n;
        for (int i = 0; i < (1 << sb); i++) scr[i] = -1;
        for (int q = r0; q < r1; q++) {
            uint32_t h = q + 8 <= n ? hslot(in + q) : 0;
            int s2 = (q + 8 <= n ? hsh(in + q, 13) : 0) & ((1 << sb) - 1);
            cT[q] = tab[h];
            cL[q] = -1;
            if (scr[s2] < 0) scr[s2] = q; else if (k < lmax) cL[q] = scr[s2];
        }
        while (p < r1) {
            int best = 0, bc = -1;
            if (p >= 1 && p <= mstart) {
                int cs[2] = {cT[p], cL[p]}, ok[2], l[2] = {0, 0};
                for (int j = 0; j < 2; j++) {
                    int c = cs[j];
                    ok[j] = !(c < 0 || c >= p || p - c > 65535) && rd32(in + c) == rd32(in + p);
                    if (ok[j]) { l[j] = 4; while (p + l[j] < mlimit && in[p + l[j]] == in[c + l[j]]) l[j]++; }
                }
                int pick = -1;
                if (pol == 7) {
                    int l12 = l[1] < 12 ? l[1] : 12;
                    if (ok[1] && (!ok[0] || (l[0] < 12 && l12 >= l[0]))) pick = 1;
                    else if (ok[0]) pick = 0;
                } else {
                    if (ok[0]) pick = 0;
                    if (ok[1] && (pick < 0 || l[1] >= l[0])) pick = 1;
                }
                if (pick >= 0) { best = l[pick]; bc = cs[pick]; }
            }
            ins[nins] = p; insc[nins++] = k;
            if (best >= 4) {
                int m = p, c = bc, len = best, b = 0;
                while (b < 4 && m > anchor && c > 0 && in[m - 1] == in[c - 1]) { m--; c--; len++; b++; }
                int lit = m - anchor;
                out += 1 + ext(lit) + lit + 2 + ext(len - 4);
                p = m + len;
                anchor = p;
                ins[nins] = p - 2; insc[nins++] = (p - 2) / 64 > k ? (p - 2) / 64 : k;
            } else p++;
        }
    }
    out += 1 + ext(n - anchor) + n - anchor;
    free(cT); free(cL); free(ins); free(insc);
    return out;
}


/* Round 6: key length and T-probe density.  The product policy of
 * model4 (pol 7, lag 3, 6 in-chunk bits, catch-up <= 4, table scaled onto g_tsize entries by
 * v_mul_hi_u32 as lz4_encode.hip does) with the hash over `key` bytes (5..8, the GPU's
 * two / three full-rate 24-bit multiplies) and the table candidate T probed only at
 * positions p % tmod == 0 (every walked position is still inserted; L everywhere).
 * Returns the compressed size, adds the block's sequence count to *nseq. */
static uint32_t hkey(const uint8_t *p, int key) {
    uint32_t x0 = rd32(p), x1 = rd32(p + 4);
    uint32_t lo = x0 & 0xFFFFFF, hi = (x0 >> 24) | (x1 << 8);
    if (key == 5) hi &= 0xFFFF;
    hi &= 0xFFFFFF;
    uint32_t v = lo * 0x9E3779u + hi * 0xC2B2AEu;
    if (key == 7) v += (x1 >> 16 & 0xFF) * 0x27D4EBu;         /* byte 6 */
    if (key == 8) v += (x1 >> 16) * 0x27D4EBu;                 /* bytes 6-7 */
    return v;
}
static uint32_t kslot(const uint8_t *p, int key) {
    return (uint32_t)(((uint64_t)hkey(p, key) * (uint32_t)g_tsize) >> 32);
}
static int g_lag = 3, g_bcap = 4, g_noL = 0, g_near = 0, g_nearbits = 6, g_nearwin = 768, g_allins = 0, g_insd = 0;
static FILE *g_seqf = NULL;   /* SEQDUMP: (lit, match length, offset) int32 triples per sequence, -1 -1 -1 per block end */
/* SEQDUMP also prints, for the T gather of the HEAD policy: lanes with no candidate, a candidate
   <= 832 bytes back (in the ring at C1) that verifies / does not, one further back that verifies /
   does not, all lanes; distinct 64-byte lines per chunk, all lanes / near lanes on one line
   (profiles/r6_encoder_policy_ab.txt call 16) */
static long g_cnt[6], g_lines[3];
static long model5(const uint8_t *in, int n, int key, int tmod, long *nseq)
{
    int tab[8192], near[1024], tabold[64];
    for (int i = 0; i < 8192; i++) tab[i] = -1;
    for (int i = 0; i < 1024; i++) near[i] = -1;
    int *cT = malloc(4 * n), *cL = malloc(4 * n), scr[64];
    int *ins = malloc(8 * n), *insc = malloc(8 * n), nins = 0, done = 0;
    const int lag = g_lag, mstart = n - 12, mlimit = n - 5, nch = (n + 63) / 64;
    long out = 0;
    int anchor = 0, p = 0;
    for (int k = 0; k < nch; k++) {
        while (done < nins && insc[done] <= k - lag - 1) {
            int q = ins[done++];
            if (q + 8 <= n) tab[kslot(in + q, key)] = q;
        }
        int r0 = 64 * k, r1 = r0 + 64 < n ? r0 + 64 : n;
        for (int i = 0; i < 64; i++) scr[i] = -1;
        for (int q = r0; q < r1; q++) {
            uint32_t h = q + 8 <= n ? kslot(in + q, key) : 0;
            cT[q] = (q % tmod == 0) ? tab[h] : -1;
            tabold[q - r0] = tab[h];
            {
                const int c = cT[q];
                g_cnt[5]++;
                if (c < 4 || c >= q || q + 8 > n) g_cnt[0]++;
                else {
                    const int ok = rd32(in + c) == rd32(in + q);
                    g_cnt[(q - c <= 832 ? 1 : 3) + !ok]++;
                }
            }
            cL[q] = -1;
            if (g_near == 2) {
                /* one ds_max_rtn per lane on ((k+1) << 6 | 63 - lane) over 2^nearbits buckets,
                 * lanes in order: the first lane of a bucket gets the earliest lane of the last
                 * earlier chunk that had it, later lanes the earliest lane of this chunk */
                const int nb = h & ((1 << g_nearbits) - 1);
                const int r = near[nb] < 0 ? 0 : near[nb];
                const int w = ((k + 1) << 6) | (63 - (q - r0));
                if (w > r) near[nb] = w;
                const int c = 64 * (r >> 6) - 1 - (r & 63);
                if (r && q - c <= g_nearwin && (!g_noL || (r >> 6) != k + 1)) cL[q] = c;
                continue;
            }
            if (scr[h & 63] < 0) {
                scr[h & 63] = q;
                /* near: the latest position of the earlier chunks with the same low bits */
                const int nb = h & ((1 << g_nearbits) - 1);
                if (g_near && near[nb] >= 0 && q - near[nb] <= g_nearwin) cL[q] = near[nb];
            } else if (!g_noL) cL[q] = scr[h & 63];
        }
        {   /* distinct 64-B lines of the T gather (in[T-4, T+12) per valid lane, the lane's own p line
               otherwise): every lane, and with lanes whose candidate is <= 832 back verified from LDS */
            long ls[2][160]; int nl[2] = {0, 0};
            for (int q = r0; q < r1; q++) {
                const int c = cT[q], valid = c >= 4 && c < q && q + 8 <= n;
                for (int v = 0; v < 2; v++) {
                    const int use = valid && !(v && q - c <= 832);
                    const long a0 = use ? c - 4 : q, a1 = use ? c + 11 : q;
                    for (long L = a0 >> 6; L <= a1 >> 6; L++) {
                        int f = 0;
                        for (int i = 0; i < nl[v]; i++) f |= ls[v][i] == L;
                        if (!f) ls[v][nl[v]++] = L;
                    }
                }
            }
            g_lines[0] += nl[0]; g_lines[1] += nl[1]; g_lines[2]++;
        }
        if (g_near == 1)
            for (int q = r0; q < r1; q++) if (q + 8 <= n) near[kslot(in + q, key) & ((1 << g_nearbits) - 1)] = q;
        if (g_allins)   /* the producer inserts every position of the chunk after its lookups
                           (only over entries more than g_insd bytes back: the value the lane
                           read, so lanes of one chunk decide on the same old entry) */
            for (int q = r0; q < r1; q++) {
                if (q + 8 > n) continue;
                const uint32_t h = kslot(in + q, key);
                const int old = tabold[q - r0];
                if (old < 0 || q - old > g_insd) tab[h] = q;
            }
        while (p < r1) {
            int best = 0, bc = -1;
            if (p >= 1 && p <= mstart) {
                int cs[2] = {cT[p], cL[p]}, ok[2], l[2] = {0, 0};
                for (int j = 0; j < 2; j++) {
                    int c = cs[j];
                    ok[j] = !(c < 0 || c >= p || p - c > 65535) && rd32(in + c) == rd32(in + p);
                    if (ok[j]) { l[j] = 4; while (p + l[j] < mlimit && in[p + l[j]] == in[c + l[j]]) l[j]++; }
                }
                int pick = -1, l12 = l[1] < 12 ? l[1] : 12;
                if (ok[1] && (!ok[0] || (l[0] < 12 && l12 >= l[0]))) pick = 1;
                else if (ok[0]) pick = 0;
                if (pick >= 0) { best = l[pick]; bc = cs[pick]; }
            }
            if (!g_allins) { ins[nins] = p; insc[nins++] = k; }
            if (best >= 4) {
                int m = p, c = bc, len = best, b = 0;
                while (b < g_bcap && m > anchor && c > 0 && in[m - 1] == in[c - 1]) { m--; c--; len++; b++; }
                int lit = m - anchor;
                out += 1 + ext(lit) + lit + 2 + ext(len - 4);
                (*nseq)++;
                if (g_seqf) { const int t[3] = {lit, len, m - c}; fwrite(t, 4, 3, g_seqf); }
                p = m + len;
                anchor = p;
                if (!g_allins) { ins[nins] = p - 2; insc[nins++] = (p - 2) / 64 > k ? (p - 2) / 64 : k; }
            } else p++;
        }
    }
    out += 1 + ext(n - anchor) + n - anchor;
    if (g_seqf) { const int t[3] = {n - anchor, -1, -1}; fwrite(t, 4, 3, g_seqf); }
    free(cT); free(cL); free(ins); free(insc);
    return out;
}

static void key_study(const uint8_t *buf, int n, int nb, const char *what)
{
    if (getenv("LAGSTUDY")) {
        struct { int lag, bcap, ts, noL; } V[] = {{3,4,7200,0},{0,4,7200,0},{3,1000,7200,0},{3,4,8192,0},
            {0,1000,8192,0},{3,4,7200,1},{1,4,7200,0},{2,4,7200,0}};
        for (unsigned i = 0; i < sizeof(V)/sizeof(V[0]); i++) {
            g_lag = V[i].lag; g_bcap = V[i].bcap; g_tsize = V[i].ts; g_noL = V[i].noL;
            long tot = 0, nseq = 0;
            for (int b = 0; b < nb; b++) tot += model5(buf + (size_t)b * n, n, 5, 1, &nseq);
            printf("%-5s lag %d bcap %4d table %d noL %d  ratio %.4f  seq %7.1f\n", what, g_lag, g_bcap,
                   g_tsize, g_noL, (double)n * nb / tot, (double)nseq / nb);
        }
        g_lag = 3; g_bcap = 4; g_noL = 0;
    }
    g_tsize = getenv("TSIZE") ? atoi(getenv("TSIZE")) : 7200;
    if (getenv("SEQDUMP")) {   /* the HEAD policy's parse of these blocks -> sequences */
        g_allins = 1; g_noL = 1; g_tsize = 7328;
        g_seqf = fopen(getenv("SEQDUMP"), "wb");
        long tot = 0, nseq = 0;
        for (int b = 0; b < nb; b++) tot += model5(buf + (size_t)b * n, n, 7, 1, &nseq);
        fclose(g_seqf);
        g_seqf = NULL;
        printf("%-5s HEAD policy ratio %.4f seq %.1f\n", what, (double)n * nb / tot, (double)nseq / nb);
        printf("lanes: none %.3f  near ok %.3f bad %.3f  far ok %.3f bad %.3f\n", (double)g_cnt[0] / g_cnt[5],
               (double)g_cnt[1] / g_cnt[5], (double)g_cnt[2] / g_cnt[5], (double)g_cnt[3] / g_cnt[5],
               (double)g_cnt[4] / g_cnt[5]);
        printf("gather lines/chunk: all %.2f  far-only %.2f\n", (double)g_lines[0] / g_lines[2], (double)g_lines[1] / g_lines[2]);
        exit(0);
    }
    if (getenv("ALLINS")) {
        const int ds[] = {0, 0, 256, 1024, 4096, 16384, 1 << 20};
        const int nv = getenv("ALLINS")[0] == '2' ? 2 : 7;
        g_noL = getenv("NOL") ? 1 : 0;
        g_bcap = getenv("BCAP") ? atoi(getenv("BCAP")) : 4;
        for (int key = 6; key <= 8; key++)
            for (int ai = 0; ai < nv; ai++) {
                g_allins = ai > 0; g_insd = ds[ai];
                long tot = 0, nseq = 0;
                const int tm = getenv("TMOD") ? atoi(getenv("TMOD")) : 1;
                for (int b = 0; b < nb; b++) tot += model5(buf + (size_t)b * n, n, key, tm, &nseq);
                printf("%-5s key %d all-positions %d  dist %7d  ratio %.4f  seq %7.1f\n", what, key, g_allins, g_insd,
                       (double)n * nb / tot, (double)nseq / nb);
            }
        g_allins = 0;
        return;
    }
    if (getenv("NEAR")) {
        const int nbits[] = {6, 7, 8};
        const int tm = atoi(getenv("NEAR"));
        const int mode = getenv("NEARMODE") ? atoi(getenv("NEARMODE")) : 1;
        for (int key = 5; key <= 8; key++)
            for (int i = -1; i < 3; i++) {
                g_near = i >= 0 ? mode : 0; g_nearbits = i >= 0 ? nbits[i] : 6;
                long tot = 0, nseq = 0;
                for (int b = 0; b < nb; b++) tot += model5(buf + (size_t)b * n, n, key, tm, &nseq);
                printf("%-5s key %d T every %d near %d bits %2d  ratio %.4f  seq %7.1f\n", what, key, tm, g_near,
                       g_nearbits, (double)n * nb / tot, (double)nseq / nb);
            }
        g_near = 0;
        return;
    }
    for (int tmod = 1; tmod <= 2; tmod++)
        for (int key = 5; key <= 8; key++) {
            long tot = 0, nseq = 0;
            for (int b = 0; b < nb; b++) tot += model5(buf + (size_t)b * n, n, key, tmod, &nseq);
            printf("%-5s key %d  T every %d  ratio %.4f  sequences/block %7.1f\n", what, key, tmod,
                   (double)n * nb / tot, (double)nseq / nb);
        }
    g_tsize = 8192;
}

int main(int argc, char **argv)
{
    const int n = 65536, nb = argc > 1 ? atoi(argv[1]) : 16;
    uint8_t *buf = malloc((size_t)n * nb + 16);
    synth_blocks(buf, n, n, 0, nb, 1);
    if (argc > 2) {   /* key study: App. C blocks, then the blocks of file argv[2] */
        key_study(buf, n, nb, "appC");
        FILE *f = fopen(argv[2], "rb");
        if (!f) return 1;
        const int nt = (int)fread(buf, 1, (size_t)n * nb, f) / n;
        fclose(f);
        key_study(buf, n, nt, "file");
        free(buf);
        return 0;
    }
    struct { int hlog, insert, R, inround, back; const char *name; } P[] = {
        {12, 0, 2048, 1, 0, "current: 4096, all positions, 2048 rounds, in-round"},
        {13, 0, 2048, 1, 0, "8192, all positions, 2048 rounds, in-round"},
        {13, 1, 1, 0, 0, "8192, walked only, sequential (ref-like)"},
        {13, 1, 1, 0, 1, "8192, walked only, sequential, back-ext (ref-like)"},
        {13, 1, 64, 0, 1, "8192, walked only, 64 rounds, back-ext"},
        {13, 1, 64, 1, 1, "8192, walked only, 64 rounds, in-round, back-ext"},
        {12, 1, 64, 1, 1, "4096, walked only, 64 rounds, in-round, back-ext"},
        {13, 1, 256, 1, 1, "8192, walked only, 256 rounds, in-round, back-ext"},
        {13, 1, 2048, 1, 1, "8192, walked only, 2048 rounds, in-round, back-ext"},
        {12, 0, 2048, 1, 1, "4096, all positions, 2048 rounds, in-round, back-ext"},
        {13, 0, 2048, 1, 1, "8192, all positions, 2048 rounds, in-round, back-ext"},
        {14, 0, 2048, 1, 1, "16384, all positions, 2048 rounds, in-round, back-ext"},
    };
    for (unsigned k = 0; k < sizeof(P) / sizeof(P[0]); k++) {
        long tot = 0;
        for (int b = 0; b < nb; b++)
            tot += model(buf + (size_t)b * n, n, P[k].hlog, P[k].insert, P[k].R, P[k].inround, P[k].back);
        printf("%-62s ratio %.4f\n", P[k].name, (double)n * nb / tot);
    }
    struct { int hlog, R, sb, bcap, end2; } Q[] = {
        {13, 64, 8, 4, 1}, {13, 64, 8, 4, 0}, {13, 64, 8, 0, 1}, {13, 64, 8, 64, 1}, {13, 64, 0, 4, 1},
        {12, 64, 8, 4, 1}, {13, 128, 8, 4, 1}, {13, 64, 6, 4, 1}, {14, 64, 8, 4, 1}};
    for (unsigned k = 0; k < 2 * sizeof(Q) / sizeof(Q[0]); k++) {
        g_hash = k >= sizeof(Q) / sizeof(Q[0]);
        if (g_hash && k % (sizeof(Q) / sizeof(Q[0])) != 0) continue;
        long tot = 0;
        for (int b = 0; b < nb; b++)
            tot += model2(buf + (size_t)b * n, n, Q[k % (sizeof(Q) / sizeof(Q[0]))].hlog,
                          Q[k % (sizeof(Q) / sizeof(Q[0]))].R, Q[k % (sizeof(Q) / sizeof(Q[0]))].sb,
                          Q[k % (sizeof(Q) / sizeof(Q[0]))].bcap, Q[k % (sizeof(Q) / sizeof(Q[0]))].end2);
        const unsigned kq = k % (sizeof(Q) / sizeof(Q[0]));
        printf("wave: hash %d hlog %d R %d scratch-bits %d back-cap %d end-2 %d  ratio %.4f\n", g_hash,
               Q[kq].hlog, Q[kq].R, Q[kq].sb, Q[kq].bcap, Q[kq].end2, (double)n * nb / tot);
    }
    struct { int hlog, R, lag, sb, bcap; } T3[] = {
        {13, 64, 0, 8, 4}, {13, 64, 1, 8, 4}, {13, 64, 2, 8, 4}, {12, 64, 0, 8, 4}, {12, 64, 1, 8, 4},
        {13, 64, 0, 8, 64}, {13, 64, 0, 6, 4}, {14, 64, 1, 8, 4}, {12, 128, 0, 8, 4}};
    for (unsigned k = 0; k < sizeof(T3) / sizeof(T3[0]); k++) {
        long tot = 0;
        for (int b = 0; b < nb; b++)
            tot += model3(buf + (size_t)b * n, n, T3[k].hlog, T3[k].R, T3[k].lag, T3[k].sb, T3[k].bcap);
        printf("prod/cons: hlog %d R %d lag %d scratch-bits %d back-cap %d       ratio %.4f\n", T3[k].hlog,
               T3[k].R, T3[k].lag, T3[k].sb, T3[k].bcap, (double)n * nb / tot);
    }
    for (int pol = 0; pol <= 7; pol += 7) {
        long tot = 0;
        for (int b = 0; b < nb; b++) tot += model4(buf + (size_t)b * n, n, 3, pol, 6, 1 << 20);
        printf("kernel policy: lag 3, L bits 6, pol %d                  ratio %.4f\n", pol,
               (double)n * nb / tot);
    }
    {   /* the in-chunk candidate only for the first lmax chunks (short offsets cluster at
           the block start: App. C offsets are uniform over the window so far) */
        const int lm[] = {0, 2, 4, 8, 16, 32, 64, 128, 1 << 20};
        for (unsigned k = 0; k < sizeof(lm) / sizeof(lm[0]); k++) {
            long tot = 0;
            for (int b = 0; b < nb; b++) tot += model4(buf + (size_t)b * n, n, 3, 7, 6, lm[k]);
            printf("kernel policy pol 7, L for the first %7d chunks          ratio %.4f\n", lm[k],
                   (double)n * nb / tot);
        }
    }
    for (int lag = 3; lag <= 6; lag++) {
        long tot = 0;
        g_tsize = 6912;
        for (int b = 0; b < nb; b++) tot += model4(buf + (size_t)b * n, n, lag, 7, 6, 1 << 20);
        printf("kernel policy pol 7, table 6912, lag %d                   ratio %.4f\n", lag,
               (double)n * nb / tot);
        g_tsize = 8192;
    }
    {
        const int ts[] = {8192, 7552, 7168, 7040, 6656, 6144, 4096};
        for (unsigned k = 0; k < sizeof(ts) / sizeof(ts[0]); k++) {
            long tot = 0;
            g_tsize = ts[k];
            for (int b = 0; b < nb; b++) tot += model4(buf + (size_t)b * n, n, 3, 7, 6, 1 << 20);
            printf("kernel policy pol 7, table of %5d entries                 ratio %.4f\n", ts[k],
                   (double)n * nb / tot);
        }
        g_tsize = 8192;
    }
    free(buf);
    return 0;
}
