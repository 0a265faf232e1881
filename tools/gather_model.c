/* gather_model.c -- DESIGN TOOL (not product, not oracle): how many distinct 128-byte lines
 * the encoder's per-step candidate gathers touch (the vector-memory work that bounds
 * lz4_encode_kernel: TA/TD ~83-96 % busy, profiles/r4_mem_passes.json), and how many a
 * pre-filter would keep.  Follows tools/enc_model.c model4 (the product's parse: 64-lane
 * chunks, table of walked positions + match_end - 2 with a lag of 3 chunks, in-chunk
 * candidate L, pol 7), table of 7200 entries.
 *   gcc -O2 -o /tmp/gather_model tools/gather_model.c oracle/synth.c && /tmp/gather_model 16
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void synth_blocks(uint8_t *out, int n, long long stride, long long first, int nb, int kind);
static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static int ext(int v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }
static const int TS = 7200;
static uint32_t hslot(const uint8_t *p) {
    uint32_t x = rd32(p), b4 = p[4];
    uint32_t lo = x & 0xFFFFFF, hi = (x >> 24) | (b4 << 8);
    uint32_t v = lo * 0x9E3779u + hi * 0xC2B2AEu;
    return (uint32_t)(((uint64_t)v * (uint32_t)TS) >> 32);
}
static uint32_t htag(const uint8_t *p) {   /* 8 more key bits: a second multiply */
    uint32_t x = rd32(p), b4 = p[4];
    return ((x * 0x2545F491u) ^ (b4 * 0x9E37u)) >> 24;
}
static int lines(uint32_t *a, int n) {   /* distinct 128-B lines among byte ranges [a, a+16) */
    uint32_t l[128];
    int k = 0;
    for (int i = 0; i < n; i++) {
        uint32_t x = a[i] >> 7, y = (a[i] + 15) >> 7;
        l[k++] = x;
        if (y != x) l[k++] = y;
    }
    int d = 0;
    for (int i = 0; i < k; i++) {
        int seen = 0;
        for (int j = 0; j < i; j++) if (l[j] == l[i]) { seen = 1; break; }
        d += !seen;
    }
    return d;
}

int main(int argc, char **argv)
{
    const int n = 65536, nb = argc > 1 ? atoi(argv[1]) : 16, lag = 3;
    const int pol = argc > 2 ? atoi(argv[2]) : 7;   /* 7: the product; 8: T whenever it verifies, else L;
                                                       9: L whenever it verifies, else T */
    uint8_t *buf = malloc((size_t)n * nb + 16);
    synth_blocks(buf, n, n, 0, nb, 1);
    long steps = 0, l_all = 0, l_valid = 0, l_ver = 0, l_tag = 0, lanes = 0, valid = 0, ver = 0,
         tagok = 0, out = 0, members = 0, memT = 0;
    for (int b = 0; b < nb; b++) {
        const uint8_t *in = buf + (size_t)b * n;
        static int tab[8192];
        static uint8_t tg[8192];
        for (int i = 0; i < TS; i++) { tab[i] = 0; tg[i] = 0; }
        int *ins = malloc(8 * n), *insc = malloc(8 * n), nins = 0, done = 0;
        int *cT = malloc(4 * n), *cL = malloc(4 * n), *tok = malloc(4 * n), scr[64];
        const int mstart = n - 12, mlimit = n - 5, nch = n / 64;
        int anchor = 0, p = 0;
        for (int k = 0; k < nch; k++) {
            while (done < nins && insc[done] <= k - lag - 1) {
                int q = ins[done++];
                if (q + 8 <= n) { tab[hslot(in + q)] = q; tg[hslot(in + q)] = (uint8_t)htag(in + q); }
            }
            const int r0 = 64 * k;
            uint32_t a_all[64], a_valid[64], a_ver[64], a_tag[64];
            int n_valid = 0, n_ver = 0, n_tag = 0;
            for (int i = 0; i < 64; i++) scr[i] = -1;
            for (int q = r0; q < r0 + 64; q++) {
                const int ok8 = q + 8 <= n;
                uint32_t h = ok8 ? hslot(in + q) : 0;
                cT[q] = tab[h];
                int s2 = (ok8 ? (h & 63) : 0);
                cL[q] = -1;
                if (scr[s2] < 0) scr[s2] = q; else cL[q] = scr[s2];
                uint32_t c = (uint32_t)cT[q], pm1 = (uint32_t)q - 1u;
                uint32_t addr = (c < pm1 ? c : pm1);
                addr = addr >= 4 ? addr - 4 : 0;
                a_all[q - r0] = addr;
                const int isval = cT[q] < q && cT[q] >= 4;
                if (isval) a_valid[n_valid++] = addr;
                const int isver = isval && rd32(in + cT[q]) == rd32(in + q);
                if (isver) a_ver[n_ver++] = addr;
                tok[q] = isval && ok8 && tg[h] == (uint8_t)htag(in + q);
                if (tok[q]) a_tag[n_tag++] = addr;
                lanes++; valid += isval; ver += isver; tagok += tok[q];
            }
            l_all += lines(a_all, 64);
            l_valid += lines(a_valid, n_valid);
            l_ver += lines(a_ver, n_ver);
            l_tag += lines(a_tag, n_tag);
            steps++;
            while (p < r0 + 64) {   /* the greedy walk (pol 7) */
                int best = 0, bc = -1, usedT = 0;
                if (p >= 1 && p <= mstart) {
                    int cs[2] = {cT[p], cL[p]}, ok[2], l[2] = {0, 0};
                    for (int j = 0; j < 2; j++) {
                        int c = cs[j];
                        ok[j] = !(c < 0 || c >= p || (j == 0 && c < 4)) && rd32(in + c) == rd32(in + p);
                        if (ok[j]) { l[j] = 4; while (p + l[j] < mlimit && in[p + l[j]] == in[c + l[j]]) l[j]++; }
                    }
                    int pick = -1, l12 = l[1] < 12 ? l[1] : 12;
                    if (pol == 8) pick = ok[0] ? 0 : (ok[1] ? 1 : -1);
                    else if (pol == 9) pick = ok[1] ? 1 : (ok[0] ? 0 : -1);
                    else if (pol == 10) {   /* L measured to 8 bytes only */
                        int l8 = l[1] < 8 ? l[1] : 8;
                        if (ok[1] && (!ok[0] || (l[0] < 8 && l8 >= l[0]))) pick = 1;
                        else if (ok[0]) pick = 0;
                    }
                    else if (ok[1] && (!ok[0] || (l[0] < 12 && l12 >= l[0]))) pick = 1;
                    else if (ok[0]) pick = 0;
                    if (pick >= 0) { best = l[pick]; bc = cs[pick]; usedT = pick == 0; }
                }
                ins[nins] = p; insc[nins++] = k;
                if (best >= 4) {
                    members++; memT += usedT;
                    int m = p, c = bc, len = best, bb = 0;
                    while (bb < 4 && m > anchor && c > 0 && in[m - 1] == in[c - 1]) { m--; c--; len++; bb++; }
                    int lit = m - anchor;
                    out += 1 + ext(lit) + lit + 2 + ext(len - 4);
                    p = m + len;
                    anchor = p;
                    ins[nins] = p - 2; insc[nins++] = (p - 2) / 64 > k ? (p - 2) / 64 : k;
                } else p++;
            }
        }
        out += 1 + ext(n - anchor) + n - anchor;
        free(ins); free(insc); free(cT); free(cL); free(tok);
    }
    printf("ratio %.4f (model, table %d)\n", (double)n * nb / out, TS);
    printf("per 64-lane step: distinct 128-B lines of the T gather: all lanes %.2f, lanes with a "
           "valid candidate %.2f, lanes whose candidate verifies 4 bytes %.2f, lanes passing an "
           "8-bit tag %.2f\n", (double)l_all / steps, (double)l_valid / steps, (double)l_ver / steps,
           (double)l_tag / steps);
    printf("lanes: valid %.1f %%, verified %.1f %%, tag-pass %.1f %%; members per step %.2f (T %.2f)\n",
           100.0 * valid / lanes, 100.0 * ver / lanes, 100.0 * tagok / lanes, (double)members / steps,
           (double)memT / steps);
    return 0;
}
