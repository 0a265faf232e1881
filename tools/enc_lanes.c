/* enc_lanes.c -- DESIGN TOOL (not product, not oracle): per-chunk lane statistics of the
 * product encoder's candidate policy (tools/enc_model.c model4, pol 7, lag 3): how many of
 * a chunk's 64 lanes verify a candidate and how long the picked candidates are, to size
 * the producer's measurement stages.
 *   gcc -O2 -o /tmp/enc_lanes tools/enc_lanes.c oracle/synth.c && /tmp/enc_lanes 16 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void synth_blocks(uint8_t *out, int n, long long stride, long long first, int nb, int kind);
static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint32_t hsh(const uint8_t *p) {
    uint32_t x = rd32(p), b4 = p[4];
    uint32_t lo = x & 0xFFFFFF, hi = (x >> 24) | (b4 << 8);
    return (lo * 0x9E3779u + hi * 0xC2B2AEu) >> 19;
}

int main(int argc, char **argv)
{
    const int n = 65536, nb = argc > 1 ? atoi(argv[1]) : 16, lag = 3;
    uint8_t *buf = malloc((size_t)n * nb + 16);
    synth_blocks(buf, n, n, 0, nb, 1);
    long hist_ok[65] = {0}, hist_len[8] = {0}, chunks = 0, lanes_ok = 0, members = 0;
    long hist_ge[5][65];   /* picked length >= 8, 12, 16, 20, 24 per chunk */
    memset(hist_ge, 0, sizeof hist_ge);
    const int th[5] = {8, 12, 16, 20, 24};
    for (int b = 0; b < nb; b++) {
        const uint8_t *in = buf + (size_t)b * n;
        int tab[8192];
        for (int i = 0; i < 8192; i++) tab[i] = -1;
        int *ins = malloc(8 * n), *insc = malloc(8 * n), nins = 0, done = 0;
        int cT[64], cL[64], scr[64], len[64];
        int anchor = 0, p = 0;
        const int mstart = n - 12, mlimit = n - 5;
        for (int k = 0; k < n / 64; k++) {
            while (done < nins && insc[done] <= k - lag - 1) {
                int q = ins[done++];
                if (q + 8 <= n) tab[hsh(in + q)] = q;
            }
            for (int i = 0; i < 64; i++) scr[i] = -1;
            int nok = 0, ge[5] = {0};
            for (int l = 0; l < 64; l++) {
                int q = 64 * k + l;
                uint32_t h = q + 8 <= n ? hsh(in + q) : 0;
                cT[l] = tab[h];
                cL[l] = -1;
                if (scr[h & 63] < 0) scr[h & 63] = q; else cL[l] = scr[h & 63];
                int best = 0;
                if (q >= 1 && q <= mstart) {
                    int cs[2] = {cT[l], cL[l]}, ok[2], ll[2] = {0, 0};
                    for (int j = 0; j < 2; j++) {
                        int c = cs[j];
                        ok[j] = !(c < 4 || c >= q) && rd32(in + c) == rd32(in + q);
                        if (ok[j]) { ll[j] = 4; while (q + ll[j] < mlimit && in[q + ll[j]] == in[c + ll[j]]) ll[j]++; }
                    }
                    if (ok[0] || ok[1]) nok++;
                    int l12 = ll[1] < 12 ? ll[1] : 12;
                    if (ok[1] && (!ok[0] || (ll[0] < 12 && l12 >= ll[0]))) best = ll[1];
                    else if (ok[0]) best = ll[0];
                }
                len[l] = best;
                for (int t = 0; t < 5; t++) ge[t] += best >= th[t];
                if (best) hist_len[best >= 64 ? 7 : best / 10]++;
            }
            hist_ok[nok]++;
            for (int t = 0; t < 5; t++) hist_ge[t][ge[t]]++;
            lanes_ok += nok;
            chunks++;
            /* walk the chunk (greedy, catch-up ignored for the statistics) */
            while (p < 64 * k + 64) {
                int l = p - 64 * k;
                ins[nins] = p; insc[nins++] = k;
                if (len[l] >= 4) {
                    members++;
                    p += len[l];
                    anchor = p;
                    ins[nins] = p - 2; insc[nins++] = (p - 2) / 64 > k ? (p - 2) / 64 : k;
                } else p++;
            }
        }
        (void)anchor;
        free(ins); free(insc);
    }
    printf("chunks %ld: verified lanes per chunk avg %.2f, members per chunk %.2f\n", chunks,
           (double)lanes_ok / chunks, (double)members / chunks);
    for (int t = 0; t < 5; t++) {
        long s = 0, over16 = 0, over32 = 0;
        for (int i = 0; i <= 64; i++) { s += (long)i * hist_ge[t][i]; if (i > 16) over16 += hist_ge[t][i]; if (i > 32) over32 += hist_ge[t][i]; }
        printf("picked len >= %2d: avg %.2f lanes per chunk; chunks with > 16: %.2f%%, > 32: %.3f%%\n",
               th[t], (double)s / chunks, 100.0 * over16 / chunks, 100.0 * over32 / chunks);
    }
    long s16 = 0, s32 = 0;
    for (int i = 0; i <= 64; i++) { if (i > 16) s16 += hist_ok[i]; if (i > 32) s32 += hist_ok[i]; }
    printf("verified: chunks with > 16: %.2f%%, > 32: %.3f%%\n", 100.0 * s16 / chunks, 100.0 * s32 / chunks);
    printf("picked length histogram (x10):");
    for (int i = 0; i < 8; i++) printf(" %ld", hist_len[i]);
    printf("\n");
    return 0;
}
