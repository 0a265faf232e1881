/*
 * synth.c -- TEST INFRASTRUCTURE: host versions of the synthetic block
 * generators of SURVEY.md Appendix C.  The device generator in the product
 * library (APE_LZ4_synth_blocks_dev) must produce identical bytes; tests check
 * that, and bench.py uses these for the CPU-baseline sample.
 *
 *   xorshift64: s ^= s<<13; s ^= s>>7; s ^= s<<17   (value returned = new s)
 *   seed(block) = block * 0x9E3779B97F4A7C15 + 1
 *   rand: successive xs() words, little-endian, 8 bytes at a time
 *   comp: LZ77-like mix of 16-letter literals and back-copies (overlap allowed)
 */
#include <stdint.h>
#include <string.h>

static inline uint64_t xs(uint64_t *s)
{
    uint64_t x = *s;
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    *s = x;
    return x;
}

uint64_t synth_seed(uint64_t block) { return block * 0x9E3779B97F4A7C15ULL + 1ULL; }

void synth_rand(uint8_t *out, int n, uint64_t block)
{
    uint64_t s = synth_seed(block);
    int i = 0;
    while (i < n) {
        uint64_t w = xs(&s);
        for (int k = 0; k < 8 && i < n; k++, i++) out[i] = (uint8_t)(w >> (8 * k));
    }
}

void synth_comp(uint8_t *out, int n, uint64_t block)
{
    uint64_t s = synth_seed(block);
    int i = 0;
    while (i < n) {
        uint64_t r = xs(&s);
        if (i >= 64 && (r & 3) != 0) {
            int len = 4 + (int)((r >> 32) % 60);
            int win = i < 65535 ? i : 65535;
            int off = 1 + (int)((r >> 8) % (uint64_t)win);
            for (int k = 0; k < len && i < n; k++, i++) out[i] = out[i - off];
        } else {
            int len = 1 + (int)((r >> 8) % 16);
            for (int k = 0; k < len && i < n; k++, i++) out[i] = (uint8_t)('a' + (xs(&s) & 15));
        }
    }
}

/* kind: 0 = rand, 1 = comp.  Fills nblocks blocks of `n` bytes at `stride`. */
void synth_blocks(uint8_t *out, int n, long long stride, long long first_block, int nblocks,
                  int kind)
{
    for (int b = 0; b < nblocks; b++) {
        uint8_t *p = out + (long long)b * stride;
        if (kind == 0) synth_rand(p, n, (uint64_t)(first_block + b));
        else synth_comp(p, n, (uint64_t)(first_block + b));
    }
}
