/*
 * ape_lz4_host.c -- host (CPU) implementation of the ape_lz4.h entry points that
 * are NOT on the GPU hot path: chained streaming compression (the ape_socket
 * TX path, ref src/ape_socket.c:811-871), dictionary/prefix decoding (the RX
 * path, :1333-1467), decompress_fast and compress_destSize (SURVEY.md section
 * 8(f) rows 3-4: "these start as CPU restatements").
 *
 * These are inherently sequential per stream (each 8 KiB chunk depends on the
 * previous 64 KiB of history) and are called one small block at a time, so a
 * kernel launch per call would cost more than the work.  The one-shot block
 * codec -- the batchable path -- never comes here: see ape_lz4_api.c.
 *
 * The stream format/behaviour follows the reference exactly so that streams
 * produced by either side interoperate (LZ4 v1.7.1, ref src/ape_lz4.c).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ape_lz4_host.h"

typedef uint8_t byte;

enum { MINMATCH = 4, LASTLIT = 5, MFLIMIT = 12, MINLEN = 13, WINDOW = 65536 };
enum { TBL_U32, TBL_U16 };
enum { DICT_NONE, DICT_PREFIX, DICT_EXT };

static inline uint32_t ld32(const void *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t ld64(const void *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint16_t ld16(const void *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline void copy8(byte *d, const byte *s) { uint64_t t = ld64(s); memcpy(d, &t, 8); }

/* the reference's 64-bit hash of 5 bytes (ref :456-462) */
static inline unsigned hpos(const byte *p, int tbl)
{
    const unsigned bits = tbl == TBL_U16 ? 13 : 12;
    return (unsigned)((ld64(p) * 889523592379ULL) >> (40 - bits)) & ((1u << bits) - 1);
}

static inline unsigned common_len(const byte *a, const byte *b, const byte *end)
{
    const byte *a0 = a;
    for (; a + 8 <= end; a += 8, b += 8) {
        uint64_t d = ld64(a) ^ ld64(b);
        if (d) return (unsigned)(a - a0) + (unsigned)(__builtin_ctzll(d) >> 3);
    }
    if (a + 4 <= end && ld32(a) == ld32(b)) { a += 4; b += 4; }
    if (a + 2 <= end && ld16(a) == ld16(b)) { a += 2; b += 2; }
    if (a < end && *a == *b) a++;
    return (unsigned)(a - a0);
}

static inline byte *put_run(byte *op, size_t v)
{
    for (; v >= 255; v -= 255) *op++ = 255;
    *op++ = (byte)v;
    return op;
}

/* --------------------------------------------------------------------------
 * compressor core (ref LZ4_compress_generic :530-755).  Table entries are
 * offsets from a virtual origin `org` = src - cur; in ext-dict mode offsets
 * below `cur` address the dictionary, whose end is glued to `cur`.
 * ------------------------------------------------------------------------ */
typedef struct {
    hst_stream *st;
    const byte *src, *iend;
    uintptr_t cur;     /* virtual offset of src */
    int tbl, dict, small;
    const byte *dend;  /* ext dictionary end */
} cctx;

static inline uint32_t tget(const cctx *c, unsigned h)
{
    return c->tbl == TBL_U16 ? ((const uint16_t *)c->st->table)[h] : c->st->table[h];
}
static inline void tset(cctx *c, unsigned h, uintptr_t v)
{
    if (c->tbl == TBL_U16) ((uint16_t *)c->st->table)[h] = (uint16_t)v;
    else c->st->table[h] = (uint32_t)v;
}
/* real address of virtual offset v */
static inline const byte *vaddr(const cctx *c, uintptr_t v)
{
    if (c->dict == DICT_EXT && v < c->cur) return c->dend - (c->cur - v);
    return c->src + (v - c->cur);
}

/* always inlined: every caller passes its table/dict/limited mode as constants, so each
 * call site compiles to a specialised loop, as the reference's LZ4_FORCE_INLINE
 * LZ4_compress_generic does (ref :530) -- the generic loop was ~45 % slower */
static inline __attribute__((always_inline))
int compress_core(hst_stream *st, const byte *src, byte *dst, int n, int cap,
                         int limited, int tbl, int dict, int small, unsigned accel)
{
    cctx c;
    const byte *ip = src, *anchor = src;
    const byte *const iend = src + n, *const mfl = iend - MFLIMIT, *const mlim = iend - LASTLIT;
    byte *op = dst, *const oend = dst + cap;
    unsigned fh;
    c.st = st; c.src = src; c.iend = iend; c.tbl = tbl; c.dict = dict; c.small = small;
    c.cur = dict == DICT_NONE ? 0 : st->currentOffset;
    c.dend = st->dictionary ? st->dictionary + st->dictSize : NULL;
    const uintptr_t low_ref = c.cur - st->dictSize;   /* oldest usable (dictSmall) */
    const uintptr_t low_prefix = dict == DICT_PREFIX ? c.cur - st->dictSize : c.cur;

    if ((uint32_t)n > (uint32_t)HST_MAX_INPUT) return 0;
    if (tbl == TBL_U16 && n >= HST_LIMIT64K) return 0;
    if (n < MINLEN) goto tail;

    tset(&c, hpos(ip, tbl), c.cur);
    ip++;
    fh = hpos(ip, tbl);
    for (;;) {
        const byte *ref;
        uintptr_t rv;
        int in_dict = 0;
        byte *tok;
        {   /* search (:591-619) */
            const byte *fwd = ip;
            unsigned step = 1, tries = accel << 6;
            for (;;) {
                unsigned h = fh;
                ip = fwd;
                fwd += step;
                step = tries++ >> 6;
                if (fwd > mfl) goto tail;
                rv = tget(&c, h);
                in_dict = dict == DICT_EXT && rv < c.cur;
                fh = hpos(fwd, tbl);
                tset(&c, h, c.cur + (uintptr_t)(ip - src));
                if (small && rv < low_ref) continue;
                if (tbl != TBL_U16 && rv + 65535 < c.cur + (uintptr_t)(ip - src)) continue;
                ref = vaddr(&c, rv);
                if (ld32(ref) == ld32(ip)) break;
            }
        }
        {   /* extend backwards (:623-627) */
            uintptr_t lowv = in_dict ? c.cur - st->dictSize : low_prefix;
            while (ip > anchor && rv > lowv && ip[-1] == ref[-1]) { ip--; ref--; rv--; }
        }
        {   /* literals (:631-650) */
            size_t lit = (size_t)(ip - anchor);
            tok = op++;
            if (limited && op + lit + 8 + lit / 255 > oend) return 0;
            if (lit >= 15) { *tok = 15 << 4; op = put_run(op, lit - 15); }
            else *tok = (byte)(lit << 4);
            {   /* 8-byte units (the reference's wildCopy, :646): at most 7 bytes past
                   op + lit, which stay below the end of dst -- limited mode checked
                   op + lit + 8 <= oend above; otherwise an offset, the last token and
                   >= 5 last literals still follow within cap -- and reads stay below
                   ip + 8 <= iend - 4 (ip <= mflimit) */
                byte *d = op;
                const byte *q = anchor;
                do { copy8(d, q); d += 8; q += 8; } while (d < op + lit);
            }
            op += lit;
        }
        for (;;) {  /* match (:652-698), possibly repeated (:709-726) */
            unsigned ml;
            uint16_t off = (uint16_t)(c.cur + (uintptr_t)(ip - src) - rv);
            memcpy(op, &off, 2);
            op += 2;
            if (in_dict) {
                const byte *lim = ip + (c.dend - ref);
                if (lim > mlim) lim = mlim;
                ml = common_len(ip + MINMATCH, ref + MINMATCH, lim);
                ip += MINMATCH + ml;
                if (ip == lim) {
                    unsigned more = common_len(ip, src, mlim);
                    ml += more;
                    ip += more;
                }
            } else {
                ml = common_len(ip + MINMATCH, ref + MINMATCH, mlim);
                ip += MINMATCH + ml;
            }
            if (limited && op + 6 + (ml >> 8) > oend) return 0;
            if (ml >= 15) {
                *tok += 15;
                ml -= 15;
                for (; ml >= 510; ml -= 510) { *op++ = 255; *op++ = 255; }
                if (ml >= 255) { ml -= 255; *op++ = 255; }
                *op++ = (byte)ml;
            } else {
                *tok += (byte)ml;
            }
            anchor = ip;
            if (ip > mfl) goto tail;
            tset(&c, hpos(ip - 2, tbl), c.cur + (uintptr_t)(ip - 2 - src));
            {
                unsigned h = hpos(ip, tbl);
                rv = tget(&c, h);
                in_dict = dict == DICT_EXT && rv < c.cur;
                tset(&c, h, c.cur + (uintptr_t)(ip - src));
                if ((small ? rv >= low_ref : 1) && rv + 65535 >= c.cur + (uintptr_t)(ip - src)) {
                    ref = vaddr(&c, rv);
                    if (ld32(ref) == ld32(ip)) {
                        tok = op++;
                        *tok = 0;
                        continue;
                    }
                }
            }
            fh = hpos(++ip, tbl);
            break;
        }
    }
tail: { /* last literals (:732-751) */
        size_t run = (size_t)(iend - anchor);
        if (limited && (size_t)(op - dst) + run + 1 + (run + 240) / 255 > (size_t)(uint32_t)cap)
            return 0;
        if (run >= 15) { *op++ = 15 << 4; op = put_run(op, run - 15); }
        else *op++ = (byte)(run << 4);
        memcpy(op, anchor, run);
        op += run;
    }
    return (int)(op - dst);
}

/* destSize variant (ref :843-1021): fill `target` bytes with as much input as fits */
static int destsize_core(hst_stream *st, const byte *src, byte *dst, int *srcSize, int target,
                         int tbl)
{
    cctx c;
    const byte *ip = src, *anchor = src;
    const byte *const iend = src + *srcSize, *const mfl = iend - MFLIMIT, *const mlim = iend - LASTLIT;
    byte *op = dst, *const oend = dst + target;
    byte *const lit_max = oend - 11, *const match_max = oend - 6, *const seq_max = lit_max - 1;
    unsigned fh;
    c.st = st; c.src = src; c.iend = iend; c.tbl = tbl; c.dict = DICT_NONE; c.small = 0;
    c.cur = 0; c.dend = NULL;

    if (target < 1) return 0;
    if ((uint32_t)*srcSize > (uint32_t)HST_MAX_INPUT) return 0;
    if (tbl == TBL_U16 && *srcSize >= HST_LIMIT64K) return 0;
    if (*srcSize < MINLEN) goto tail;
    *srcSize = 0;
    tset(&c, hpos(ip, tbl), 0);
    ip++;
    fh = hpos(ip, tbl);
    for (;;) {
        const byte *ref;
        byte *tok;
        {
            const byte *fwd = ip;
            unsigned step = 1, tries = 1u << 6;
            for (;;) {
                unsigned h = fh;
                ip = fwd;
                fwd += step;
                step = tries++ >> 6;
                if (fwd > mfl) goto tail;
                ref = src + tget(&c, h);
                fh = hpos(fwd, tbl);
                tset(&c, h, (uintptr_t)(ip - src));
                if (tbl != TBL_U16 && ref + 65535 < ip) continue;
                if (ld32(ref) == ld32(ip)) break;
            }
        }
        while (ip > anchor && ref > src && ip[-1] == ref[-1]) { ip--; ref--; }
        {
            unsigned lit = (unsigned)(ip - anchor);
            tok = op++;
            if (op + (lit + 240) / 255 + lit > lit_max) { op--; goto tail; }
            if (lit >= 15) { *tok = 15 << 4; op = put_run(op, lit - 15); }
            else *tok = (byte)(lit << 4);
            memcpy(op, anchor, lit);
            op += lit;
        }
        for (;;) {
            size_t ml;
            uint16_t off = (uint16_t)(ip - ref);
            memcpy(op, &off, 2);
            op += 2;
            ml = common_len(ip + MINMATCH, ref + MINMATCH, mlim);
            if (op + (ml + 240) / 255 > match_max) ml = 14 + (size_t)(match_max - op) * 255;
            ip += MINMATCH + ml;
            if (ml >= 15) {
                *tok += 15;
                ml -= 15;
                while (ml >= 255) { ml -= 255; *op++ = 255; }
                *op++ = (byte)ml;
            } else {
                *tok += (byte)ml;
            }
            anchor = ip;
            if (ip > mfl || op > seq_max) goto tail;
            tset(&c, hpos(ip - 2, tbl), (uintptr_t)(ip - 2 - src));
            {
                unsigned h = hpos(ip, tbl);
                ref = src + tget(&c, h);
                tset(&c, h, (uintptr_t)(ip - src));
                if (ref + 65535 >= ip && ld32(ref) == ld32(ip)) {
                    tok = op++;
                    *tok = 0;
                    continue;
                }
            }
            fh = hpos(++ip, tbl);
            break;
        }
    }
tail: {
        size_t run = (size_t)(iend - anchor);
        if (op + 1 + (run + 240) / 255 + run > oend) {
            run = (size_t)(oend - op) - 1;
            run -= (run + 240) / 255;
        }
        ip = anchor + run;
        if (run >= 15) { *op++ = 15 << 4; op = put_run(op, run - 15); }
        else *op++ = (byte)(run << 4);
        memcpy(op, anchor, run);
        op += run;
    }
    *srcSize = (int)(ip - src);
    return (int)(op - dst);
}

/* --------------------------------------------------------------------------
 * decoder core (ref APE_LZ4_decompress_generic :1275-1469).
 * low = first byte a match may reference (dest - prefix); with ext dict,
 * offsets reaching below `low` continue into [dstart, dstart + dsize).
 * ------------------------------------------------------------------------ */
/* always inlined per call site, like LZ4_decompress_generic (ref :1275) */
static inline __attribute__((always_inline))
int decode_core(const byte *src, byte *dst, int isize, int osize, int safe, int partial,
                       int target, int ext, const byte *low, const byte *dstart, size_t dsize)
{
    static const int inc32[8] = {4, 1, 2, 1, 4, 4, 4, 4};
    static const int dec64[8] = {0, 0, 0, -1, 0, 1, 2, 3};
    const byte *ip = src;
    const byte *const iend = src + isize;
    byte *op = dst;
    byte *const oend = dst + osize;
    /* signed distances instead of pointer compares past the buffers */
    const intptr_t oend_i = osize;
    intptr_t oexit = target;
    const intptr_t lowlim = (low - dst) - (intptr_t)dsize;
    const byte *const dend = dstart ? dstart + dsize : NULL;
    const int chk_off = safe && dsize < WINDOW;

    if (partial && oexit > oend_i - MFLIMIT) oexit = oend_i - MFLIMIT;
    if (osize == 0) {
        if (safe) return (isize == 1 && *ip == 0) ? 0 : -1;
        return *ip == 0 ? 1 : -1;
    }
    for (;;) {
        const unsigned token = *ip++;
        size_t len = token >> 4;
        intptr_t o = op - dst, cpy;
        const byte *ref;
        if (len == 15) {
            unsigned s;
            /* The reference reads the first length byte unconditionally (ref :1330-1337), one
             * byte past src when the token is the last input byte.  That byte cannot change
             * the outcome: with ip past iend every later check fails and the result is
             * -(consumed + 1) - 1 whatever it holds, so return that without reading it.  Only
             * the first read can be out of range: the loop condition bounds the others. */
            if (safe && ip >= iend) return -(int)(ip - src) - 2;
            do {
                s = *ip++;
                len += s;
            } while ((safe ? (ip - src) < (intptr_t)isize - 15 : 1) && s == 255);
        }
        cpy = o + (intptr_t)len;
        if (safe ? (cpy > (partial ? oexit : oend_i - MFLIMIT) ||
                    (ip - src) + (intptr_t)len > (intptr_t)isize - 8)
                 : cpy > oend_i - 8) {
            if (partial) {
                if (cpy > oend_i) goto fail;
                if (safe && (ip - src) + (intptr_t)len > (intptr_t)isize) goto fail;
            } else {
                if (!safe && cpy != oend_i) goto fail;
                if (safe && ((ip - src) + (intptr_t)len != (intptr_t)isize || cpy > oend_i))
                    goto fail;
            }
            memcpy(op, ip, len);
            ip += len;
            op += len;
            break;
        }
        {   /* 8-byte literal copy; may write up to 7 bytes past cpy (inside dst) */
            byte *d = op;
            const byte *s = ip;
            do { copy8(d, s); d += 8; s += 8; } while (d < dst + cpy);
        }
        ip += len;
        op = dst + cpy;
        o = cpy - (intptr_t)ld16(ip);
        ip += 2;
        if (chk_off && o < lowlim) goto fail;
        len = token & 15;
        if (len == 15) {
            unsigned s;
            do {
                if (safe && ip > iend - LASTLIT) goto fail;
                s = *ip++;
                len += s;
            } while (s == 255);
        }
        len += MINMATCH;
        if (ext && o < low - dst) {  /* match starts in the external dictionary */
            const size_t back = (size_t)((low - dst) - o);
            if (op + len > oend - LASTLIT) goto fail;
            if (len <= back) {
                memmove(op, dend - back, len);
                op += len;
            } else {
                size_t rest = len - back;
                memcpy(op, dend - back, back);
                op += back;
                if (rest > (size_t)(op - low)) {
                    const byte *from = low;
                    byte *e = op + rest;
                    while (op < e) *op++ = *from++;
                } else {
                    memcpy(op, low, rest);
                    op += rest;
                }
            }
            continue;
        }
        ref = dst + o;
        cpy = (op - dst) + (intptr_t)len;
        {
            const intptr_t dist = op - ref;
            if (dist < 8) {
                op[0] = ref[0]; op[1] = ref[1]; op[2] = ref[2]; op[3] = ref[3];
                ref += inc32[dist];
                { uint32_t t = ld32(ref); memcpy(op + 4, &t, 4); }
                op += 8;
                ref -= dec64[dist];
            } else {
                copy8(op, ref);
                op += 8;
                ref += 8;
            }
        }
        if (cpy > oend_i - 12) {
            if (cpy > oend_i - LASTLIT) goto fail;
            if (op < oend - 8) {
                byte *d = op;
                const byte *s = ref;
                do { copy8(d, s); d += 8; s += 8; } while (d < oend - 8);
                ref += (oend - 8) - op;
                op = oend - 8;
            }
            while (op < dst + cpy) *op++ = *ref++;
        } else {
            byte *d = op;
            const byte *s = ref;
            do { copy8(d, s); d += 8; s += 8; } while (d < dst + cpy);
        }
        op = dst + cpy;
    }
    return safe ? (int)(op - dst) : (int)(ip - src);
fail:
    return -(int)(ip - src) - 1;
}

/* ------------------------------ public (host) ----------------------------- */
void hst_reset(hst_stream *s) { memset(s, 0, sizeof *s); }

int hst_compress_extstate(hst_stream *s, const char *src, char *dst, int n, int cap, int accel)
{
    const int bound = (uint32_t)n > (uint32_t)HST_MAX_INPUT ? 0 : n + n / 255 + 16;
    hst_reset(s);
    if (accel < 1) accel = 1;
    if (n < HST_LIMIT64K) {
        if (cap < bound)
            return compress_core(s, (const byte *)src, (byte *)dst, n, cap, 1, TBL_U16,
                                 DICT_NONE, 0, (unsigned)accel);
        return compress_core(s, (const byte *)src, (byte *)dst, n, cap, 0, TBL_U16, DICT_NONE,
                             0, (unsigned)accel);
    }
    return compress_core(s, (const byte *)src, (byte *)dst, n, cap, cap < bound, TBL_U32,
                         DICT_NONE, 0, (unsigned)accel);
}

int hst_compress_force(const char *src, char *dst, int n, int cap, int accel)
{
    hst_stream s;
    hst_reset(&s);
    return compress_core(&s, (const byte *)src, (byte *)dst, n, cap, 1,
                         n < HST_LIMIT64K ? TBL_U16 : TBL_U32, DICT_NONE, 0, (unsigned)accel);
}

int hst_compress_destSize(const char *src, char *dst, int *srcSize, int target)
{
    hst_stream s;
    const int n = *srcSize;
    const int bound = (uint32_t)n > (uint32_t)HST_MAX_INPUT ? 0 : n + n / 255 + 16;
    hst_reset(&s);
    if (target >= bound) return hst_compress_extstate(&s, src, dst, n, target, 1);
    return destsize_core(&s, (const byte *)src, (byte *)dst, srcSize, target,
                         n < HST_LIMIT64K ? TBL_U16 : TBL_U32);
}

int hst_loadDict(hst_stream *d, const char *dict, int size)
{
    const byte *p = (const byte *)dict, *const end = p + size;
    uint32_t base;
    if (d->initCheck || d->currentOffset > (1u << 30)) hst_reset(d);
    if (size < 8) { d->dictionary = NULL; d->dictSize = 0; return 0; }
    if (end - p > WINDOW) p = end - WINDOW;
    d->currentOffset += WINDOW;
    base = d->currentOffset;
    d->dictionary = p;
    d->dictSize = (uint32_t)(end - p);
    d->currentOffset += d->dictSize;
    for (const byte *q = p; q <= end - 8; q += 3) d->table[hpos(q, TBL_U32)] = base + (uint32_t)(q - p);
    return (int)d->dictSize;
}

static void renorm(hst_stream *d, const byte *smallest)
{
    if (d->currentOffset > 0x80000000u || (size_t)d->currentOffset > (size_t)smallest) {
        const uint32_t delta = d->currentOffset - WINDOW;
        const byte *dend = d->dictionary + d->dictSize;
        for (int i = 0; i < HST_TABLE; i++) d->table[i] = d->table[i] < delta ? 0 : d->table[i] - delta;
        d->currentOffset = WINDOW;
        if (d->dictSize > WINDOW) d->dictSize = WINDOW;
        d->dictionary = dend - d->dictSize;
    }
}

int hst_compress_continue(hst_stream *d, const char *source, char *dest, int n, int cap,
                          int accel)
{
    const byte *src = (const byte *)source;
    const byte *dend = d->dictionary + d->dictSize;
    const byte *smallest = src;
    int r, small;
    if (d->initCheck) return 0;
    if (d->dictSize > 0 && smallest > dend) smallest = dend;
    renorm(d, smallest);
    if (accel < 1) accel = 1;
    {
        const byte *send = src + n;
        if (send > d->dictionary && send < dend) {
            d->dictSize = (uint32_t)(dend - send);
            if (d->dictSize > WINDOW) d->dictSize = WINDOW;
            if (d->dictSize < 4) d->dictSize = 0;
            d->dictionary = dend - d->dictSize;
        }
    }
    small = d->dictSize < WINDOW && d->dictSize < d->currentOffset;
    if (dend == src) {
        r = compress_core(d, src, (byte *)dest, n, cap, 1, TBL_U32, DICT_PREFIX, small, (unsigned)accel);
        d->dictSize += (uint32_t)n;
        d->currentOffset += (uint32_t)n;
        return r;
    }
    r = compress_core(d, src, (byte *)dest, n, cap, 1, TBL_U32, DICT_EXT, small, (unsigned)accel);
    d->dictionary = src;
    d->dictSize = (uint32_t)n;
    d->currentOffset += (uint32_t)n;
    return r;
}

int hst_compress_forceExtDict(hst_stream *d, const char *source, char *dest, int n)
{
    const byte *dend = d->dictionary + d->dictSize;
    const byte *smallest = dend < (const byte *)source ? dend : (const byte *)source;
    int r;
    renorm(d, smallest);
    r = compress_core(d, (const byte *)source, (byte *)dest, n, 0, 0, TBL_U32, DICT_EXT, 0, 1);
    d->dictionary = (const byte *)source;
    d->dictSize = (uint32_t)n;
    d->currentOffset += (uint32_t)n;
    return r;
}

int hst_saveDict(hst_stream *d, char *safe, int size)
{
    const byte *prev_end = d->dictionary + d->dictSize;
    if ((uint32_t)size > WINDOW) size = WINDOW;
    if ((uint32_t)size > d->dictSize) size = (int)d->dictSize;
    memmove(safe, prev_end - size, (size_t)size);
    d->dictionary = (const byte *)safe;
    d->dictSize = (uint32_t)size;
    return size;
}

int hst_decompress_fast(const char *s, char *d, int osize)
{
    return decode_core((const byte *)s, (byte *)d, 0, osize, 0, 0, 0, 0,
                       (const byte *)d - WINDOW, NULL, WINDOW);
}

int hst_decompress_safe_prefix64k(const char *s, char *d, int csize, int cap)
{
    return decode_core((const byte *)s, (byte *)d, csize, cap, 1, 0, 0, 0,
                       (const byte *)d - WINDOW, NULL, WINDOW);
}

int hst_decompress_safe_extdict(const char *s, char *d, int csize, int cap, const char *dict,
                                int dsize)
{
    return decode_core((const byte *)s, (byte *)d, csize, cap, 1, 0, 0, 1, (const byte *)d,
                       (const byte *)dict, (size_t)dsize);
}

/* decompress_safe / _safe_partial of one block without a dictionary (ref :1472-1487) */
int hst_decompress_block(const char *s, char *d, int csize, int cap, int partial, int target)
{
    if (partial)
        return decode_core((const byte *)s, (byte *)d, csize, cap, 1, 1, target, 0,
                           (const byte *)d, NULL, 0);
    return decode_core((const byte *)s, (byte *)d, csize, cap, 1, 0, 0, 0, (const byte *)d,
                       NULL, 0);
}

int hst_decompress_usingDict(const char *s, char *d, int csize, int cap, int safe,
                             const char *dict, int dsize)
{
    const int isz = safe ? csize : 0;
    if (dsize == 0)
        return decode_core((const byte *)s, (byte *)d, isz, cap, safe, 0, 0, 0, (const byte *)d,
                           NULL, 0);
    if (dict + dsize == d) {
        if (dsize >= WINDOW - 1)
            return decode_core((const byte *)s, (byte *)d, isz, cap, safe, 0, 0, 0,
                               (const byte *)d - WINDOW, NULL, 0);
        return decode_core((const byte *)s, (byte *)d, isz, cap, safe, 0, 0, 0,
                           (const byte *)d - dsize, NULL, 0);
    }
    return decode_core((const byte *)s, (byte *)d, isz, cap, safe, 0, 0, 1, (const byte *)d,
                       (const byte *)dict, (size_t)dsize);
}

int hst_setStreamDecode(hst_stream_dec *sd, const char *dict, int size)
{
    sd->prefixSize = (size_t)size;
    sd->prefixEnd = (const byte *)dict + size;
    sd->externalDict = NULL;
    sd->extDictSize = 0;
    return 1;
}

int hst_decompress_continue(hst_stream_dec *sd, const char *src, char *dst, int csize, int cap,
                            int safe)
{
    int r;
    const int isz = safe ? csize : 0;
    if (sd->prefixEnd == (const byte *)dst) {
        r = decode_core((const byte *)src, (byte *)dst, isz, cap, safe, 0, 0, 1,
                        sd->prefixEnd - sd->prefixSize, sd->externalDict, sd->extDictSize);
        if (r <= 0) return r;
        sd->prefixSize += safe ? (size_t)r : (size_t)cap;
        sd->prefixEnd += safe ? r : cap;
    } else {
        sd->extDictSize = sd->prefixSize;
        sd->externalDict = safe ? sd->prefixEnd - sd->extDictSize
                                : (const byte *)dst - sd->extDictSize; /* ref :1604 */
        r = decode_core((const byte *)src, (byte *)dst, isz, cap, safe, 0, 0, 1,
                        (const byte *)dst, sd->externalDict, sd->extDictSize);
        if (r <= 0) return r;
        sd->prefixSize = safe ? (size_t)r : (size_t)cap;
        sd->prefixEnd = (const byte *)dst + (safe ? r : cap);
    }
    return r;
}
