/*
 * lz4_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A bit-exact CPU restatement of libapenetwork's in-tree LZ4 v1.7.1 block codec
 * (/root/reference/src/ape_lz4.c).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library.  The product library
 * (libapenetwork_amd/libape_lz4_amd.so) never links or calls it.
 *
 * Parity pin: tests/test_oracle_golden.py checks every function here against
 * golden vectors produced by the reference itself (oracle/_ref, built from the
 * reference sources by oracle/Makefile; generator tests/golden/gen_golden.py).
 *
 * Style: everything is restated with explicit integer offsets instead of the
 * reference's "virtual" pointers (base = src - currentOffset may point before
 * any allocation), so the arithmetic is defined C while producing the same
 * bytes and the same return codes.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MINMATCH 4            /* ape_lz4.c:237 */
#define ORC_COPYLENGTH 8          /* :239 */
#define ORC_LASTLITERALS 5        /* :240 */
#define ORC_MFLIMIT 12            /* :241 */
#define ORC_MINLENGTH 13          /* :242 */
#define ORC_MAX_DISTANCE 65535    /* :248-249 */
#define ORC_ML_MASK 15u           /* :251-252 */
#define ORC_RUN_MASK 15u          /* :253-254 */
#define ORC_HASHLOG 12            /* :393 (LZ4_MEMORY_USAGE 14 - 2) */
#define ORC_LIMIT64K (65536 + 11) /* :398 */
#define ORC_SKIP_TRIGGER 6        /* :399 */
#define ORC_MAX_INPUT 0x7E000000  /* ape_lz4.h:123 */
#define ORC_STREAM_BYTES 16416    /* ape_lz4.h:240-241 */
#define ORC_GB (1u << 30)

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

enum { T_U32 = 1, T_U16 = 2 };           /* byU32 / byU16, :417 */
enum { D_NONE = 0, D_PREFIX, D_EXTDICT }; /* :419 */

/* The stream state, same field order as APE_LZ4_stream_t_internal (:407-414). */
typedef struct {
    u32 table[1 << ORC_HASHLOG];
    u32 currentOffset;
    u32 initCheck;
    const u8 *dictionary;
    u8 *bufferStart;
    u32 dictSize;
} orc_stream;

typedef struct {
    const u8 *externalDict; /* :1499-1504 */
    size_t extDictSize;
    const u8 *prefixEnd;
    size_t prefixSize;
} orc_stream_dec;

static u32 rd32(const u8 *p) { u32 v; memcpy(&v, p, 4); return v; }
static u64 rd64(const u8 *p) { u64 v; memcpy(&v, p, 8); return v; }
static u16 rd16(const u8 *p) { u16 v; memcpy(&v, p, 2); return v; }
/* 8-byte load-then-store copy (LZ4_copy8, :214-217): defined even when the
 * two ranges overlap (offset 0 streams), like the reference's codegen. */
static void cp8(u8 *d, const u8 *s) { u64 t; memcpy(&t, s, 8); memcpy(d, &t, 8); }

int orc_versionNumber(void) { return 10701; } /* ape_lz4.h:52-58 */
int orc_compressBound(int n) /* ape_lz4.h:124-127 */
{
    return ((unsigned)n > (unsigned)ORC_MAX_INPUT) ? 0 : n + n / 255 + 16;
}
int orc_sizeofState(void) { return ORC_STREAM_BYTES; }

/* 5-byte multiplicative hash of the 64-bit build (:456-462, 470-473). */
static u32 orc_hash(const u8 *p, int ttype)
{
    const u32 hlog = (ttype == T_U16) ? ORC_HASHLOG + 1 : ORC_HASHLOG;
    return (u32)((rd64(p) * 889523592379ULL) >> (40 - hlog)) & ((1u << hlog) - 1);
}

/* Common-prefix length of [a, limit) against b (LZ4_count, :359-386). */
static unsigned orc_count(const u8 *a, const u8 *b, const u8 *limit)
{
    const u8 *s = a;
    while (a < limit - 7) {
        u64 x = rd64(a) ^ rd64(b);
        if (x) return (unsigned)(a - s) + (unsigned)(__builtin_ctzll(x) >> 3);
        a += 8; b += 8;
    }
    if (a < limit - 3 && rd32(a) == rd32(b)) { a += 4; b += 4; }
    if (a < limit - 1 && rd16(a) == rd16(b)) { a += 2; b += 2; }
    if (a < limit && *a == *b) a++;
    return (unsigned)(a - s);
}

/* Table access.  Positions are stored relative to a virtual base
 * (src - currentOffset); we keep "virtual indices" v = position - base, so the
 * byte a virtual index points to is src[v - cur] (or the dictionary for
 * v < cur in ext-dict mode).                                     (:475-528) */
static void tput(orc_stream *c, u32 h, u32 v, int ttype)
{
    if (ttype == T_U16) ((u16 *)c->table)[h] = (u16)v;
    else c->table[h] = v;
}
static u32 tget(orc_stream *c, u32 h, int ttype)
{
    return ttype == T_U16 ? ((u16 *)c->table)[h] : c->table[h];
}

/*
 * LZ4_compress_generic (:530-755).  Positions inside `src` are plain offsets
 * i in [0, n).  The virtual index of offset i is vi = cur + i where cur is the
 * stream's currentOffset (0 for noDict).  Candidates with vi < cur live before
 * `src`: in the prefix (withPrefix64k: same address space, byte = src[vi-cur])
 * or in the external dictionary (usingExtDict: byte = dictEnd[vi - cur]).
 */
static int orc_compress_generic(orc_stream *c, const u8 *src, u8 *dst, int n, int cap,
                                int limited, int ttype, int dmode, int dictSmall,
                                u32 accel)
{
    const u32 cur = (dmode == D_NONE) ? 0 : c->currentOffset;
    const u8 *dictEnd = c->dictionary ? c->dictionary + c->dictSize : NULL;
    /* lowRefLimit = src - dictSize (:542), as a virtual index */
    const int64_t lowRef = (int64_t)cur - (int64_t)c->dictSize;
    const int64_t mflimit = (int64_t)n - ORC_MFLIMIT;
    const int64_t mlimit = (int64_t)n - ORC_LASTLITERALS;
    int64_t ip = 0, anchor = 0; /* offsets in src */
    int64_t op = 0;             /* offset in dst */
    int64_t lowLimit;           /* virtual index below which catch-up stops */
    int inDict = 0;             /* refDelta != 0 (:555) */
    u32 fwdH;

    if ((u32)n > (u32)ORC_MAX_INPUT) return 0; /* :558 */
    lowLimit = (dmode == D_PREFIX) ? (int64_t)cur - (int64_t)c->dictSize : (int64_t)cur;
    if (ttype == T_U16 && n >= ORC_LIMIT64K) return 0; /* :575 */
    if (n < ORC_MINLENGTH) goto last_literals;        /* :577 */

    tput(c, orc_hash(src, ttype), cur + 0, ttype); /* :582 */
    ip = 1;
    fwdH = orc_hash(src + 1, ttype);

    for (;;) {
        int64_t mv; /* match virtual index */
        int64_t token;
        const u8 *mptr; /* real address of the match */
        {
            int64_t fwd = ip;
            unsigned step = 1, nb = accel << ORC_SKIP_TRIGGER;
            for (;;) { /* :596-619 */
                u32 h = fwdH;
                ip = fwd;
                fwd += step;
                step = nb++ >> ORC_SKIP_TRIGGER;
                if (fwd > mflimit) goto last_literals;
                mv = tget(c, h, ttype);
                if (dmode == D_EXTDICT) inDict = mv < (int64_t)cur;
                fwdH = orc_hash(src + fwd, ttype);
                tput(c, h, (u32)(cur + ip), ttype);
                if (dictSmall && mv < lowRef) continue;
                if (ttype != T_U16 && mv + ORC_MAX_DISTANCE < (int64_t)cur + ip) continue;
                mptr = inDict ? dictEnd + (mv - (int64_t)cur) : src + (mv - (int64_t)cur);
                if (rd32(mptr) == rd32(src + ip)) break;
            }
        }
        /* catch up (:623-627); lowLimit is dictionary start for dict matches */
        {
            int64_t lowV = inDict ? (int64_t)cur - (int64_t)c->dictSize : lowLimit;
            while (ip > anchor && mv > lowV && src[ip - 1] == mptr[-1]) {
                ip--; mv--; mptr--;
            }
        }
        {
            unsigned lit = (unsigned)(ip - anchor); /* :631-650 */
            token = op++;
            if (limited && op + lit + (2 + 1 + ORC_LASTLITERALS) + lit / 255 > cap) return 0;
            if (lit >= ORC_RUN_MASK) {
                int len = (int)lit - (int)ORC_RUN_MASK;
                dst[token] = (u8)(ORC_RUN_MASK << 4);
                for (; len >= 255; len -= 255) dst[op++] = 255;
                dst[op++] = (u8)len;
            } else {
                dst[token] = (u8)(lit << 4);
            }
            memcpy(dst + op, src + anchor, lit);
            op += lit;
        }
    next_match:
        {
            u16 off = (u16)((int64_t)cur + ip - mv); /* :654 */
            unsigned ml;
            dst[op] = (u8)off; dst[op + 1] = (u8)(off >> 8);
            op += 2;
            if (dmode == D_EXTDICT && inDict) { /* :661-673 */
                int64_t dictRemain = (int64_t)(dictEnd - mptr);
                int64_t limit = ip + dictRemain;
                if (limit > mlimit) limit = mlimit;
                ml = orc_count(src + ip + ORC_MINMATCH, mptr + ORC_MINMATCH, src + limit);
                ip += ORC_MINMATCH + ml;
                if (ip == limit) {
                    unsigned more = orc_count(src + ip, src, src + mlimit);
                    ml += more;
                    ip += more;
                }
            } else {
                ml = orc_count(src + ip + ORC_MINMATCH, mptr + ORC_MINMATCH, src + mlimit);
                ip += ORC_MINMATCH + ml;
            }
            if (limited && op + (1 + ORC_LASTLITERALS) + (ml >> 8) > cap) return 0; /* :680 */
            if (ml >= ORC_ML_MASK) { /* :684-697 */
                dst[token] += (u8)ORC_ML_MASK;
                ml -= ORC_ML_MASK;
                for (; ml >= 510; ml -= 510) { dst[op++] = 255; dst[op++] = 255; }
                if (ml >= 255) { ml -= 255; dst[op++] = 255; }
                dst[op++] = (u8)ml;
            } else {
                dst[token] += (u8)ml;
            }
        }
        anchor = ip;
        if (ip > mflimit) break; /* :703 */
        tput(c, orc_hash(src + ip - 2, ttype), (u32)(cur + ip - 2), ttype); /* :706 */
        {
            u32 h = orc_hash(src + ip, ttype); /* :709-726 */
            mv = tget(c, h, ttype);
            if (dmode == D_EXTDICT) inDict = mv < (int64_t)cur;
            tput(c, h, (u32)(cur + ip), ttype);
            mptr = inDict ? dictEnd + (mv - (int64_t)cur) : src + (mv - (int64_t)cur);
            if ((dictSmall ? mv >= lowRef : 1) && mv + ORC_MAX_DISTANCE >= (int64_t)cur + ip &&
                rd32(mptr) == rd32(src + ip)) {
                token = op++;
                dst[token] = 0;
                goto next_match;
            }
        }
        fwdH = orc_hash(src + (++ip), ttype); /* :729 */
    }

last_literals: /* :732-751 */
    {
        size_t run = (size_t)(n - anchor);
        if (limited && (size_t)op + run + 1 + ((run + 255 - ORC_RUN_MASK) / 255) > (u32)cap)
            return 0;
        if (run >= ORC_RUN_MASK) {
            size_t acc = run - ORC_RUN_MASK;
            dst[op++] = (u8)(ORC_RUN_MASK << 4);
            for (; acc >= 255; acc -= 255) dst[op++] = 255;
            dst[op++] = (u8)acc;
        } else {
            dst[op++] = (u8)(run << 4);
        }
        memcpy(dst + op, src + anchor, run);
        op += run;
    }
    return (int)op;
}

void orc_resetStream(void *s) { memset(s, 0, ORC_STREAM_BYTES); } /* :1088-1091 */

int orc_compress_fast_extState(void *state, const char *src, char *dst, int n, int cap,
                               int accel) /* :758-786 */
{
    orc_stream *c = (orc_stream *)state;
    int ttype = (n < ORC_LIMIT64K) ? T_U16 : T_U32;
    orc_resetStream(state);
    if (accel < 1) accel = 1;
    return orc_compress_generic(c, (const u8 *)src, (u8 *)dst, n,
                                cap >= orc_compressBound(n) ? 0 : cap,
                                cap >= orc_compressBound(n) ? 0 : 1, ttype, D_NONE, 0,
                                (u32)accel);
}

int orc_compress_fast(const char *src, char *dst, int n, int cap, int accel) /* :789 */
{
    u64 st[ORC_STREAM_BYTES / 8];
    return orc_compress_fast_extState(st, src, dst, n, cap, accel);
}

int orc_compress_default(const char *src, char *dst, int n, int cap) /* :811 */
{
    return orc_compress_fast(src, dst, n, cap, 1);
}

int orc_compress_fast_force(const char *src, char *dst, int n, int cap, int accel) /* :821 */
{
    u64 st[ORC_STREAM_BYTES / 8];
    orc_resetStream(st);
    return orc_compress_generic((orc_stream *)st, (const u8 *)src, (u8 *)dst, n, cap, 1,
                                n < ORC_LIMIT64K ? T_U16 : T_U32, D_NONE, 0, (u32)accel);
}

/* compress_destSize (:843-1067) */
static int orc_destsize_generic(orc_stream *c, const u8 *src, u8 *dst, int *srcSizePtr,
                                int target, int ttype)
{
    const int64_t n = *srcSizePtr;
    const int64_t mflimit = n - ORC_MFLIMIT, mlimit = n - ORC_LASTLITERALS;
    const int64_t oend = target;
    const int64_t oMaxLit = target - 2 - 8 - 1;
    const int64_t oMaxMatch = target - (ORC_LASTLITERALS + 1);
    const int64_t oMaxSeq = oMaxLit - 1;
    int64_t ip = 0, anchor = 0, op = 0;
    u32 fwdH;

    if (target < 1) return 0;
    if ((u32)*srcSizePtr > (u32)ORC_MAX_INPUT) return 0;
    if (ttype == T_U16 && *srcSizePtr >= ORC_LIMIT64K) return 0;
    if (*srcSizePtr < ORC_MINLENGTH) goto last_literals;

    *srcSizePtr = 0;
    tput(c, orc_hash(src, ttype), 0, ttype);
    ip = 1;
    fwdH = orc_hash(src + 1, ttype);
    for (;;) {
        int64_t m, token;
        {
            int64_t fwd = ip;
            unsigned step = 1, nb = 1u << ORC_SKIP_TRIGGER;
            for (;;) {
                u32 h = fwdH;
                ip = fwd;
                fwd += step;
                step = nb++ >> ORC_SKIP_TRIGGER;
                if (fwd > mflimit) goto last_literals;
                m = tget(c, h, ttype);
                fwdH = orc_hash(src + fwd, ttype);
                tput(c, h, (u32)ip, ttype);
                if (ttype != T_U16 && m + ORC_MAX_DISTANCE < ip) continue;
                if (rd32(src + m) == rd32(src + ip)) break;
            }
        }
        while (ip > anchor && m > 0 && src[ip - 1] == src[m - 1]) { ip--; m--; }
        {
            unsigned lit = (unsigned)(ip - anchor);
            token = op++;
            if (op + ((lit + 240) / 255) + lit > oMaxLit) { op--; goto last_literals; }
            if (lit >= ORC_RUN_MASK) {
                unsigned len = lit - ORC_RUN_MASK;
                dst[token] = (u8)(ORC_RUN_MASK << 4);
                for (; len >= 255; len -= 255) dst[op++] = 255;
                dst[op++] = (u8)len;
            } else {
                dst[token] = (u8)(lit << 4);
            }
            memcpy(dst + op, src + anchor, lit);
            op += lit;
        }
    next_match:
        {
            u16 off = (u16)(ip - m);
            size_t ml;
            dst[op] = (u8)off; dst[op + 1] = (u8)(off >> 8);
            op += 2;
            ml = orc_count(src + ip + ORC_MINMATCH, src + m + ORC_MINMATCH, src + mlimit);
            if (op + (int64_t)((ml + 240) / 255) > oMaxMatch)
                ml = (15 - 1) + (size_t)(oMaxMatch - op) * 255;
            ip += ORC_MINMATCH + (int64_t)ml;
            if (ml >= ORC_ML_MASK) {
                dst[token] += (u8)ORC_ML_MASK;
                ml -= ORC_ML_MASK;
                while (ml >= 255) { ml -= 255; dst[op++] = 255; }
                dst[op++] = (u8)ml;
            } else {
                dst[token] += (u8)ml;
            }
        }
        anchor = ip;
        if (ip > mflimit) break;
        if (op > oMaxSeq) break;
        tput(c, orc_hash(src + ip - 2, ttype), (u32)(ip - 2), ttype);
        {
            u32 h = orc_hash(src + ip, ttype);
            m = tget(c, h, ttype);
            tput(c, h, (u32)ip, ttype);
            if (m + ORC_MAX_DISTANCE >= ip && rd32(src + m) == rd32(src + ip)) {
                token = op++;
                dst[token] = 0;
                goto next_match;
            }
        }
        fwdH = orc_hash(src + (++ip), ttype);
    }
last_literals:
    {
        size_t run = (size_t)(n - anchor);
        if (op + 1 + (int64_t)((run + 240) / 255) + (int64_t)run > oend) {
            run = (size_t)(oend - op) - 1;
            run -= (run + 240) / 255;
        }
        ip = anchor + (int64_t)run;
        if (run >= ORC_RUN_MASK) {
            size_t acc = run - ORC_RUN_MASK;
            dst[op++] = (u8)(ORC_RUN_MASK << 4);
            for (; acc >= 255; acc -= 255) dst[op++] = 255;
            dst[op++] = (u8)acc;
        } else {
            dst[op++] = (u8)(run << 4);
        }
        memcpy(dst + op, src + anchor, run);
        op += (int64_t)run;
    }
    *srcSizePtr = (int)ip;
    return (int)op;
}

int orc_compress_destSize(const char *src, char *dst, int *srcSizePtr, int target) /* :1048 */
{
    u64 st[ORC_STREAM_BYTES / 8];
    orc_resetStream(st);
    if (target >= orc_compressBound(*srcSizePtr))
        return orc_compress_fast_extState(st, src, dst, *srcSizePtr, target, 1);
    return orc_destsize_generic((orc_stream *)st, (const u8 *)src, (u8 *)dst, srcSizePtr,
                                target, *srcSizePtr < ORC_LIMIT64K ? T_U16 : T_U32);
}

/* ---- streaming compression (:1074-1263) ---- */
void *orc_createStream(void)
{
    void *s = calloc(8, ORC_STREAM_BYTES / 8);
    orc_resetStream(s);
    return s;
}
int orc_freeStream(void *s) { free(s); return 0; }

int orc_loadDict(void *s, const char *dict, int dictSize) /* :1101-1133 */
{
    orc_stream *d = (orc_stream *)s;
    const u8 *p = (const u8 *)dict;
    const u8 *end = p + dictSize;
    u32 cur;
    if (d->initCheck || d->currentOffset > ORC_GB) orc_resetStream(s);
    if (dictSize < 8) { d->dictionary = NULL; d->dictSize = 0; return 0; }
    if (end - p > 65536) p = end - 65536;
    d->currentOffset += 65536;
    cur = d->currentOffset; /* base = p - cur: virtual index of p is cur */
    d->dictionary = p;
    d->dictSize = (u32)(end - p);
    d->currentOffset += d->dictSize;
    {
        const u8 *q = p;
        while (q <= end - 8) {
            d->table[orc_hash(q, T_U32)] = cur + (u32)(q - p);
            q += 3;
        }
    }
    return (int)d->dictSize;
}

/* LZ4_renormDictT (:1136-1157); `smallest` compared as an address. */
static void orc_renorm(orc_stream *d, const u8 *smallest)
{
    if (d->currentOffset > 0x80000000u || (size_t)d->currentOffset > (size_t)smallest) {
        u32 delta = d->currentOffset - 65536;
        const u8 *dictEnd = d->dictionary + d->dictSize;
        int i;
        for (i = 0; i < (1 << ORC_HASHLOG); i++)
            d->table[i] = (d->table[i] < delta) ? 0 : d->table[i] - delta;
        d->currentOffset = 65536;
        if (d->dictSize > 65536) d->dictSize = 65536;
        d->dictionary = dictEnd - d->dictSize;
    }
}

int orc_compress_fast_continue(void *s, const char *source, char *dest, int n, int cap,
                               int accel) /* :1160-1220 */
{
    orc_stream *d = (orc_stream *)s;
    const u8 *src = (const u8 *)source;
    const u8 *dictEnd = d->dictionary + d->dictSize;
    const u8 *smallest = src;
    int r;
    if (d->initCheck) return 0;
    if (d->dictSize > 0 && smallest > dictEnd) smallest = dictEnd;
    orc_renorm(d, smallest);
    if (accel < 1) accel = 1;
    {
        const u8 *srcEnd = src + n;
        if (srcEnd > d->dictionary && srcEnd < dictEnd) {
            d->dictSize = (u32)(dictEnd - srcEnd);
            if (d->dictSize > 65536) d->dictSize = 65536;
            if (d->dictSize < 4) d->dictSize = 0;
            d->dictionary = dictEnd - d->dictSize;
        }
    }
    if (dictEnd == src) {
        int small = d->dictSize < 65536 && d->dictSize < d->currentOffset;
        r = orc_compress_generic(d, src, (u8 *)dest, n, cap, 1, T_U32, D_PREFIX, small,
                                 (u32)accel);
        d->dictSize += (u32)n;
        d->currentOffset += (u32)n;
        return r;
    }
    {
        int small = d->dictSize < 65536 && d->dictSize < d->currentOffset;
        r = orc_compress_generic(d, src, (u8 *)dest, n, cap, 1, T_U32, D_EXTDICT, small,
                                 (u32)accel);
        d->dictionary = src;
        d->dictSize = (u32)n;
        d->currentOffset += (u32)n;
        return r;
    }
}

int orc_compress_forceExtDict(void *s, const char *source, char *dest, int n) /* :1224 */
{
    orc_stream *d = (orc_stream *)s;
    const u8 *dictEnd = d->dictionary + d->dictSize;
    const u8 *smallest = dictEnd;
    int r;
    if (smallest > (const u8 *)source) smallest = (const u8 *)source;
    orc_renorm(d, smallest);
    r = orc_compress_generic(d, (const u8 *)source, (u8 *)dest, n, 0, 0, T_U32, D_EXTDICT,
                             0, 1);
    d->dictionary = (const u8 *)source;
    d->dictSize = (u32)n;
    d->currentOffset += (u32)n;
    return r;
}

int orc_saveDict(void *s, char *safe, int dictSize) /* :1248-1263 */
{
    orc_stream *d = (orc_stream *)s;
    const u8 *prevEnd = d->dictionary + d->dictSize;
    if ((u32)dictSize > 65536) dictSize = 65536;
    if ((u32)dictSize > d->dictSize) dictSize = (int)d->dictSize;
    memmove(safe, prevEnd - dictSize, (size_t)dictSize);
    d->dictionary = (const u8 *)safe;
    d->dictSize = (u32)dictSize;
    return dictSize;
}

/*
 * APE_LZ4_decompress_generic (:1275-1469), restated with signed offsets.
 * safe = endOnInputSize; partial = partialDecoding; dmode/lowPrefix/dict as in
 * the reference.  `prefixLen` = dest - lowPrefix (0 for noDict, 64 KiB for the
 * withPrefix64k forms, dictSize for usingDict-as-prefix).
 */
static int orc_decompress_generic(const u8 *src, u8 *dst, int inputSize, int outputSize,
                                  int safe, int partial, int target, int dmode,
                                  int64_t prefixLen, const u8 *dictStart, size_t dictSize)
{
    int64_t ip = 0;
    const int64_t iend = inputSize;
    int64_t op = 0;
    const int64_t oend = outputSize;
    int64_t oexit = target;
    /* lowLimit = lowPrefix - dictSize, relative to dest */
    const int64_t lowLimit = -prefixLen - (int64_t)dictSize;
    const u8 *dictEnd = dictStart ? dictStart + dictSize : NULL;
    static const int dec32[8] = {4, 1, 2, 1, 4, 4, 4, 4};
    static const int dec64[8] = {0, 0, 0, -1, 0, 1, 2, 3};
    const int checkOffset = safe && dictSize < 65536;

    if (partial && oexit > oend - ORC_MFLIMIT) oexit = oend - ORC_MFLIMIT;
    if (safe && outputSize == 0) return (inputSize == 1 && src[0] == 0) ? 0 : -1;
    if (!safe && outputSize == 0) return src[0] == 0 ? 1 : -1;

    for (;;) {
        unsigned token;
        int64_t length, cpy, m;
        token = src[ip++];
        length = token >> 4;
        if (length == ORC_RUN_MASK) { /* :1331-1342 */
            unsigned s;
            do {
                s = src[ip++];
                length += s;
            } while ((safe ? ip < iend - (int64_t)ORC_RUN_MASK : 1) && s == 255);
        }
        cpy = op + length; /* :1345-1370 */
        if ((safe && ((cpy > (partial ? oexit : oend - ORC_MFLIMIT)) ||
                      (ip + length > iend - (2 + 1 + ORC_LASTLITERALS)))) ||
            (!safe && cpy > oend - ORC_COPYLENGTH)) {
            if (partial) {
                if (cpy > oend) goto err;
                if (safe && ip + length > iend) goto err;
            } else {
                if (!safe && cpy != oend) goto err;
                if (safe && (ip + length != iend || cpy > oend)) goto err;
            }
            memcpy(dst + op, src + ip, (size_t)length);
            ip += length;
            op += length;
            break;
        }
        /* wildCopy: copies in 8-byte units, may run up to 7 bytes past cpy */
        {
            int64_t k = 0;
            do { cp8(dst + op + k, src + ip + k); k += 8; } while (op + k < cpy);
        }
        ip += length;
        op = cpy;
        m = cpy - rd16(src + ip); /* :1373-1376 */
        ip += 2;
        if (checkOffset && m < lowLimit) goto err;
        length = token & ORC_ML_MASK; /* :1379-1391 */
        if (length == ORC_ML_MASK) {
            unsigned s;
            do {
                if (safe && ip > iend - ORC_LASTLITERALS) goto err;
                s = src[ip++];
                length += s;
            } while (s == 255);
        }
        length += ORC_MINMATCH;

        if (dmode == D_EXTDICT && m < -prefixLen) { /* :1394-1424 */
            if (op + length > oend - ORC_LASTLITERALS) goto err;
            if (length <= -prefixLen - m) {
                memmove(dst + op, dictEnd - (-prefixLen - m), (size_t)length);
                op += length;
            } else {
                int64_t cs = -prefixLen - m;
                memcpy(dst + op, dictEnd - cs, (size_t)cs);
                op += cs;
                cs = length - cs;
                if (cs > op + prefixLen) {
                    int64_t e = op + cs, from = -prefixLen;
                    while (op < e) { dst[op] = dst[from]; op++; from++; }
                } else {
                    memcpy(dst + op, dst - prefixLen, (size_t)cs);
                    op += cs;
                }
            }
            continue;
        }

        cpy = op + length; /* :1427-1457 */
        if (op - m < 8) {
            int64_t d = op - m;
            dst[op] = dst[m]; dst[op + 1] = dst[m + 1];
            dst[op + 2] = dst[m + 2]; dst[op + 3] = dst[m + 3];
            m += dec32[d];
            { u32 t4; memcpy(&t4, dst + m, 4); memcpy(dst + op + 4, &t4, 4); }
            op += 8;
            m -= dec64[d];
        } else {
            cp8(dst + op, dst + m);
            op += 8;
            m += 8;
        }
        if (cpy > oend - 12) {
            if (cpy > oend - ORC_LASTLITERALS) goto err;
            if (op < oend - 8) {
                int64_t k = 0;
                do { cp8(dst + op + k, dst + m + k); k += 8; } while (op + k < oend - 8);
                m += (oend - 8) - op;
                op = oend - 8;
            }
            while (op < cpy) dst[op++] = dst[m++];
        } else {
            int64_t k = 0;
            do { cp8(dst + op + k, dst + m + k); k += 8; } while (op + k < cpy);
        }
        op = cpy;
    }
    return safe ? (int)op : (int)ip;
err:
    return (int)(-ip) - 1;
}

int orc_decompress_safe(const char *s, char *d, int csize, int cap) /* :1472 */
{
    return orc_decompress_generic((const u8 *)s, (u8 *)d, csize, cap, 1, 0, 0, D_NONE, 0,
                                  NULL, 0);
}
int orc_decompress_safe_partial(const char *s, char *d, int csize, int target, int cap)
{ /* :1480 */
    return orc_decompress_generic((const u8 *)s, (u8 *)d, csize, cap, 1, 1, target, D_NONE,
                                  0, NULL, 0);
}
int orc_decompress_fast(const char *s, char *d, int osize) /* :1489 */
{
    return orc_decompress_generic((const u8 *)s, (u8 *)d, 0, osize, 0, 0, 0, D_PREFIX,
                                  65536, NULL, 65536);
}

/* ---- streaming decompression (:1499-1672) ---- */
void *orc_createStreamDecode(void) { return calloc(1, sizeof(orc_stream_dec)); }
int orc_freeStreamDecode(void *s) { free(s); return 0; }
int orc_setStreamDecode(void *s, const char *dict, int dictSize)
{
    orc_stream_dec *d = (orc_stream_dec *)s;
    d->prefixSize = (size_t)dictSize;
    d->prefixEnd = (const u8 *)dict + dictSize;
    d->externalDict = NULL;
    d->extDictSize = 0;
    return 1;
}

static int orc_dec_cont(orc_stream_dec *d, const char *src, char *dst, int csize, int cap,
                        int safe)
{
    int r;
    if (d->prefixEnd == (const u8 *)dst) {
        r = orc_decompress_generic((const u8 *)src, (u8 *)dst, safe ? csize : 0, cap, safe, 0,
                                   0, D_EXTDICT, (int64_t)d->prefixSize, d->externalDict,
                                   d->extDictSize);
        if (r <= 0) return r;
        if (safe) { d->prefixSize += (size_t)r; d->prefixEnd += r; }
        else { d->prefixSize += (size_t)cap; d->prefixEnd += cap; }
    } else {
        d->extDictSize = d->prefixSize;
        d->externalDict = safe ? d->prefixEnd - d->extDictSize
                               : (const u8 *)dst - d->extDictSize;
        r = orc_decompress_generic((const u8 *)src, (u8 *)dst, safe ? csize : 0, cap, safe, 0,
                                   0, D_EXTDICT, 0, d->externalDict, d->extDictSize);
        if (r <= 0) return r;
        if (safe) { d->prefixSize = (size_t)r; d->prefixEnd = (const u8 *)dst + r; }
        else { d->prefixSize = (size_t)cap; d->prefixEnd = (const u8 *)dst + cap; }
    }
    return r;
}
int orc_decompress_safe_continue(void *s, const char *src, char *dst, int csize, int cap)
{
    return orc_dec_cont((orc_stream_dec *)s, src, dst, csize, cap, 1);
}
int orc_decompress_fast_continue(void *s, const char *src, char *dst, int osize)
{
    return orc_dec_cont((orc_stream_dec *)s, src, dst, 0, osize, 0);
}

static int orc_using_dict(const char *src, char *dst, int csize, int cap, int safe,
                          const char *dictStart, int dictSize) /* :1625-1646 */
{
    if (dictSize == 0)
        return orc_decompress_generic((const u8 *)src, (u8 *)dst, csize, cap, safe, 0, 0,
                                      D_NONE, 0, NULL, 0);
    if (dictStart + dictSize == dst) {
        if (dictSize >= 65535)
            return orc_decompress_generic((const u8 *)src, (u8 *)dst, csize, cap, safe, 0, 0,
                                          D_PREFIX, 65536, NULL, 0);
        return orc_decompress_generic((const u8 *)src, (u8 *)dst, csize, cap, safe, 0, 0,
                                      D_NONE, dictSize, NULL, 0);
    }
    return orc_decompress_generic((const u8 *)src, (u8 *)dst, csize, cap, safe, 0, 0,
                                  D_EXTDICT, 0, (const u8 *)dictStart, (size_t)dictSize);
}
int orc_decompress_safe_usingDict(const char *s, char *d, int csize, int cap,
                                  const char *dict, int dictSize)
{
    return orc_using_dict(s, d, csize, cap, 1, dict, dictSize);
}
int orc_decompress_fast_usingDict(const char *s, char *d, int osize, const char *dict,
                                  int dictSize)
{
    return orc_using_dict(s, d, 0, osize, 0, dict, dictSize);
}
int orc_decompress_safe_forceExtDict(const char *s, char *d, int csize, int cap,
                                     const char *dict, int dictSize) /* :1665 */
{
    return orc_decompress_generic((const u8 *)s, (u8 *)d, csize, cap, 1, 0, 0, D_EXTDICT, 0,
                                  (const u8 *)dict, (size_t)dictSize);
}
int orc_decompress_safe_withPrefix64k(const char *s, char *d, int csize, int cap) /* :1771 */
{
    return orc_decompress_generic((const u8 *)s, (u8 *)d, csize, cap, 1, 0, 0, D_PREFIX,
                                  65536, NULL, 65536);
}
int orc_decompress_fast_withPrefix64k(const char *s, char *d, int osize) /* :1779 */
{
    return orc_decompress_generic((const u8 *)s, (u8 *)d, 0, osize, 0, 0, 0, D_PREFIX, 65536,
                                  NULL, 65536);
}
