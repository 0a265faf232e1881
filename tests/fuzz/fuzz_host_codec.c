/*
 * fuzz_host_codec.c -- CPU sanitizer / differential fuzz harness of the product's host codec
 * (TEST INFRASTRUCTURE; SURVEY.md App. D item 4, section 5 "Race detection / sanitizers").
 *
 * The product side is libapenetwork_amd/csrc/ape_lz4_api.c + ape_lz4_host.c compiled into
 * this executable with -fsanitize=address,undefined: the exact code every one-shot and stream
 * call of ape_lz4.h runs by default, i.e. what ape_socket.c:832-857 (TX) and :1386-1421 (RX)
 * would run on network input.  The checker is the reference src/ape_lz4.c itself, compiled
 * from its own source by oracle/Makefile (oracle/_ref/libape_lz4_ref.so, not instrumented),
 * loaded with dlopen(RTLD_LOCAL) and called through dlsym, so its symbols never bind to the
 * product's.  Every case compares the return value and the produced bytes; every input is
 * copied into a heap buffer of exactly its size and every output buffer is exactly `cap`
 * bytes, so any read past src or write past dst[0:cap) in the product is an ASan report.
 *
 * Only the reference's own srcSize == 0 quirk is kept (it reads src[0]: ref :1330, SURVEY
 * App. B): such inputs get a 1-byte allocation.  Compression capacities are >= 0: with a
 * negative maxOutputSize the reference's last-literals check compares against
 * (U32)maxOutputSize (ref :736-739) and writes a short input's literals anyway, and the
 * product keeps that return value; there is no buffer to stay inside of.  Decoders do get
 * negative capacities (neither side writes then).
 *
 * Two front ends share run_case():
 *   - a seeded mutation driver (main, default): valid blocks and streams made by the reference
 *     encoder from generated data, then mutated, at random caps/targets/accelerations;
 *     `fuzz_host_codec [iterations] [seed] [seconds]`.
 *   - libFuzzer (-DAPE_LIBFUZZER, clang -fsanitize=fuzzer,address,undefined): the first bytes
 *     of the input choose the entry point and its integer arguments.
 *
 * Entry points compared (ape_lz4.h): decompress_safe, decompress_safe_partial,
 * decompress_safe_usingDict (prefix-contiguous and separate dictionaries, empty dict),
 * decompress_safe_continue + setStreamDecode over a 64 KiB ring (the socket RX path),
 * decompress_safe_withPrefix64k, decompress_safe_forceExtDict, compress_default,
 * compress_limitedOutput, compress_fast (acceleration), compress_fast_continue + saveDict
 * (the socket TX path, random caps), compress_destSize, and decompress_fast on valid blocks.
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/ape_lz4.h"

typedef int (*fn_dec)(const char *, char *, int, int);
typedef int (*fn_decp)(const char *, char *, int, int, int);
typedef int (*fn_decd)(const char *, char *, int, int, const char *, int);
typedef int (*fn_comp)(const char *, char *, int, int);
typedef int (*fn_compf)(const char *, char *, int, int, int);
typedef int (*fn_dsz)(const char *, char *, int *, int);
typedef void *(*fn_new)(void);
typedef int (*fn_free)(void *);
typedef int (*fn_cfc)(void *, const char *, char *, int, int, int);
typedef int (*fn_save)(void *, char *, int);
typedef int (*fn_setsd)(void *, const char *, int);
typedef int (*fn_dsc)(void *, const char *, char *, int, int);
typedef int (*fn_fast)(const char *, char *, int);

static struct {
    fn_dec decompress_safe, withPrefix64k;
    fn_decp partial;
    fn_decd usingDict, forceExtDict;
    fn_comp compress_default, limitedOutput;
    fn_compf compress_fast;
    fn_dsz destSize;
    fn_new createStream, createStreamDecode;
    fn_free freeStream, freeStreamDecode;
    fn_cfc fast_continue;
    fn_save saveDict;
    fn_setsd setStreamDecode;
    fn_dsc safe_continue;
    fn_fast decompress_fast;
} R;

static unsigned long long g_cases, g_fail;

static void *must(void *h, const char *name)
{
    void *p = dlsym(h, name);
    if (!p) { fprintf(stderr, "reference lacks %s\n", name); exit(2); }
    return p;
}

static void load_reference(const char *path)
{
    void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "dlopen %s: %s\n", path, dlerror()); exit(2); }
    R.decompress_safe = (fn_dec)must(h, "APE_LZ4_decompress_safe");
    R.withPrefix64k = (fn_dec)must(h, "APE_LZ4_decompress_safe_withPrefix64k");
    R.partial = (fn_decp)must(h, "APE_LZ4_decompress_safe_partial");
    R.usingDict = (fn_decd)must(h, "APE_LZ4_decompress_safe_usingDict");
    R.forceExtDict = (fn_decd)must(h, "APE_LZ4_decompress_safe_forceExtDict");
    R.compress_default = (fn_comp)must(h, "APE_LZ4_compress_default");
    R.limitedOutput = (fn_comp)must(h, "APE_LZ4_compress_limitedOutput");
    R.compress_fast = (fn_compf)must(h, "APE_LZ4_compress_fast");
    R.destSize = (fn_dsz)must(h, "APE_LZ4_compress_destSize");
    R.createStream = (fn_new)must(h, "APE_LZ4_createStream");
    R.createStreamDecode = (fn_new)must(h, "APE_LZ4_createStreamDecode");
    R.freeStream = (fn_free)must(h, "APE_LZ4_freeStream");
    R.freeStreamDecode = (fn_free)must(h, "APE_LZ4_freeStreamDecode");
    R.fast_continue = (fn_cfc)must(h, "APE_LZ4_compress_fast_continue");
    R.saveDict = (fn_save)must(h, "APE_LZ4_saveDict");
    R.setStreamDecode = (fn_setsd)must(h, "APE_LZ4_setStreamDecode");
    R.safe_continue = (fn_dsc)must(h, "APE_LZ4_decompress_safe_continue");
    R.decompress_fast = (fn_fast)must(h, "APE_LZ4_decompress_fast");
    /* the product is linked into this executable; the reference must not resolve to it */
    if ((void *)R.decompress_safe == (void *)&APE_LZ4_decompress_safe) {
        fprintf(stderr, "reference symbols bound to the product\n");
        exit(2);
    }
}

/* ------------------------------------------------------------------------------------- */
static uint64_t rs;
static uint64_t rnd(void)
{
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return rs;
}
static int rint_(int lo, int hi) { return lo + (int)(rnd() % (uint64_t)(hi - lo + 1)); }

static char *exact(const void *p, int n)
{
    char *b = (char *)malloc(n > 0 ? (size_t)n : 1);
    if (n > 0) memcpy(b, p, (size_t)n);
    else b[0] = (char)rnd();   /* srcSize 0: both sides read this byte (the quirk) */
    return b;
}

static void report(const char *what, int a, int b, int x, int y)
{
    g_fail++;
    if (g_fail <= 20)
        fprintf(stderr, "MISMATCH %s: product %d reference %d (args %d %d)\n", what, a, b, x, y);
}

#define CHECK(what, a, b, pa, pb, x, y)                                                     \
    do {                                                                                    \
        g_cases++;                                                                          \
        if ((a) != (b) || ((a) > 0 && memcmp((pa), (pb), (size_t)(a)) != 0))               \
            report(what, (a), (b), (x), (y));                                               \
    } while (0)

/* outputs get identical prefills: an offset-0 match copies prior dst contents (App. B) */
static void prefill(char *a, char *b, int n, unsigned seed)
{
    for (int i = 0; i < n; i++) a[i] = b[i] = (char)(seed * 131u + (unsigned)i * 7u);
}

/* ---- decoders on arbitrary bytes ---- */
static void case_decode(const uint8_t *s, int n, int cap, int target, int dsize, int mode)
{
    char *src = exact(s, n);
    int capb = cap > 0 ? cap : 0;
    char *pa = (char *)malloc((size_t)capb), *pb = (char *)malloc((size_t)capb);
    int a, b;
    prefill(pa, pb, capb, (unsigned)n);
    switch (mode) {
    case 0:
        a = APE_LZ4_decompress_safe(src, pa, n, cap);
        b = R.decompress_safe(src, pb, n, cap);
        CHECK("decompress_safe", a, b, pa, pb, n, cap);
        break;
    case 1:
        a = APE_LZ4_decompress_safe_partial(src, pa, n, target, cap);
        b = R.partial(src, pb, n, target, cap);
        CHECK("decompress_safe_partial", a, b, pa, pb, n, target);
        break;
    default: {
        /* dictionary: separate buffer, or contiguous in front of dst (prefix), or empty */
        int ds = dsize;
        char *da = (char *)malloc((size_t)ds + (size_t)capb);
        char *db = (char *)malloc((size_t)ds + (size_t)capb);
        for (int i = 0; i < ds; i++) da[i] = db[i] = (char)('a' + (rnd() & 15));
        prefill(da + ds, db + ds, capb, (unsigned)n);
        if (mode == 2) {        /* separate: dict in its own exact buffer */
            char *xa = exact(da, ds), *xb = exact(db, ds);
            a = APE_LZ4_decompress_safe_usingDict(src, pa, n, cap, xa, ds);
            b = R.usingDict(src, pb, n, cap, xb, ds);
            CHECK("usingDict(separate)", a, b, pa, pb, n, ds);
            if (ds > 0) {
                a = APE_LZ4_decompress_safe_forceExtDict(src, pa, n, cap, xa, ds);
                b = R.forceExtDict(src, pb, n, cap, xb, ds);
                CHECK("forceExtDict", a, b, pa, pb, n, ds);
            }
            free(xa);
            free(xb);
        } else {                /* prefix: dict immediately before dst */
            a = APE_LZ4_decompress_safe_usingDict(src, da + ds, n, cap, da, ds);
            b = R.usingDict(src, db + ds, n, cap, db, ds);
            CHECK("usingDict(prefix)", a, b, da + ds, db + ds, n, ds);
            if (ds >= 65536) {
                a = APE_LZ4_decompress_safe_withPrefix64k(src, da + ds, n, cap);
                b = R.withPrefix64k(src, db + ds, n, cap);
                CHECK("withPrefix64k", a, b, da + ds, db + ds, n, cap);
            }
        }
        free(da);
        free(db);
    }
    }
    free(src);
    free(pa);
    free(pb);
}

/* ---- socket RX: decompress_safe_continue over a 64 KiB ring (ape_socket.c:1386-1421) ---- */
#define RING (64 * 1024)
#define CHUNK 8192
static void case_stream_rx(const uint8_t *s, int n, const int *lens, int nblk)
{
    char *ra = (char *)malloc(RING), *rb = (char *)malloc(RING);
    void *sa = APE_LZ4_createStreamDecode(), *sb = R.createStreamDecode();
    int pos = 0, off = 0;
    memset(ra, 0, RING);
    memset(rb, 0, RING);
    for (int k = 0; k < nblk && off <= n; k++) {
        int len = lens[k] < n - off ? lens[k] : n - off;
        char *src = exact(s + off, len);
        int a, b;
        if (pos + CHUNK > RING) pos = 0;
        a = APE_LZ4_decompress_safe_continue(sa, src, ra + pos, len, CHUNK);
        b = R.safe_continue(sb, src, rb + pos, len, CHUNK);
        CHECK("decompress_safe_continue", a, b, ra + pos, rb + pos, len, k);
        free(src);
        off += len;
        if (a <= 0 || a != b) break;
        pos += a;
    }
    APE_LZ4_freeStreamDecode(sa);
    R.freeStreamDecode(sb);
    free(ra);
    free(rb);
}

/* ---- encoders ---- */
static void case_compress(const uint8_t *s, int n, int cap, int accel, int mode)
{
    char *src = exact(s, n);
    int capb = cap > 0 ? cap : 0;
    char *pa = (char *)malloc((size_t)capb), *pb = (char *)malloc((size_t)capb);
    int a, b;
    if (mode == 0) {
        a = APE_LZ4_compress_default(src, pa, n, cap);
        b = R.compress_default(src, pb, n, cap);
        CHECK("compress_default", a, b, pa, pb, n, cap);
    } else if (mode == 1) {
        a = APE_LZ4_compress_limitedOutput(src, pa, n, cap);
        b = R.limitedOutput(src, pb, n, cap);
        CHECK("compress_limitedOutput", a, b, pa, pb, n, cap);
    } else if (mode == 2) {
        a = APE_LZ4_compress_fast(src, pa, n, cap, accel);
        b = R.compress_fast(src, pb, n, cap, accel);
        CHECK("compress_fast", a, b, pa, pb, n, accel);
    } else {
        int na = n, nb = n;
        a = APE_LZ4_compress_destSize(src, pa, &na, cap);
        b = R.destSize(src, pb, &nb, cap);
        CHECK("compress_destSize", a, b, pa, pb, n, cap);
        if (na != nb) report("compress_destSize srcSize", na, nb, n, cap);
    }
    if (mode <= 1 && a > 0 && a == b) { /* the block decodes back with decompress_fast too */
        char *blk = exact(pa, a), *oa = (char *)malloc((size_t)n);
        int r = APE_LZ4_decompress_fast(blk, oa, n);
        g_cases++;
        if (r != a || memcmp(oa, src, (size_t)n) != 0) report("decompress_fast", r, a, n, 0);
        free(blk);
        free(oa);
    }
    free(src);
    free(pa);
    free(pb);
}

/* ---- socket TX: compress_fast_continue on 8 KiB chunks + saveDict (ape_socket.c:811-871) ---- */
static void case_stream_tx(const uint8_t *s, int n, int capslack, int accel)
{
    void *sa = APE_LZ4_createStream(), *sb = R.createStream();
    char *da = (char *)malloc(RING), *db = (char *)malloc(RING);
    for (int off = 0; off < n; off += CHUNK) {
        int len = n - off < CHUNK ? n - off : CHUNK;
        int cap = APE_LZ4_COMPRESSBOUND(len) - capslack;
        if (cap < 0) cap = 0;
        char *src = exact(s + off, len);
        char *pa = (char *)malloc((size_t)cap), *pb = (char *)malloc((size_t)cap);
        int a = APE_LZ4_compress_fast_continue(sa, src, pa, len, cap, accel);
        int b = R.fast_continue(sb, src, pb, len, cap, accel);
        int x, y;
        CHECK("compress_fast_continue", a, b, pa, pb, len, cap);
        x = APE_LZ4_saveDict(sa, da, RING);
        y = R.saveDict(sb, db, RING);
        g_cases++;
        if (x != y || memcmp(da, db, (size_t)x) != 0) report("saveDict", x, y, off, 0);
        free(src);
        free(pa);
        free(pb);
        if (a != b) break;
    }
    APE_LZ4_freeStream(sa);
    R.freeStream(sb);
    free(da);
    free(db);
}

/* ------------------------------------------------------------------------------------- */
/* One case from an opcode and integer arguments (shared by both front ends). */
static void run_case(unsigned op, unsigned a0, unsigned a1, const uint8_t *p, int n)
{
    switch (op % 9) {
    case 0: case_decode(p, n, (int)(a0 % 70000) - 16, 0, 0, 0); break;
    case 1: case_decode(p, n, (int)(a0 % 70000) - 16, (int)(a1 % 70000) - 16, 0, 1); break;
    case 2: case_decode(p, n, (int)(a0 % 70000), 0, (int)(a1 % 70000), 2); break;
    case 3: case_decode(p, n, (int)(a0 % 70000), 0, (int)(a1 % 70000), 3); break;
    case 4: case_compress(p, n, (int)(a0 % 70000), 1, (int)(a1 & 1)); break;
    case 5: case_compress(p, n, (int)(a0 % 70000), (int)(a1 % 10) - 1, 2); break;
    case 6: case_compress(p, n, (int)(a0 % 70000), 1, 3); break;
    case 7: case_stream_tx(p, n, (int)(a0 % 24), (int)(a1 % 4)); break;
    default: {
        int lens[16];
        for (int k = 0; k < 16; k++) lens[k] = 1 + (int)((a0 >> (k & 31)) ^ (a1 * (k + 1))) % 9000;
        case_stream_rx(p, n, lens, 16);
    }
    }
}

#ifdef APE_LIBFUZZER
static int g_loaded;
int LLVMFuzzerTestOneInput(const uint8_t *d, size_t sz)
{
    unsigned a0, a1;
    if (!g_loaded) {
        const char *p = getenv("APE_REF_LIB");
        load_reference(p ? p : "oracle/_ref/libape_lz4_ref.so");
        g_loaded = 1;
    }
    if (sz < 9 || sz > 200000) return 0;
    memcpy(&a0, d + 1, 4);
    memcpy(&a1, d + 5, 4);
    rs = (uint64_t)a0 * 0x9E3779B97F4A7C15ULL + a1 + 1;
    run_case(d[0], a0, a1, d + 9, (int)sz - 9);
    if (g_fail) abort();
    return 0;
}
#else
/* ---- generators and mutators for the seeded driver ---- */
static int gen(uint8_t *o, int n)
{
    int kind = rint_(0, 5);
    for (int i = 0; i < n;) {
        uint64_t r = rnd();
        if (kind == 0) o[i++] = (uint8_t)r;                                 /* random */
        else if (kind == 1) o[i++] = (uint8_t)('a' + (r & 15));             /* 16 letters */
        else if (kind == 2) o[i++] = (uint8_t)(r % 3 == 0 ? r >> 8 : 0);    /* sparse */
        else if (kind == 3) { o[i] = (uint8_t)(i % (1 + (int)(r % 9))); i++; } /* periodic */
        else {                                                             /* App. C-like */
            if (i >= 64 && (r & 3)) {
                int len = 4 + (int)((r >> 32) % 60), off = 1 + (int)((r >> 8) % (uint64_t)(i < 65535 ? i : 65535));
                for (int k = 0; k < len && i < n; k++, i++) o[i] = o[i - off];
            } else {
                int len = 1 + (int)((r >> 8) % 16);
                for (int k = 0; k < len && i < n; k++) o[i++] = (uint8_t)('a' + (rnd() & 15));
            }
        }
    }
    return n;
}

static int pick_size(void)
{
    int c = rint_(0, 9);
    if (c == 0) return rint_(0, 20);
    if (c < 6) return rint_(0, 600);
    if (c < 9) return rint_(0, 9000);
    return rint_(60000, 66000);
}

static void mutate(uint8_t *b, int *n, int maxn)
{
    int k = rint_(0, 4);
    for (int m = 0; m <= k; m++) {
        int c = rint_(0, 7);
        if (*n == 0) c = 6;
        switch (c) {
        case 0: b[rint_(0, *n - 1)] ^= (uint8_t)(1u << rint_(0, 7)); break;
        case 1: b[rint_(0, *n - 1)] = (uint8_t)rnd(); break;
        case 2: b[rint_(0, *n - 1)] = (uint8_t)(rint_(0, 1) ? 0xFF : 0xF0 | rint_(0, 15)); break;
        case 3: *n = rint_(0, *n); break;                                   /* truncate */
        case 4: { int i = rint_(0, *n - 1); b[i] = 0; if (i + 1 < *n) b[i + 1] = 0; break; } /* offset 0 */
        case 5: { int i = rint_(0, *n - 1); while (i < *n && rint_(0, 7)) b[i++] = 0xFF; break; }
        default:
            if (*n < maxn) b[(*n)++] = (uint8_t)(rint_(0, 1) ? 0xFF : rnd());
        }
    }
}

int main(int argc, char **argv)
{
    long iters = argc > 1 ? atol(argv[1]) : 20000;
    uint64_t seed = argc > 2 ? strtoull(argv[2], NULL, 0) : 1;
    double secs = argc > 3 ? atof(argv[3]) : 0;
    const char *ref = getenv("APE_REF_LIB");
    const int MAXN = 140000;
    uint8_t *raw = (uint8_t *)malloc(MAXN), *blk = (uint8_t *)malloc(MAXN);
    time_t t0 = time(NULL);
    long it;
    load_reference(ref ? ref : "oracle/_ref/libape_lz4_ref.so");
    rs = seed * 0x9E3779B97F4A7C15ULL + 1;

    /* fixed regression cases first (a final token with literal length 15) */
    {
        static const uint8_t t1[] = {0xFF}, t2[] = {0xF0}, t3[] = {0x00};
        case_decode(t1, 1, 64, 0, 0, 0);
        case_decode(t1, 1, 1, 0, 0, 0);
        case_decode(t1, 1, 64, 10, 0, 1);
        case_decode(t2, 1, 64, 0, 0, 0);
        case_decode(t2, 1, 64, 0, 100, 2);
        case_decode(t2, 1, 64, 0, 100, 3);
        case_decode(t3, 1, 0, 0, 0, 0);
        case_decode(t3, 0, 8, 0, 0, 0);     /* srcSize 0: reads src[0] (quirk, kept) */
    }
    for (it = 0; it < iters; it++) {
        int n = pick_size(), op = rint_(0, 8), bn;
        if (secs > 0 && (it & 255) == 0 && difftime(time(NULL), t0) > secs) break;
        gen(raw, n);
        if (op >= 4 && op <= 7) {            /* encoders take the raw data */
            unsigned a0 = (unsigned)rnd(), a1 = (unsigned)rnd();
            if (rint_(0, 3)) a0 = (unsigned)(APE_LZ4_COMPRESSBOUND(n) + 16 - rint_(0, n / 2 + 20));
            run_case((unsigned)op, a0, a1, raw, n);
            continue;
        }
        /* decoders: a reference-compressed block (or chained stream), then mutated */
        if (op == 8) {
            void *st = R.createStream();
            int lens[16], nb = 0;
            char *dict = (char *)malloc(RING);
            bn = 0;
            for (int off = 0; off < n && nb < 16; off += CHUNK) {
                int len = n - off < CHUNK ? n - off : CHUNK;
                int c = R.fast_continue(st, (const char *)raw + off, (char *)blk + bn, len,
                                        APE_LZ4_COMPRESSBOUND(len), 1);
                R.saveDict(st, dict, RING);
                lens[nb++] = c;
                bn += c;
            }
            R.freeStream(st);
            free(dict);
            if (rint_(0, 2)) mutate(blk, &bn, MAXN);
            case_stream_rx(blk, bn, lens, nb);
            continue;
        }
        bn = R.compress_default((const char *)raw, (char *)blk, n, APE_LZ4_COMPRESSBOUND(n));
        if (rint_(0, 3)) mutate(blk, &bn, MAXN);
        {
            int exactcap = n, c = rint_(0, 5);
            int cap = c == 0 ? exactcap : c == 1 ? exactcap - 1 : c == 2 ? exactcap + rint_(1, 64)
                    : c == 3 ? rint_(-4, 70000) : rint_(0, exactcap + 16);
            int target = rint_(-4, exactcap + 16);
            int ds = rint_(0, 3) == 0 ? 0 : rint_(0, 3) == 0 ? 65536 + rint_(0, 64) : rint_(1, 70000);
            if (op < 2) case_decode(blk, bn, cap, target, 0, op);
            else case_decode(blk, bn, cap, 0, ds, op == 2 ? 2 : 3);
        }
    }
    printf("fuzz_host_codec: %ld iterations, %llu comparisons, %llu mismatches, %.0f s\n", it,
           g_cases, g_fail, difftime(time(NULL), t0));
    free(raw);
    free(blk);
    return g_fail ? 1 : 0;
}
#endif
