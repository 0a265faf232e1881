/*
 * cpu_bench.c -- TEST INFRASTRUCTURE: the CPU baseline of bench.py.
 *
 * Times a codec's compress_default + decompress_safe over a bounded sample of
 * independent blocks with a static block partition over `nthreads` pthreads
 * (one block = one task, as BASELINE.md section 4 prescribes).  The codec is
 * loaded with dlopen: either the reference itself (oracle/_ref/libape_lz4_ref.so,
 * symbol prefix "APE_LZ4_", kind "reference") or the oracle restatement
 * (oracle/liblz4_oracle.so, prefix "orc_", kind "port").
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef int (*comp_fn)(const char *, char *, int, int);
typedef int (*dec_fn)(const char *, char *, int, int);

void synth_blocks(uint8_t *out, int n, long long stride, long long first_block, int nblocks,
                  int kind);

typedef struct {
    comp_fn comp;
    dec_fn dec;
    const uint8_t *in;
    uint8_t *cmp, *out;
    int *csz;
    int n, cap, b0, b1, phase, bad;
} task_t;

static void *worker(void *arg)
{
    task_t *t = (task_t *)arg;
    for (int b = t->b0; b < t->b1; b++) {
        const char *src = (const char *)t->in + (long long)b * t->n;
        char *c = (char *)t->cmp + (long long)b * t->cap;
        if (t->phase == 0) {
            t->csz[b] = t->comp(src, c, t->n, t->cap);
        } else {
            char *o = (char *)t->out + (long long)b * t->n;
            int r = t->dec(c, o, t->csz[b], t->n);
            if (r != t->n) t->bad++;
        }
    }
    return NULL;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static double run_phase(task_t *tasks, int nthreads, int phase)
{
    pthread_t th[256];
    double t0 = now_s();
    for (int i = 0; i < nthreads; i++) {
        tasks[i].phase = phase;
        pthread_create(&th[i], NULL, worker, &tasks[i]);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    return now_s() - t0;
}

/*
 * Returns 0 on success.  out[0] = compress seconds, out[1] = decompress seconds,
 * out[2] = total compressed bytes, out[3] = round-trip failures,
 * out[4] = uncompressed bytes.  `reps` timed repetitions (after one warm-up),
 * times are summed over reps.
 */
int cpu_bench_run(const char *lib, const char *prefix, int nthreads, int nblocks, int n,
                  int kind, int reps, double *out)
{
    char name[128];
    void *h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "cpu_bench: %s\n", dlerror()); return -1; }
    snprintf(name, sizeof name, "%scompress_default", prefix);
    comp_fn comp = (comp_fn)dlsym(h, name);
    snprintf(name, sizeof name, "%sdecompress_safe", prefix);
    dec_fn dec = (dec_fn)dlsym(h, name);
    if (!comp || !dec || nthreads < 1 || nthreads > 256) return -2;
    int cap = n + n / 255 + 16;
    uint8_t *in = malloc((size_t)nblocks * n);
    uint8_t *cmp = malloc((size_t)nblocks * cap);
    uint8_t *o = malloc((size_t)nblocks * n);
    int *csz = calloc((size_t)nblocks, sizeof(int));
    if (!in || !cmp || !o || !csz) return -3;
    synth_blocks(in, n, n, 0, nblocks, kind);
    memset(cmp, 0, (size_t)nblocks * cap); /* pre-fault */
    memset(o, 0, (size_t)nblocks * n);
    task_t tasks[256];
    for (int i = 0; i < nthreads; i++) {
        tasks[i] = (task_t){comp, dec, in, cmp, o, csz, n, cap,
                            (int)((long long)nblocks * i / nthreads),
                            (int)((long long)nblocks * (i + 1) / nthreads), 0, 0};
    }
    run_phase(tasks, nthreads, 0); /* warm-up */
    run_phase(tasks, nthreads, 1);
    double tc = 0, td = 0;
    for (int r = 0; r < reps; r++) {
        tc += run_phase(tasks, nthreads, 0);
        td += run_phase(tasks, nthreads, 1);
    }
    long long tot = 0;
    int bad = 0;
    for (int b = 0; b < nblocks; b++) tot += csz[b];
    for (int i = 0; i < nthreads; i++) bad += tasks[i].bad;
    if (memcmp(in, o, (size_t)nblocks * n) != 0) bad++;
    out[0] = tc;
    out[1] = td;
    out[2] = (double)tot;
    out[3] = bad;
    out[4] = (double)nblocks * n;
    free(in); free(cmp); free(o); free(csz);
    dlclose(h);
    return 0;
}

/*
 * Chained-stream baseline (the reference socket's codec use):
 * each thread runs one stream over its contiguous range of blocks, cut into
 * `chunk`-byte pieces -- TX compress_fast_continue per chunk on one stream state
 * (history = the previous input, in place, as ape_socket.c:832 sees it), RX
 * decompress_safe_continue per chunk into one contiguous output (prefix mode,
 * ape_lz4.c:1555-1584).  Same out[] layout as cpu_bench_run (bytes = payload).
 */
typedef void *(*mk_fn)(void);
typedef int (*free_fn)(void *);
typedef int (*ccont_fn)(void *, const char *, char *, int, int, int);
typedef int (*dcont_fn)(void *, const char *, char *, int, int);

typedef struct {
    mk_fn mk, mkd;
    free_fn fr, frd;
    ccont_fn cc;
    dcont_fn dc;
    const uint8_t *in;
    uint8_t *cmp, *out;
    int *csz;
    long long c0, c1;   /* chunk range */
    int chunk, cap, phase, bad;
} stask_t;

static void *sworker(void *arg)
{
    stask_t *t = (stask_t *)arg;
    if (t->phase == 0) {
        void *s = t->mk();
        for (long long c = t->c0; c < t->c1; c++)
            t->csz[c] = t->cc(s, (const char *)t->in + c * t->chunk, (char *)t->cmp + c * t->cap,
                              t->chunk, t->cap, 1);
        t->fr(s);
    } else {
        void *d = t->mkd();
        for (long long c = t->c0; c < t->c1; c++) {
            int r = t->dc(d, (const char *)t->cmp + c * t->cap, (char *)t->out + c * t->chunk,
                          t->csz[c], t->chunk);
            if (r != t->chunk) t->bad++;
        }
        t->frd(d);
    }
    return NULL;
}

static double run_sphase(stask_t *tasks, int nthreads, int phase)
{
    pthread_t th[256];
    double t0 = now_s();
    for (int i = 0; i < nthreads; i++) {
        tasks[i].phase = phase;
        pthread_create(&th[i], NULL, sworker, &tasks[i]);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    return now_s() - t0;
}

int cpu_stream_run(const char *lib, const char *prefix, int nthreads, int nblocks, int n,
                   int chunk, int kind, int reps, double *out)
{
    char name[128];
    void *h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "cpu_bench: %s\n", dlerror()); return -1; }
#define SYM(var, type, nm) snprintf(name, sizeof name, "%s" nm, prefix); type var = (type)dlsym(h, name)
    SYM(mk, mk_fn, "createStream");
    SYM(fr, free_fn, "freeStream");
    SYM(mkd, mk_fn, "createStreamDecode");
    SYM(frd, free_fn, "freeStreamDecode");
    SYM(cc, ccont_fn, "compress_fast_continue");
    SYM(dc, dcont_fn, "decompress_safe_continue");
#undef SYM
    if (!mk || !fr || !mkd || !frd || !cc || !dc || nthreads < 1 || nthreads > 256 ||
        chunk <= 0 || n % chunk)
        return -2;
    const int cap = chunk + chunk / 255 + 16;
    const long long nch = (long long)nblocks * (n / chunk);
    uint8_t *in = malloc((size_t)nblocks * n);
    uint8_t *cmp = malloc((size_t)nch * cap);
    uint8_t *o = malloc((size_t)nblocks * n);
    int *csz = calloc((size_t)nch, sizeof(int));
    if (!in || !cmp || !o || !csz) return -3;
    synth_blocks(in, n, n, 0, nblocks, kind);
    memset(cmp, 0, (size_t)nch * cap);
    memset(o, 0, (size_t)nblocks * n);
    stask_t tasks[256];
    for (int i = 0; i < nthreads; i++) {
        /* whole blocks per thread, so every stream starts at a block boundary */
        const long long b0 = (long long)nblocks * i / nthreads, b1 = (long long)nblocks * (i + 1) / nthreads;
        tasks[i] = (stask_t){mk, mkd, fr, frd, cc, dc, in, cmp, o, csz,
                             b0 * (n / chunk), b1 * (n / chunk), chunk, cap, 0, 0};
    }
    run_sphase(tasks, nthreads, 0); /* warm-up */
    run_sphase(tasks, nthreads, 1);
    double tc = 0, td = 0;
    for (int r = 0; r < reps; r++) {
        tc += run_sphase(tasks, nthreads, 0);
        td += run_sphase(tasks, nthreads, 1);
    }
    long long tot = 0;
    int bad = 0;
    for (long long c = 0; c < nch; c++) tot += csz[c];
    for (int i = 0; i < nthreads; i++) bad += tasks[i].bad;
    if (memcmp(in, o, (size_t)nblocks * n) != 0) bad++;
    out[0] = tc;
    out[1] = td;
    out[2] = (double)tot;
    out[3] = bad;
    out[4] = (double)nblocks * n;
    free(in); free(cmp); free(o); free(csz);
    dlclose(h);
    return 0;
}

/*
 * Handle-based form (bench.py's thread sweep): the sample is
 * generated once (in parallel, untimed, pre-faulted), compressed once untimed so
 * decode-only timings have input, then timed at any number of thread counts.
 *   h = cpu_bench_prepare(lib, prefix, nblocks, n, kind, gen_threads)
 *   cpu_bench_time(h, nthreads, reps, mode, out)   mode 0 = compress + decompress,
 *                                                  mode 1 = decompress only
 *   cpu_bench_free(h)
 * out[] as cpu_bench_run.  Every timed decompress is checked against the input.
 */
typedef struct {
    void *dl;
    comp_fn comp;
    dec_fn dec;
    uint8_t *in, *cmp, *out;
    int *csz;
    int n, cap, nblocks;
} bench_t;

typedef struct {
    uint8_t *out;
    int n, kind;
    long long first;
    int count;
} gen_t;

static void *gen_worker(void *arg)
{
    gen_t *g = (gen_t *)arg;
    if (g->count > 0) synth_blocks(g->out, g->n, g->n, g->first, g->count, g->kind);
    return NULL;
}

void *cpu_bench_prepare(const char *lib, const char *prefix, int nblocks, int n, int kind,
                        int gen_threads)
{
    char name[128];
    bench_t *b = calloc(1, sizeof *b);
    if (!b || nblocks < 1 || n < 1) { free(b); return NULL; }
    b->dl = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
    if (!b->dl) { fprintf(stderr, "cpu_bench: %s\n", dlerror()); free(b); return NULL; }
    snprintf(name, sizeof name, "%scompress_default", prefix);
    b->comp = (comp_fn)dlsym(b->dl, name);
    snprintf(name, sizeof name, "%sdecompress_safe", prefix);
    b->dec = (dec_fn)dlsym(b->dl, name);
    b->n = n;
    b->cap = n + n / 255 + 16;
    b->nblocks = nblocks;
    b->in = malloc((size_t)nblocks * n);
    b->cmp = malloc((size_t)nblocks * b->cap);
    b->out = malloc((size_t)nblocks * n);
    b->csz = calloc((size_t)nblocks, sizeof(int));
    if (!b->comp || !b->dec || !b->in || !b->cmp || !b->out || !b->csz) {
        free(b->in); free(b->cmp); free(b->out); free(b->csz);
        dlclose(b->dl);
        free(b);
        return NULL;
    }
    if (gen_threads < 1) gen_threads = 1;
    if (gen_threads > 256) gen_threads = 256;
    pthread_t th[256];
    gen_t g[256];
    for (int i = 0; i < gen_threads; i++) {
        long long b0 = (long long)nblocks * i / gen_threads, b1 = (long long)nblocks * (i + 1) / gen_threads;
        g[i] = (gen_t){b->in + b0 * n, n, kind, b0, (int)(b1 - b0)};
        pthread_create(&th[i], NULL, gen_worker, &g[i]);
    }
    for (int i = 0; i < gen_threads; i++) pthread_join(th[i], NULL);
    memset(b->out, 0, (size_t)nblocks * n); /* pre-fault */
    /* one untimed compress (also pre-faults cmp) so decode-only runs have input */
    task_t tasks[256];
    for (int i = 0; i < gen_threads; i++)
        tasks[i] = (task_t){b->comp, b->dec, b->in, b->cmp, b->out, b->csz, n, b->cap,
                            (int)((long long)nblocks * i / gen_threads),
                            (int)((long long)nblocks * (i + 1) / gen_threads), 0, 0};
    run_phase(tasks, gen_threads, 0);
    return b;
}

int cpu_bench_time(void *h, int nthreads, int reps, int mode, double *out)
{
    bench_t *b = (bench_t *)h;
    if (!b || nthreads < 1 || nthreads > 256 || reps < 1) return -1;
    task_t tasks[256];
    for (int i = 0; i < nthreads; i++)
        tasks[i] = (task_t){b->comp, b->dec, b->in, b->cmp, b->out, b->csz, b->n, b->cap,
                            (int)((long long)b->nblocks * i / nthreads),
                            (int)((long long)b->nblocks * (i + 1) / nthreads), 0, 0};
    if (mode == 0) run_phase(tasks, nthreads, 0); /* warm-up */
    run_phase(tasks, nthreads, 1);
    for (int i = 0; i < nthreads; i++) tasks[i].bad = 0;
    double tc = 0, td = 0;
    for (int r = 0; r < reps; r++) {
        if (mode == 0) tc += run_phase(tasks, nthreads, 0);
        td += run_phase(tasks, nthreads, 1);
    }
    long long tot = 0;
    int bad = 0;
    for (int k = 0; k < b->nblocks; k++) tot += b->csz[k];
    for (int i = 0; i < nthreads; i++) bad += tasks[i].bad;
    if (memcmp(b->in, b->out, (size_t)b->nblocks * b->n) != 0) bad++;
    memset(b->out, 0, (size_t)b->nblocks * b->n);
    out[0] = tc;
    out[1] = td;
    out[2] = (double)tot;
    out[3] = bad;
    out[4] = (double)b->nblocks * b->n;
    return 0;
}

void cpu_bench_free(void *h)
{
    bench_t *b = (bench_t *)h;
    if (!b) return;
    free(b->in); free(b->cmp); free(b->out); free(b->csz);
    dlclose(b->dl);
    free(b);
}

/* ---------------------------------------------------------------------------------
 * cpu_sock_run: the reference's own LZ4 socket codec over loopback TCP (BASELINE config
 * 5 CPU baseline).  Restates the codec calls of ape_socket.c without
 * its event loop:
 *   TX (ape_socket_write, src/ape_socket.c:811-871): each message is cut into 8 KiB
 *     blocks (APE_LZ4_BLOCK_SIZE, :39), each compressed with compress_fast_continue
 *     (accel 1) into [int32 size][block], then saveDict(64 KiB) (:856); write() the frames;
 *   RX (ape_socket_read_lz4_stream, :1333-1467): read() into a buffer, take complete
 *     frames [int32 size][block] (a split-safe parser: the reference's desyncs),
 *     decompress_safe_continue into an 8 KiB block, append it to the 64 KiB dictionary
 *     buffer (memmove when full, :1398-1413) and setStreamDecode on it (:1421).
 * Threads: nthr TX threads and nthr RX threads (nthr <= nconn), thread t serving the
 * connections i = t, t + nthr, ... -- one connection per thread pair for nthr = nconn (the
 * config 5 single connection), an event loop per core for many connections (a TX thread
 * sends message m of each of its connections in turn; an RX thread polls its sockets).
 * Messages are the App. C blocks of `msg` bytes (the benchmark's 64 KiB).  Timed region =
 * the GPU leg's (bench.py sock_leg): every message is generated before the clock starts and
 * the delivered payload is compared after it stops, so the clock holds only
 * compress/frame/write and read/parse/decode/ring work.  out: [0] seconds, [1] payload
 * bytes, [2] wire bytes, [3] errors.
 * --------------------------------------------------------------------------------- */
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

typedef void *(*smk_fn)(void);
typedef int (*sfree_fn)(void *);
typedef int (*scc_fn)(void *, const char *, char *, int, int, int);
typedef int (*ssave_fn)(void *, char *, int);
typedef int (*sdc_fn)(void *, const char *, char *, int, int);
typedef int (*ssetd_fn)(void *, const char *, int);

enum { SK_BLOCK = 8192, SK_DICT = 65536, SK_RBUF = 1 << 20 };

typedef struct {
    smk_fn mk, mkd;
    sfree_fn fr, frd;
    scc_fn cc;
    ssave_fn save;
    sdc_fn dc;
    ssetd_fn setd;
} skfn_t;

typedef struct {               /* one connection */
    int fd_tx, fd_rx;
    uint8_t *src;              /* nmsg * msg bytes, generated before the clock starts */
    uint8_t *dst;              /* nmsg * msg bytes, the delivered payload */
    long long delivered, wire;
    void *st, *sd;             /* TX stream, RX stream decode */
    char *dict_tx, *ring, *rbuf;
    size_t used;
    int dpos, eof, bad;
} sconn_t;

typedef struct {               /* one TX or RX thread */
    const skfn_t *f;
    sconn_t *cs;
    int nconn, nthr, t, msg, nmsg;
} sthr_t;

static int sk_write_all(int fd, const char *p, size_t n)
{
    while (n) {
        ssize_t w = write(fd, p, n);
        if (w <= 0) return -1;
        p += w;
        n -= (size_t)w;
    }
    return 0;
}

/* TX: compress + frame + write only; message m of every connection of the thread in turn */
static void *sk_tx(void *arg)
{
    sthr_t *T = (sthr_t *)arg;
    const int cap = SK_BLOCK + SK_BLOCK / 255 + 16;
    char *frames = malloc((size_t)(T->msg / SK_BLOCK + 1) * (cap + 4));
    for (int m = 0; m < T->nmsg && frames; m++) {
        for (int i = T->t; i < T->nconn; i += T->nthr) {
            sconn_t *c = &T->cs[i];
            if (c->bad) continue;
            const uint8_t *msg = c->src + (size_t)m * T->msg;
            int pos = 0;
            for (int off = 0; off < T->msg; off += SK_BLOCK) {
                const int len = T->msg - off < SK_BLOCK ? T->msg - off : SK_BLOCK;
                const int r = T->f->cc(c->st, (const char *)msg + off, frames + pos + 4, len, cap, 1);
                if (r <= 0) { c->bad++; break; }
                memcpy(frames + pos, &r, 4);
                pos += 4 + r;
            }
            T->f->save(c->st, c->dict_tx, SK_DICT);
            if (c->bad || sk_write_all(c->fd_tx, frames, (size_t)pos) != 0) { c->bad++; continue; }
            c->wire += pos;
        }
    }
    for (int i = T->t; i < T->nconn; i += T->nthr) shutdown(T->cs[i].fd_tx, SHUT_WR);
    free(frames);
    return NULL;
}

/* one connection's complete frames: decode, dictionary ring, deliver; 0 or -1 */
static int sk_consume(const skfn_t *f, sconn_t *c, long long total)
{
    const int cap = SK_BLOCK + SK_BLOCK / 255 + 16;
    char tmp[SK_BLOCK];
    size_t p = 0;
    while (c->used - p >= 4) {
        int32_t sz;
        memcpy(&sz, c->rbuf + p, 4);
        if (sz <= 0 || sz > cap) return -1;
        if (c->used - p - 4 < (size_t)sz) break;
        const int rc = f->dc(c->sd, c->rbuf + p + 4, tmp, sz, SK_BLOCK);
        if (rc <= 0) return -1;
        if (c->dpos + rc > SK_DICT) {   /* :1398-1413 */
            const int need = rc - (SK_DICT - c->dpos);
            memmove(c->ring, c->ring + need, (size_t)(c->dpos - need));
            memcpy(c->ring + c->dpos - need, tmp, (size_t)rc);
            c->dpos = SK_DICT;
        } else {
            memcpy(c->ring + c->dpos, tmp, (size_t)rc);
            c->dpos += rc;
        }
        f->setd(c->sd, c->ring, c->dpos);
        if (c->delivered + rc > total) return -1;
        memcpy(c->dst + c->delivered, tmp, (size_t)rc);   /* the application's callback, :1423 */
        c->delivered += rc;
        p += 4 + (size_t)sz;
    }
    memmove(c->rbuf, c->rbuf + p, c->used - p);
    c->used -= p;
    return 0;
}

/* RX: poll the thread's sockets, read + parse + decode + ring, until every one hits EOF */
static void *sk_rx(void *arg)
{
    sthr_t *T = (sthr_t *)arg;
    const long long total = (long long)T->nmsg * T->msg;
    const int mine = (T->nconn - T->t + T->nthr - 1) / T->nthr;
    struct pollfd *pf = calloc((size_t)mine, sizeof *pf);
    int *idx = calloc((size_t)mine, sizeof *idx);
    if (!pf || !idx) { free(pf); free(idx); return NULL; }
    for (;;) {
        int np = 0;
        for (int i = T->t; i < T->nconn; i += T->nthr) {
            if (T->cs[i].eof || T->cs[i].bad) continue;
            pf[np].fd = T->cs[i].fd_rx;
            pf[np].events = POLLIN;
            pf[np].revents = 0;
            idx[np++] = i;
        }
        if (np == 0) break;
        if (np > 1 && poll(pf, (nfds_t)np, -1) < 0) continue;
        for (int q = 0; q < np; q++) {
            if (np > 1 && !(pf[q].revents & (POLLIN | POLLHUP | POLLERR))) continue;
            sconn_t *c = &T->cs[idx[q]];
            ssize_t r = read(c->fd_rx, c->rbuf + c->used, SK_RBUF - c->used);
            if (r < 0) { c->bad++; continue; }
            if (r == 0) { c->eof = 1; continue; }
            c->used += (size_t)r;
            if (sk_consume(T->f, c, total) != 0) c->bad++;
        }
    }
    free(pf);
    free(idx);
    return NULL;
}

int cpu_sock_run2(const char *lib, const char *prefix, int nconn, int msg, int nmsg, int kind,
                  int nthr, double *out)
{
    char name[128];
    void *h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
    if (!h || nconn < 1 || nconn > 4096 || msg <= 0 || nmsg < 0 || nthr < 1) return -1;
    if (nthr > nconn) nthr = nconn;
    skfn_t f;
    memset(&f, 0, sizeof f);
#define SYM(var, type, nm) snprintf(name, sizeof name, "%s" nm, prefix); f.var = (type)dlsym(h, name)
    SYM(mk, smk_fn, "createStream");
    SYM(fr, sfree_fn, "freeStream");
    SYM(mkd, smk_fn, "createStreamDecode");
    SYM(frd, sfree_fn, "freeStreamDecode");
    SYM(cc, scc_fn, "compress_fast_continue");
    SYM(save, ssave_fn, "saveDict");
    SYM(dc, sdc_fn, "decompress_safe_continue");
    SYM(setd, ssetd_fn, "setStreamDecode");
#undef SYM
    if (!f.mk || !f.fr || !f.mkd || !f.frd || !f.cc || !f.save || !f.dc || !f.setd) return -2;
    sconn_t *cs = calloc((size_t)nconn, sizeof(sconn_t));
    sthr_t *ts = calloc((size_t)nthr * 2, sizeof(sthr_t));
    pthread_t *th = calloc((size_t)nthr * 2, sizeof(pthread_t));
    int rc = (cs && ts && th) ? 0 : -4;
    for (int i = 0; i < nconn && rc == 0; i++) {
        sconn_t *c = &cs[i];
        c->fd_tx = c->fd_rx = -1;
        c->src = malloc((size_t)nmsg * msg + 1);
        c->dst = malloc((size_t)nmsg * msg + 1);
        c->dict_tx = malloc(SK_DICT);
        c->ring = malloc(SK_DICT);
        c->rbuf = malloc(SK_RBUF);
        c->st = f.mk();
        c->sd = f.mkd();
        if (!c->src || !c->dst || !c->dict_tx || !c->ring || !c->rbuf || !c->st || !c->sd) { rc = -4; break; }
        synth_blocks(c->src, msg, msg, (long long)i * nmsg, nmsg, kind);
        int ls = socket(AF_INET, SOCK_STREAM, 0), one = 1;
        struct sockaddr_in a;
        socklen_t al = sizeof a;
        memset(&a, 0, sizeof a);
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
        if (ls < 0 || bind(ls, (struct sockaddr *)&a, sizeof a) || listen(ls, 1) ||
            getsockname(ls, (struct sockaddr *)&a, &al)) { if (ls >= 0) close(ls); rc = -3; break; }
        c->fd_tx = socket(AF_INET, SOCK_STREAM, 0);
        if (connect(c->fd_tx, (struct sockaddr *)&a, sizeof a)) { close(ls); rc = -3; break; }
        c->fd_rx = accept(ls, NULL, NULL);
        close(ls);
        if (c->fd_rx < 0) { rc = -3; break; }
        int b = 4 << 20;
        setsockopt(c->fd_tx, SOL_SOCKET, SO_SNDBUF, &b, sizeof b);
        setsockopt(c->fd_rx, SOL_SOCKET, SO_RCVBUF, &b, sizeof b);
    }
    double t0 = 0, t1 = 0;
    if (rc == 0) {
        for (int t = 0; t < 2 * nthr; t++) {
            ts[t].f = &f;
            ts[t].cs = cs;
            ts[t].nconn = nconn;
            ts[t].nthr = nthr;
            ts[t].t = t % nthr;
            ts[t].msg = msg;
            ts[t].nmsg = nmsg;
        }
        t0 = now_s();
        for (int t = 0; t < nthr; t++) {
            pthread_create(&th[2 * t], NULL, sk_tx, &ts[t]);
            pthread_create(&th[2 * t + 1], NULL, sk_rx, &ts[nthr + t]);
        }
        for (int t = 0; t < 2 * nthr; t++) pthread_join(th[t], NULL);
        t1 = now_s();
    }
    long long wire = 0;
    int bad = 0;
    for (int i = 0; i < nconn && cs; i++) {
        sconn_t *c = &cs[i];
        if (rc == 0) {
            wire += c->wire;
            bad += c->bad;
            if (c->delivered != (long long)nmsg * msg || memcmp(c->dst, c->src, (size_t)nmsg * msg) != 0)
                bad++;
        }
        if (c->fd_tx >= 0) close(c->fd_tx);
        if (c->fd_rx >= 0) close(c->fd_rx);
        if (c->st) f.fr(c->st);
        if (c->sd) f.frd(c->sd);
        free(c->src); free(c->dst); free(c->dict_tx); free(c->ring); free(c->rbuf);
    }
    free(cs); free(ts); free(th);
    if (rc) return rc;
    out[0] = t1 - t0;
    out[1] = (double)nconn * nmsg * msg;
    out[2] = (double)wire;
    out[3] = bad;
    return 0;
}

/* one TX and one RX thread per connection (the round-3 interface) */
int cpu_sock_run(const char *lib, const char *prefix, int nconn, int msg, int nmsg, int kind,
                 double *out)
{
    return cpu_sock_run2(lib, prefix, nconn, msg, nmsg, kind, nconn, out);
}

/* sock_ceiling: plain bytes over one loopback TCP connection (no codec), `chunk`-byte
 * write()s from one thread and read()s into a buffer in another -- the ceiling of the
 * config 5 byte path.  sock_ceiling_buf: the same with the writer walking through a
 * `buf_bytes` source buffer and the reader through a `buf_bytes` destination buffer: with
 * 1 GiB buffers every syscall copies cache-cold memory, as the codec path's do (its frames
 * arrive by DMA and its receive buffer is read by DMA; sock_ceiling's one 4 MiB buffer stays
 * in the CPU caches).  out: [0] seconds, [1] bytes. */
typedef struct { int fd; long long n; int chunk; const char *buf; size_t bsz; } rawc_t;

static void *raw_tx(void *arg)
{
    rawc_t *c = (rawc_t *)arg;
    size_t pos = 0;
    for (long long left = c->n; left > 0;) {
        const int k = left < c->chunk ? (int)left : c->chunk;
        if (pos + (size_t)k > c->bsz) pos = 0;
        if (sk_write_all(c->fd, c->buf + pos, (size_t)k)) break;
        pos += (size_t)k;
        left -= k;
    }
    shutdown(c->fd, SHUT_WR);
    return NULL;
}

int sock_ceiling_buf(long long nbytes, int chunk, long long buf_bytes, double *out)
{
    if (chunk <= 0 || buf_bytes < chunk) return -1;
    char *src = malloc((size_t)buf_bytes), *dst = malloc((size_t)buf_bytes);
    if (!src || !dst) { free(src); free(dst); return -1; }
    memset(src, 0x5a, (size_t)buf_bytes);
    memset(dst, 0, (size_t)buf_bytes);
    int ls = socket(AF_INET, SOCK_STREAM, 0), one = 1, b = 4 << 20;
    struct sockaddr_in a;
    socklen_t al = sizeof a;
    memset(&a, 0, sizeof a);
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (ls < 0 || bind(ls, (struct sockaddr *)&a, sizeof a) || listen(ls, 1) ||
        getsockname(ls, (struct sockaddr *)&a, &al)) { free(src); free(dst); return -1; }
    rawc_t c = {socket(AF_INET, SOCK_STREAM, 0), nbytes, chunk, src, (size_t)buf_bytes};
    if (connect(c.fd, (struct sockaddr *)&a, sizeof a)) { free(src); free(dst); return -1; }
    const int rfd = accept(ls, NULL, NULL);
    close(ls);
    setsockopt(c.fd, SOL_SOCKET, SO_SNDBUF, &b, sizeof b);
    setsockopt(rfd, SOL_SOCKET, SO_RCVBUF, &b, sizeof b);
    pthread_t th;
    const double t0 = now_s();
    pthread_create(&th, NULL, raw_tx, &c);
    long long got = 0;
    size_t pos = 0;
    for (;;) {
        if (pos + (size_t)chunk > (size_t)buf_bytes) pos = 0;
        ssize_t r = read(rfd, dst + pos, (size_t)chunk);
        if (r <= 0) break;
        got += r;
        pos += (size_t)r;
    }
    pthread_join(th, NULL);
    const double t1 = now_s();
    close(c.fd);
    close(rfd);
    free(src);
    free(dst);
    out[0] = t1 - t0;
    out[1] = (double)got;
    return got == nbytes ? 0 : -2;
}

int sock_ceiling(long long nbytes, int chunk, double *out)
{
    return sock_ceiling_buf(nbytes, chunk, chunk, out);
}
