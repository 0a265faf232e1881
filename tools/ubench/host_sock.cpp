// host_sock.cpp -- DIAGNOSTIC (not product): what bounds config 5's socket syscalls
// (VERDICT r3 item 7).  The plain-bytes ceiling (oracle/cpu_bench.c sock_ceiling) writes
// one 4 MiB buffer over and over and reads into one 1 MiB buffer: both stay in the CPU
// caches.  The codec path writes frames that a DMA just put in pinned memory and reads into
// a receive buffer that a DMA reads next, so its syscalls copy cache-cold memory.  This
// measures one loopback TCP connection (one writer thread, one reader thread, 4 MiB
// write()s, 4 MiB read()s) for the buffer kinds involved:
//   hot      : one 4 MiB source, one 4 MiB destination (the current ceiling)
//   cold     : sources / destinations walk through 1 GiB buffers (never cache-resident)
//   pinned   : as cold, with hipHostMalloc'd buffers (the TX frame / RX result staging)
//   register : as cold, with malloc'd buffers registered by hipHostRegister (the rxbuf)
// plus single-thread memcpy bandwidth from / to each kind.  One JSON line.
//   hipcc -O2 -o host_sock host_sock.cpp
#include <hip/hip_runtime.h>
#include <arpa/inet.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

static double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

struct Tx {
    int fd;
    const char *buf;
    size_t buf_bytes, total, chunk;
};

static void *tx_main(void *a) {
    Tx *t = (Tx *)a;
    size_t pos = 0;
    for (size_t left = t->total; left;) {
        const size_t k = left < t->chunk ? left : t->chunk;
        if (pos + k > t->buf_bytes) pos = 0;
        size_t done = 0;
        while (done < k) {
            const ssize_t w = write(t->fd, t->buf + pos + done, k - done);
            if (w <= 0) return nullptr;
            done += (size_t)w;
        }
        pos += k;
        left -= k;
    }
    shutdown(t->fd, SHUT_WR);
    return nullptr;
}

// GB/s of `total` bytes over one loopback connection
static double sock_rate(const char *src, size_t src_bytes, char *dst, size_t dst_bytes, size_t total,
                        size_t chunk) {
    int ls = socket(AF_INET, SOCK_STREAM, 0), one = 1, b = 4 << 20;
    sockaddr_in a;
    socklen_t al = sizeof a;
    memset(&a, 0, sizeof a);
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    if (bind(ls, (sockaddr *)&a, sizeof a) || listen(ls, 1) || getsockname(ls, (sockaddr *)&a, &al)) return -1;
    Tx t = {socket(AF_INET, SOCK_STREAM, 0), src, src_bytes, total, chunk};
    if (connect(t.fd, (sockaddr *)&a, sizeof a)) return -1;
    const int rfd = accept(ls, nullptr, nullptr);
    close(ls);
    setsockopt(t.fd, SOL_SOCKET, SO_SNDBUF, &b, sizeof b);
    setsockopt(rfd, SOL_SOCKET, SO_RCVBUF, &b, sizeof b);
    pthread_t th;
    const double t0 = now_s();
    pthread_create(&th, nullptr, tx_main, &t);
    size_t got = 0, pos = 0;
    for (;;) {
        if (pos + chunk > dst_bytes) pos = 0;
        const ssize_t r = read(rfd, dst + pos, chunk);
        if (r <= 0) break;
        got += (size_t)r;
        pos += (size_t)r;
    }
    pthread_join(th, nullptr);
    const double dt = now_s() - t0;
    close(t.fd);
    close(rfd);
    return got == total ? total / dt / 1e9 : -2;
}

static double memcpy_rate(char *dst, const char *src, size_t bytes) {
    const size_t c = 4u << 20;
    const double t0 = now_s();
    for (size_t o = 0; o + c <= bytes; o += c) memcpy(dst + o, src + o, c);
    return bytes / (now_s() - t0) / 1e9;
}

int main() {
    const size_t G = 1ull << 30, total = 8ull << 30, chunk = 4u << 20;
    char *m_src = (char *)malloc(G), *m_dst = (char *)malloc(G), *hot_s = (char *)malloc(chunk),
         *hot_d = (char *)malloc(chunk);
    char *p_src = nullptr, *p_dst = nullptr;
    char *r_src = (char *)aligned_alloc(4096, G), *r_dst = (char *)aligned_alloc(4096, G);
    if (!m_src || !m_dst || !hot_s || !hot_d || !r_src || !r_dst) return 1;
    if (hipHostMalloc((void **)&p_src, G, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&p_dst, G, hipHostMallocDefault) != hipSuccess)
        return 2;
    if (hipHostRegister(r_src, G, hipHostRegisterDefault) != hipSuccess ||
        hipHostRegister(r_dst, G, hipHostRegisterDefault) != hipSuccess)
        return 3;
    for (char *p : {m_src, m_dst, hot_s, hot_d, p_src, p_dst, r_src, r_dst})
        memset(p, 0x5A, p == hot_s || p == hot_d ? chunk : G);
    const double hot = sock_rate(hot_s, chunk, hot_d, chunk, total, chunk);
    const double cold = sock_rate(m_src, G, m_dst, G, total, chunk);
    const double pinned = sock_rate(p_src, G, p_dst, G, total, chunk);
    const double reg = sock_rate(r_src, G, r_dst, G, total, chunk);
    const double mc_m = memcpy_rate(m_dst, m_src, G), mc_p = memcpy_rate(m_dst, p_src, G),
                 mc_pw = memcpy_rate(p_dst, m_src, G), mc_r = memcpy_rate(m_dst, r_src, G);
    printf("{\"loopback_GBps\": {\"hot_4MiB_buffers\": %.3f, \"cold_1GiB_malloc\": %.3f, "
           "\"cold_1GiB_hipHostMalloc\": %.3f, \"cold_1GiB_hipHostRegister\": %.3f}, "
           "\"memcpy_GBps_1thread\": {\"malloc_to_malloc\": %.2f, \"from_hipHostMalloc\": %.2f, "
           "\"to_hipHostMalloc\": %.2f, \"from_hipHostRegister\": %.2f}, \"bytes\": %zu, "
           "\"chunk\": %zu}\n",
           hot, cold, pinned, reg, mc_m, mc_p, mc_pw, mc_r, total, chunk);
    (void)hipHostUnregister(r_src);
    (void)hipHostUnregister(r_dst);
    (void)hipHostFree(p_src);
    (void)hipHostFree(p_dst);
    return 0;
}
