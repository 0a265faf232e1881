/*
 * ref_socket_lz4.c -- TEST DRIVER: the REFERENCE's own socket stack (src/ape_socket.c,
 * ape_buffer.c, ape_events*.c, ape_netlib.c ... compiled from /root/reference/src by
 * oracle/ref_net.sh) with LZ4 on both directions, linked against libape_lz4_amd.so in place of
 * the reference's ape_lz4.o (the drop-in behind ape_buffer/ape_socket).
 *
 * A client connects to a server over 127.0.0.1; both ends run APE_socket_enable_lz4(TX|RX)
 * (ref ape_socket.c:105-125).  The client sends NMSG messages with APE_socket_write (8 KiB
 * blocks through compress_fast_continue + saveDict, :811-871); the server's on_read gets the
 * bytes decoded by ape_socket_read_lz4_stream (decompress_safe_continue + setStreamDecode on
 * the 64 KiB dictionary ring, :1333-1467), checks them and echoes them back the same way; the
 * client checks the echo and sends the next message.  One message in flight at a time and
 * one event loop, so a message's frames are all queued before the reader's read pass: the
 * reference's reassembly of a frame split across reads stays out of scope.
 *
 * usage: ref_socket_lz4 PORT      exit status 0 = every byte equal both ways
 */
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* the reference's own headers only (ape_socket.h includes ITS ape_lz4.h): the socket code and
 * this driver are compiled against the original declarations and linked to the product .so --
 * a binary drop-in, as an embedder rebuilding nothing but the link would see it */
#include "ape_events_loop.h"
#include "ape_netlib.h"
#include "ape_socket.h"

unsigned long _ape_seed = 0x9E3779B9UL;   /* the embedder defines it (ref ape_hash.c:25) */

#define NMSG 14
static const int k_len[NMSG] = {1, 5, 100, 4096, 8191, 8192, 8193, 12000,
                                16384, 16385, 20000, 24576, 3000, 65536};
static unsigned char *msg[NMSG];
static unsigned char *srv_buf, *cli_buf;
static int cur, srv_got, cli_got, failed;

static uint64_t xs(uint64_t *s)
{
    *s ^= *s << 13;
    *s ^= *s >> 7;
    *s ^= *s << 17;
    return *s;
}

/* even messages: compressible (16 letters and back-copies, as SURVEY App. C); odd: random */
static void make_msg(unsigned char *p, int n, int k)
{
    uint64_t s = 0x9E3779B97F4A7C15ULL * (uint64_t)(k + 1) + 1;
    int i = 0;
    while (i < n) {
        const uint64_t r = xs(&s);
        if (k & 1) {
            p[i++] = (unsigned char)r;
        } else if (i >= 64 && (r & 3)) {
            const int len = 4 + (int)((r >> 32) % 60), off = 1 + (int)((r >> 8) % (uint64_t)i);
            for (int t = 0; t < len && i < n; t++, i++) p[i] = p[i - off];
        } else {
            const int len = 1 + (int)((r >> 8) % 16);
            for (int t = 0; t < len && i < n; t++, i++) p[i] = (unsigned char)('a' + (xs(&s) & 15));
        }
    }
}

static void fail(const char *what)
{
    fprintf(stderr, "ref_socket_lz4: %s (message %d, %d bytes)\n", what, cur, k_len[cur]);
    failed = 1;
    APE_loop_stop();
}

static void cli_send(ape_socket *s)
{
    if (APE_socket_write(s, msg[cur], (size_t)k_len[cur], APE_DATA_STATIC) < 0)
        fail("client write");
}

/* server side (an accepted client inherits the server's callbacks, ref :1224) */
static void srv_on_connect(ape_socket *server, ape_socket *client, ape_global *ape, void *arg)
{
    (void)server; (void)ape; (void)arg;
    APE_socket_enable_lz4(client, APE_LZ4_COMPRESS_TX | APE_LZ4_COMPRESS_RX);
}

static void srv_on_read(ape_socket *s, const uint8_t *data, size_t len, ape_global *ape, void *arg)
{
    (void)ape; (void)arg;
    if (failed) return;
    if (srv_got + (long)len > k_len[cur]) return fail("server got more bytes than sent");
    memcpy(srv_buf + srv_got, data, len);
    srv_got += (int)len;
    if (srv_got < k_len[cur]) return;
    if (memcmp(srv_buf, msg[cur], (size_t)k_len[cur])) return fail("server bytes differ");
    srv_got = 0;
    if (APE_socket_write(s, srv_buf, (size_t)k_len[cur], APE_DATA_STATIC) < 0) fail("echo write");
}

static void cli_on_connected(ape_socket *s, ape_global *ape, void *arg)
{
    (void)ape; (void)arg;
    cli_send(s);
}

static void cli_on_read(ape_socket *s, const uint8_t *data, size_t len, ape_global *ape, void *arg)
{
    (void)ape; (void)arg;
    if (failed) return;
    if (cli_got + (long)len > k_len[cur]) return fail("client got more bytes than echoed");
    memcpy(cli_buf + cli_got, data, len);
    cli_got += (int)len;
    if (cli_got < k_len[cur]) return;
    if (memcmp(cli_buf, msg[cur], (size_t)k_len[cur])) return fail("echoed bytes differ");
    cli_got = 0;
    if (++cur == NMSG) {
        APE_loop_stop();
        return;
    }
    cli_send(s);
}

int main(int argc, char **argv)
{
    const int port = argc > 1 ? atoi(argv[1]) : 47321;
    alarm(60);   /* a stalled exchange ends the test (SIGALRM) */
    srv_buf = malloc(65536);
    cli_buf = malloc(65536);
    for (int k = 0; k < NMSG; k++) {
        msg[k] = malloc((size_t)k_len[k]);
        if (!msg[k]) return 3;
        make_msg(msg[k], k_len[k], k);
    }
    if (APE_LZ4_versionNumber() != 10701) return 4;   /* the drop-in's ABI answer */
    ape_global *ape = APE_init();
    if (!ape) return 5;
    ape_socket *server = APE_socket_new(APE_SOCKET_PT_TCP, 0, ape);
    server->callbacks.on_connect = srv_on_connect;
    server->callbacks.on_read = srv_on_read;
    if (APE_socket_listen(server, (uint16_t)port, "127.0.0.1", 0, 0) != 0) return 6;
    ape_socket *client = APE_socket_new(APE_SOCKET_PT_TCP, 0, ape);
    APE_socket_enable_lz4(client, APE_LZ4_COMPRESS_TX | APE_LZ4_COMPRESS_RX);
    client->callbacks.on_connected = cli_on_connected;
    client->callbacks.on_read = cli_on_read;
    if (APE_socket_connect(client, (uint16_t)port, "127.0.0.1", 0) != 0) return 7;
    APE_loop_run(ape);
    if (failed || cur != NMSG) return 1;
    long tot = 0;
    for (int k = 0; k < NMSG; k++) tot += k_len[k];
    printf("ref_socket_lz4: %d messages, %ld bytes each way, identical\n", NMSG, tot);
    return 0;
}
