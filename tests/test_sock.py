"""Socket path (BASELINE config 5; lz4_sock.hip): the receive buffer and its frame parser
(the rewrite of ape_socket_read_lz4_stream, ref src/ape_socket.c:1333-1467, whose header
handling desyncs -- SURVEY K7: :1372-1374 uint32 pointer arithmetic, :1379 position
advanced by the whole read, :1459 memmove from an advanced pointer), and the loopback TCP
TX/RX through the GPU codec.

CPU tests: frames split at every possible point (1-byte reads, headers split over
reads, several frames per read) are recovered exactly; malformed sizes are rejected
(ref :1382-1384 bounds the size by APE_LZ4_BLOCK_COMP_SIZE).  GPU tests: a real
127.0.0.1 connection, blocks compared byte for byte, the host output pads untouched."""
import random
import socket
import threading

import numpy as np
import pytest
from lz4util import I


def frame(blocks):
    out = bytearray()
    for b in blocks:
        out += len(b).to_bytes(4, "little") + b
    return bytes(out)


def feed_and_parse(product, stream, cuts, max_block, max_frames=1000):
    """Append `stream` in pieces at `cuts`; after each append take the complete frames."""
    rb = product.RxBuf(0)
    got = []
    prev = 0
    for c in list(cuts) + [len(stream)]:
        assert rb.append(stream[prev:c]) == 0
        prev = c
        n, off = rb.frames(max_frames, max_block)
        assert n >= 0
        data = rb.data()
        for i in range(n):
            sz = int.from_bytes(data[off[i]:off[i] + 4], "little")
            assert off[i + 1] == off[i] + 4 + sz
            got.append(data[off[i] + 4:off[i + 1]])
        rb.consume(off[n])
    assert rb.used() == 0
    rb.free()
    return got


def test_rxbuf_every_split_point(product):
    rng = random.Random(5)
    blocks = [bytes(rng.getrandbits(8) for _ in range(k)) for k in (0, 1, 3, 4, 5, 17, 300)]
    stream = frame(blocks)
    for c in range(len(stream) + 1):   # one cut anywhere, headers included
        assert feed_and_parse(product, stream, [c], 1000) == blocks


def test_rxbuf_one_byte_reads_and_random_reads(product):
    rng = random.Random(7)
    blocks = [bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 2000))) for _ in range(60)]
    stream = frame(blocks)
    assert feed_and_parse(product, stream, range(1, len(stream)), 4096) == blocks
    for _ in range(20):
        cuts = sorted(rng.sample(range(1, len(stream)), rng.randrange(1, 200)))
        assert feed_and_parse(product, stream, cuts, 4096) == blocks


def test_rxbuf_max_frames_and_partial(product):
    blocks = [b"a" * 10, b"b" * 20, b"c" * 30]
    stream = frame(blocks)
    rb = product.RxBuf(16)
    rb.append(stream[:-1])                    # the last block is one byte short
    n, off = rb.frames(1, 100)
    assert n == 1 and off == [0, 14]
    n, off = rb.frames(10, 100)
    assert n == 2 and off == [0, 14, 38]
    rb.append(stream[-1:])
    n, off = rb.frames(10, 100)
    assert n == 3 and off[-1] == len(stream)
    rb.free()


@pytest.mark.parametrize("size", [-1, -2147483648, 101, 0x7FFFFFFF])
def test_rxbuf_malformed_size(product, size):
    rb = product.RxBuf(0)
    rb.append(frame([b"ok"]) + (size & 0xFFFFFFFF).to_bytes(4, "little") + b"x" * 8)
    n, off = rb.frames(10, 100)
    assert n == -1 and off == []
    rb.free()


def test_rxbuf_growth_keeps_bytes(product):
    rb = product.RxBuf(0)
    assert rb.used() == 0
    rng = random.Random(9)
    data = bytes(rng.getrandbits(8) for _ in range(100000))
    for k in range(0, len(data), 7919):
        assert rb.append(data[k:k + 7919]) == 0
    assert rb.used() == len(data) and rb.data() == data
    assert rb.prepare(1 << 20) == 0 and rb.room() >= 1 << 20
    assert rb.data() == data
    rb.consume(12345)
    assert rb.data() == data[12345:]
    rb.free()


# ---------------- GPU: loopback TCP through the codec ----------------
def _pair():
    srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    tx = socket.create_connection(srv.getsockname())
    rx, _ = srv.accept()
    srv.close()
    return tx, rx


def _blocks(cuda, product, nb, n, kind):
    g = cuda.empty((nb, n), dtype=cuda.uint8, device="cuda")
    product.synth_blocks(g, n, 11, kind)
    return g.cpu().numpy()


def _dst(nb, n, pad=64):
    buf = np.full((nb, n + pad), 0xCB, dtype=np.uint8)
    return buf


@pytest.mark.gpu
@pytest.mark.parametrize("kind,batch", [(1, 16), (0, 7), (1, 64)])
def test_socket_loopback_roundtrip(cuda, product, kind, batch):
    nb, n = 40, 65536
    src = _blocks(cuda, product, nb, n, kind)
    dst = _dst(nb, n)
    res = np.full(nb, -9, dtype=np.int32)        # every entry must be written, last batch too
    tx, rx = _pair()
    out = {}

    def txf():
        out["sent"] = product.socket_send_blocks(tx.fileno(), src, n, batch)
        tx.shutdown(socket.SHUT_WR)

    th = threading.Thread(target=txf)
    th.start()
    got = product.socket_recv_blocks(rx.fileno(), dst, n, batch, res)
    th.join()
    tx.close()
    rx.close()
    assert got == nb
    assert (res == n).all()
    assert np.array_equal(dst[:, :n], src)
    assert (dst[:, n:] == 0xCB).all()            # nothing past each block's capacity
    assert out["sent"] > 4 * nb


def _gpu_frames(cuda, product, src):
    nb, n = src.shape
    d = cuda.from_numpy(src).cuda()
    slot = (product.compressBound(n) + 15) // 16 * 16
    comp = cuda.empty((nb, slot), dtype=cuda.uint8, device="cuda")
    csz = cuda.zeros(nb, dtype=cuda.int32, device="cuda")
    sizes = cuda.full((nb,), n, dtype=cuda.int32, device="cuda")
    product.compress_batch(d, sizes, comp, csz)
    off = cuda.zeros(nb + 1, dtype=cuda.int64, device="cuda")
    product.frame_offsets(csz, off)
    frames = cuda.empty(nb * (slot + 4), dtype=cuda.uint8, device="cuda")
    product.frame_pack(comp, csz, off, frames)
    cuda.cuda.synchronize()
    return bytes(frames[:int(off[nb].item())].cpu().numpy())


def _send_pieces(sock, stream, rng, small_until):
    """Write the stream in tiny pieces (1-7 bytes: every header split) up to
    `small_until`, then in random larger pieces."""
    p = 0
    while p < len(stream):
        k = rng.randrange(1, 8) if p < small_until else rng.randrange(1, 70000)
        sock.sendall(stream[p:p + k])
        p += k
    sock.shutdown(socket.SHUT_WR)


@pytest.mark.gpu
def test_socket_recv_fragmented_sender(cuda, product):
    """K7's trigger: headers split across reads.  A sender writing 1-7 byte pieces."""
    nb, n = 24, 65536
    src = _blocks(cuda, product, nb, n, 1)
    stream = _gpu_frames(cuda, product, src)
    dst = _dst(nb, n)
    res = np.zeros(nb, dtype=np.int32)
    tx, rx = _pair()
    th = threading.Thread(target=_send_pieces, args=(tx, stream, random.Random(3), 40000))
    th.start()
    got = product.socket_recv_blocks(rx.fileno(), dst, n, 5, res)
    th.join()
    tx.close()
    rx.close()
    assert got == nb and (res == n).all()
    assert np.array_equal(dst[:, :n], src) and (dst[:, n:] == 0xCB).all()


@pytest.mark.gpu
@pytest.mark.parametrize("damage", ["truncated", "oversized_header", "negative_header"])
def test_socket_recv_malformed_stream(cuda, product, damage):
    nb, n = 6, 65536
    src = _blocks(cuda, product, nb, n, 1)
    stream = bytearray(_gpu_frames(cuda, product, src))
    if damage == "truncated":
        stream = stream[:-100]
    else:
        first = int.from_bytes(stream[0:4], "little")
        at = 4 + first                            # the second frame's header
        bad = product.compressBound(n) + 1 if damage == "oversized_header" else 0x80000000
        stream[at:at + 4] = bad.to_bytes(4, "little")
    dst = _dst(nb, n)
    res = np.zeros(nb, dtype=np.int32)
    tx, rx = _pair()
    th = threading.Thread(target=lambda: (tx.sendall(bytes(stream)), tx.shutdown(socket.SHUT_WR)))
    th.start()
    with pytest.raises(product.GpuError):
        product.socket_recv_blocks(rx.fileno(), dst, n, 4, res)
    th.join()
    tx.close()
    rx.close()
    assert (dst[:, n:] == 0xCB).all()


def test_cpu_sock_baseline_times_codec_only(oracle):
    """bench.py config5.cpu_baseline harness (oracle/cpu_bench.c cpu_sock_run): the
    reference's chained socket codec over loopback delivers every payload byte intact, over
    one and several connections.  Its messages are generated before the clock and compared
    after it; the payload count and wire bytes are returned."""
    import ctypes as C
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = C.CDLL(os.path.join(root, "oracle", "libcpubench.so"))
    lib.cpu_sock_run.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.POINTER(C.c_double)]
    ref = os.path.join(root, "oracle", "_ref", "libape_lz4_ref.so")
    path, prefix = (ref, b"APE_LZ4_") if os.path.exists(ref) else (
        os.path.join(root, "oracle", "liblz4_oracle.so"), b"orc_")
    out = (C.c_double * 4)()
    for nconn, msg, nmsg, kind in ((1, 65536, 16, 1), (3, 20000, 5, 1), (2, 65536, 4, 0)):
        assert lib.cpu_sock_run(path.encode(), prefix, nconn, msg, nmsg, kind, out) == 0
        assert out[3] == 0 and out[1] == nconn * msg * nmsg and out[0] > 0
        assert out[2] > 4 * nconn * nmsg * ((msg + 8191) // 8192)


# ---------------- chained streams: the reference wire format through the GPU ----------------
def _ref_peer():
    """The reference codec itself (oracle/_ref, compiled from src/ape_lz4.c) as the peer of
    the GPU chain; the restatement where _ref is absent."""
    import ctypes as C
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ref = os.path.join(root, "oracle", "_ref", "libape_lz4_ref.so")
    if os.path.exists(ref):
        L, pre = C.CDLL(ref), "APE_LZ4_"
    else:
        L, pre = C.CDLL(os.path.join(root, "oracle", "liblz4_oracle.so")), "orc_"
    f = {}
    for name, res, args in (("createStream", C.c_void_p, []), ("freeStream", C.c_int, [C.c_void_p]),
                            ("createStreamDecode", C.c_void_p, []),
                            ("freeStreamDecode", C.c_int, [C.c_void_p]),
                            ("compress_fast_continue", C.c_int,
                             [C.c_void_p, C.c_char_p, C.c_void_p, C.c_int, C.c_int, C.c_int]),
                            ("saveDict", C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
                            ("decompress_safe_continue", C.c_int,
                             [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
                            ("setStreamDecode", C.c_int, [C.c_void_p, C.c_void_p, C.c_int])):
        fn = getattr(L, pre + name)
        fn.restype, fn.argtypes = res, args
        f[name] = fn
    return f


def _ref_tx(peer, msgs):
    """ape_socket_write's LZ4 path (src/ape_socket.c:811-871) for one connection: every
    message in 8 KiB chunks, compress_fast_continue into [int32 size][block], saveDict."""
    import ctypes as C
    st = C.c_void_p(peer["createStream"]())
    dictbuf = C.create_string_buffer(65536)
    out, keep = bytearray(), []
    for msg in msgs:
        mb = C.create_string_buffer(bytes(msg), len(msg) + 16)
        keep.append(mb)
        for pos in range(0, len(msg), 8192):
            ln = min(8192, len(msg) - pos)
            ob = C.create_string_buffer(8240 + 64)
            r = peer["compress_fast_continue"](st, C.cast(C.byref(mb, pos), C.c_char_p), ob, ln, 8240, 1)
            assert r > 0
            out += r.to_bytes(4, "little") + ob.raw[:r]
        peer["saveDict"](st, dictbuf, 65536)
    peer["freeStream"](st)
    return bytes(out)


def _ref_rx(peer, stream):
    """ape_socket_read_lz4_stream's decode (:1386-1421) for one connection: each frame with
    decompress_safe_continue into an 8 KiB buffer, appended to the 64 KiB dictionary buffer
    (memmove when full), setStreamDecode on it.  Returns the plain bytes (None on an error)."""
    import ctypes as C
    sd = C.c_void_p(peer["createStreamDecode"]())
    ring = C.create_string_buffer(65536)
    rp, p, plain = 0, 0, bytearray()
    while p < len(stream):
        sz = int.from_bytes(stream[p:p + 4], "little", signed=True)
        if sz <= 0 or sz > 8240 or p + 4 + sz > len(stream):
            return None
        blk = C.create_string_buffer(stream[p + 4:p + 4 + sz], sz + 16)
        tmp = C.create_string_buffer(8192 + 64)
        r = peer["decompress_safe_continue"](sd, blk, tmp, sz, 8192)
        if r <= 0:
            return None
        if rp + r > 65536:
            need = r - (65536 - rp)
            C.memmove(ring, C.byref(ring, need), rp - need)
            C.memmove(C.byref(ring, rp - need), tmp, r)
            rp = 65536
        else:
            C.memmove(C.byref(ring, rp), tmp, r)
            rp += r
        peer["setStreamDecode"](sd, ring, rp)
        plain += tmp.raw[:r]
        p += 4 + sz
    peer["freeStreamDecode"](sd)
    return bytes(plain)


def _chain_msgs(cuda, product, nmsg, nconn, msg_len, seed):
    rng = random.Random(seed)
    msgs = np.zeros((nmsg, nconn, msg_len), dtype=np.uint8)
    for m in range(nmsg):
        for i in range(nconn):
            kind = rng.choice(["comp", "comp", "text", "rand"])
            msgs[m, i] = np.frombuffer(I.make(kind, msg_len, seed=seed * 1000 + m * nconn + i), dtype=np.uint8)
    return msgs


def _drain(sock):
    out = bytearray()
    while True:
        b = sock.recv(1 << 20)
        if not b:
            return bytes(out)
        out += b


@pytest.mark.gpu
@pytest.mark.parametrize("msg_len,nmsg,per_round", [(65536, 6, 0), (65536, 7, 2), (25576, 5, 3)])
def test_chain_gpu_tx_decoded_by_reference(cuda, product, monkeypatch, msg_len, nmsg, per_round):
    """GPU chain_send writes the reference's wire format: the reference's own
    decompress_safe_continue + 64 KiB dictionary ring (ape_socket.c:1386-1421) restores every
    message of every connection -- in one round, and in rounds of 2-3 messages (window slides,
    a partial last round)."""
    if per_round:
        monkeypatch.setenv("APE_LZ4_CHAIN_ROUND", str(per_round))
    nconn = 5
    peer = _ref_peer()
    msgs = _chain_msgs(cuda, product, nmsg, nconn, msg_len, seed=msg_len)
    pairs = [_pair() for _ in range(nconn)]
    ch = product.Chain(nconn, msg_len)
    res = {}

    def txf():
        try:
            res["sent"] = ch.send([t.fileno() for t, _ in pairs], msgs)
        finally:
            for t, _ in pairs:
                t.shutdown(socket.SHUT_WR)

    th = threading.Thread(target=txf)
    th.start()
    streams = [None] * nconn
    readers = [threading.Thread(target=lambda i=i: streams.__setitem__(i, _drain(pairs[i][1])))
               for i in range(nconn)]
    for r in readers:
        r.start()
    for r in readers:
        r.join()
    th.join()
    ch.free()
    for t, r in pairs:
        t.close()
        r.close()
    assert res["sent"] == sum(len(s) for s in streams)
    nch = (msg_len + 8191) // 8192
    for i in range(nconn):
        plain = _ref_rx(peer, streams[i])
        assert plain == msgs[:, i, :].tobytes(), i
        # frame count: nch per message, sizes within the chunk bound
        p, nf = 0, 0
        while p < len(streams[i]):
            sz = int.from_bytes(streams[i][p:p + 4], "little")
            assert 0 < sz <= 8240
            p += 4 + sz
            nf += 1
        assert nf == nch * nmsg


@pytest.mark.gpu
@pytest.mark.parametrize("msg_len,nmsg,pieces,per_round,loop", [
    (65536, 6, False, 0, 1), (65536, 7, False, 2, 1), (25576, 4, True, 3, 1),
    (65536, 7, True, 2, 0)])
def test_chain_reference_tx_decoded_by_gpu(cuda, product, monkeypatch, msg_len, nmsg, pieces,
                                           per_round, loop):
    """GPU chain_recv reads the reference's wire format: frames from the reference's own
    compress_fast_continue + saveDict (ape_socket.c:811-871) decode bit-exactly -- in one round
    and in rounds of 2-3 messages (window slides, a partial last round) -- also when the sender
    writes them in 1-7-byte and random pieces (every header split: the K7 parser); with the
    looping decode (one launch per round, the default) and with a launch per chunk position."""
    if per_round:
        monkeypatch.setenv("APE_LZ4_CHAIN_ROUND", str(per_round))
    monkeypatch.setenv("APE_LZ4_CHAIN_LOOP", str(loop))
    nconn = 4
    peer = _ref_peer()
    msgs = _chain_msgs(cuda, product, nmsg, nconn, msg_len, seed=msg_len + 1)
    streams = [_ref_tx(peer, [msgs[m, i].tobytes() for m in range(nmsg)]) for i in range(nconn)]
    pairs = [_pair() for _ in range(nconn)]

    def txf(i):
        t = pairs[i][0]
        if pieces:
            _send_pieces(t, streams[i], random.Random(i), 30000)
        else:
            t.sendall(streams[i])
            t.shutdown(socket.SHUT_WR)

    ths = [threading.Thread(target=txf, args=(i,)) for i in range(nconn)]
    for t in ths:
        t.start()
    out = np.full((nmsg, nconn, msg_len + 32), 0xCB, dtype=np.uint8)
    status = np.full(nconn, -9, dtype=np.int32)
    ch = product.Chain(nconn, msg_len)
    got = ch.recv([r.fileno() for _, r in pairs], out, status)
    ch.free()
    for t in ths:
        t.join()
    for t, r in pairs:
        t.close()
        r.close()
    assert got == nmsg * nconn * msg_len and (status == 0).all()
    assert np.array_equal(out[:, :, :msg_len], msgs)
    assert (out[:, :, msg_len:] == 0xCB).all()


@pytest.mark.gpu
@pytest.mark.parametrize("split,per_round", [((2, 1, 4), 2), ((1, 6), 0), ((3, 3, 1), 16)])
def test_chain_recv_resumes_across_calls(cuda, product, monkeypatch, split, per_round):
    """the sender writes all messages at once, so one read can take in frames past
    the messages a recv call needs; those bytes stay with the chain and the next recv on it
    resumes mid-stream against the right 64 KiB history.  Several recv calls, every byte
    compared."""
    if per_round:
        monkeypatch.setenv("APE_LZ4_CHAIN_ROUND", str(per_round))
    nconn, msg_len, nmsg = 3, 65536, sum(split)
    peer = _ref_peer()
    msgs = _chain_msgs(cuda, product, nmsg, nconn, msg_len, seed=99)
    streams = [_ref_tx(peer, [msgs[m, i].tobytes() for m in range(nmsg)]) for i in range(nconn)]
    pairs = [_pair() for _ in range(nconn)]

    def txf(i):
        pairs[i][0].sendall(streams[i])
        pairs[i][0].shutdown(socket.SHUT_WR)

    ths = [threading.Thread(target=txf, args=(i,)) for i in range(nconn)]
    for t in ths:
        t.start()
    ch = product.Chain(nconn, msg_len)
    m0 = 0
    for k in split:
        out = np.full((k, nconn, msg_len), 0xCB, dtype=np.uint8)
        status = np.full(nconn, -9, dtype=np.int32)
        got = ch.recv([r.fileno() for _, r in pairs], out, status)
        assert got == k * nconn * msg_len and (status == 0).all(), (m0, status)
        assert np.array_equal(out, msgs[m0:m0 + k]), m0
        m0 += k
    ch.free()
    for t in ths:
        t.join()
    for t, r in pairs:
        t.close()
        r.close()


@pytest.mark.gpu
def test_chain_errors_are_sticky(cuda, product):
    """a failed recv has consumed frames and advanced the streams, so the chain must
    not resume after it.  Message 1 of connection 0 carries a frame whose size field is past the
    bound (malformed): the call that reaches it fails, and so does every later recv on the chain
    (status -1), though the bytes after it are intact."""
    nconn, msg_len, nmsg = 2, 65536, 4
    peer = _ref_peer()
    msgs = _chain_msgs(cuda, product, nmsg, nconn, msg_len, seed=7)
    streams = [bytearray(_ref_tx(peer, [msgs[m, i].tobytes() for m in range(nmsg)]))
               for i in range(nconn)]
    at, nfr = 0, 0
    while nfr < msg_len // 8192:   # skip message 0's frames of connection 0
        at += 4 + int.from_bytes(streams[0][at:at + 4], "little")
        nfr += 1
    streams[0][at:at + 4] = (1 << 20).to_bytes(4, "little")
    pairs = [_pair() for _ in range(nconn)]

    def txf(i):
        pairs[i][0].sendall(bytes(streams[i]))
        pairs[i][0].shutdown(socket.SHUT_WR)

    ths = [threading.Thread(target=txf, args=(i,)) for i in range(nconn)]
    for t in ths:
        t.start()
    ch = product.Chain(nconn, msg_len)
    fds = [r.fileno() for _, r in pairs]
    out = np.zeros((1, nconn, msg_len), dtype=np.uint8)
    status = np.full(nconn, -9, dtype=np.int32)
    assert ch.recv(fds, out, status) == nconn * msg_len and (status == 0).all()
    assert np.array_equal(out, msgs[0:1])
    for _ in range(2):   # the failing call, then a later one: both raise
        status[:] = -9
        with pytest.raises(product.GpuError):
            ch.recv(fds, out, status)
    assert (status == -1).all()
    ch.free()
    for t in ths:
        t.join()
    for t, r in pairs:
        t.close()
        r.close()


def test_chain_argument_checks(product):
    """Chain.send/recv check the array shapes, dtypes and strides the C side
    assumes (one row pitch = nconn x strides[1]; int32 status of length nconn)."""
    ch = object.__new__(product.Chain)
    ch.nconn, ch.msg_len, ch._c = 4, 100, None
    ok = np.zeros((2, 4, 100), dtype=np.uint8)
    ch._rows(ok, "msgs")
    ch._rows(np.zeros((2, 4, 128), dtype=np.uint8), "msgs")
    for bad in (np.zeros((2, 4, 99), dtype=np.uint8), np.zeros((2, 3, 100), dtype=np.uint8),
                np.zeros((2, 4, 100), dtype=np.int8), np.zeros((2, 4, 200), dtype=np.uint8)[:, :, ::2],
                np.zeros((4, 2, 100), dtype=np.uint8).transpose(1, 0, 2), np.zeros((4, 100), dtype=np.uint8)):
        with pytest.raises(ValueError):
            ch._rows(bad, "msgs")
    with pytest.raises(ValueError):
        ch.recv([0, 1, 2, 3], ok, np.zeros(4, dtype=np.int64))
    with pytest.raises(ValueError):
        ch.recv([0, 1, 2, 3], ok, np.zeros(3, dtype=np.int32))


@pytest.mark.gpu
def test_chain_gpu_roundtrip_and_malformed(cuda, product):
    """GPU TX -> loopback -> GPU RX over 8 connections, every byte compared; then a stream
    with one mutated block fails that connection (status != 0, GpuError), and a truncated one
    raises (early EOF)."""
    nconn, msg_len, nmsg = 8, 65536, 5
    msgs = _chain_msgs(cuda, product, nmsg, nconn, msg_len, seed=7)
    pairs = [_pair() for _ in range(nconn)]
    tx, rx = product.Chain(nconn, msg_len), product.Chain(nconn, msg_len)

    def txf():
        try:
            tx.send([t.fileno() for t, _ in pairs], msgs)
        finally:
            for t, _ in pairs:
                t.shutdown(socket.SHUT_WR)

    th = threading.Thread(target=txf)
    th.start()
    out = np.zeros((nmsg, nconn, msg_len), dtype=np.uint8)
    status = np.full(nconn, -9, dtype=np.int32)
    got = rx.recv([r.fileno() for _, r in pairs], out, status)
    th.join()
    for t, r in pairs:
        t.close()
        r.close()
    assert got == nmsg * nconn * msg_len and (status == 0).all() and np.array_equal(out, msgs)
    tx.free()
    rx.free()
    # damaged streams from the reference sender
    peer = _ref_peer()
    for damage in ("mutated", "truncated"):
        streams = [bytearray(_ref_tx(peer, [msgs[m, i].tobytes() for m in range(2)]))
                   for i in range(3)]
        if damage == "mutated":   # connection 1: the third frame's first literal run -> bad offset
            p = 0
            for _ in range(2):
                p += 4 + int.from_bytes(streams[1][p:p + 4], "little")
            streams[1][p + 4] = 0x0F   # token: no literals, match, then offset bytes of the payload
            streams[1][p + 5] = 0xFF
            streams[1][p + 6] = 0xFF
        else:
            streams[2] = streams[2][:-50]
        pairs = [_pair() for _ in range(3)]
        for (t, _), s in zip(pairs, streams):
            threading.Thread(target=lambda t=t, s=s: (t.sendall(bytes(s)), t.shutdown(socket.SHUT_WR))).start()
        ch = product.Chain(3, msg_len)
        out = np.zeros((2, 3, msg_len), dtype=np.uint8)
        status = np.zeros(3, dtype=np.int32)
        with pytest.raises(product.GpuError):
            ch.recv([r.fileno() for _, r in pairs], out, status)
        ch.free()
        for t, r in pairs:
            t.close()
            r.close()
        if damage == "mutated":
            assert status[1] != 0 and status[0] == 0 and status[2] == 0


def test_chain_reference_peer_matches_golden(golden):
    """The test-side reference peer (_ref_tx / _ref_rx: ape_socket.c's codec calls on the
    reference library) reproduces the golden socket-stream KATs byte for byte, so the GPU
    chain tests above compare against the reference's own wire format."""
    import base64
    peer = _ref_peer()
    for kat in golden["stream"]:
        msgs = [I.make(kat["content"], kat["msg_len"], seed=s) for s in kat["seeds"]]
        want = b"".join(len(base64.b64decode(f)).to_bytes(4, "little") + base64.b64decode(f)
                        for f in kat["frames_b64"])
        assert _ref_tx(peer, msgs) == want, kat["content"]
        assert _ref_rx(peer, want) == b"".join(msgs)
