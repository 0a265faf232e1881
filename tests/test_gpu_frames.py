"""Framed stream of independent blocks (the batched socket path).

Frame i = [le32 c_i][c_i compressed bytes], frames back to back -- the reference
socket's [int32 size][LZ4 block] layout (src/ape_socket.c:813-850) with
independent blocks.  Checked here: the offsets are the exclusive scan of 4 + c_i,
the packed stream parses on the host into exactly the compressed rows, and
decoding straight out of the stream matches decoding the rows (return values and
bytes), which the oracle also restores.
"""
import numpy as np
import pytest

from lz4util import I, orc_decompress

pytestmark = pytest.mark.gpu


def _blocks(n_blocks, seed):
    rng = np.random.default_rng(seed)
    out = []
    for b in range(n_blocks):
        kind = ("comp", "rand", "text", "zeros")[b % 4]
        n = int(rng.integers(0, 65537)) if b % 5 else (0, 1, 13, 4096, 65536)[b // 5 % 5]
        out.append(I.make(kind, n, seed=b + seed))
    return out


@pytest.mark.parametrize("nb", [1, 7, 1100, 2500])
def test_frames_pack_and_decode(cuda, product, oracle, nb):
    torch = cuda
    amd = product
    srcs = _blocks(nb, nb)
    S = 65536
    slot = (amd.compressBound(S) + 15) // 16 * 16
    host = np.zeros((nb, S), dtype=np.uint8)
    for i, s in enumerate(srcs):
        host[i, :len(s)] = np.frombuffer(s, dtype=np.uint8)
    src = torch.from_numpy(host).cuda()
    sizes = torch.tensor([len(s) for s in srcs], dtype=torch.int32, device="cuda")
    comp = torch.zeros((nb, slot), dtype=torch.uint8, device="cuda")
    csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
    amd.compress_batch(src, sizes, comp, csz)
    off = torch.zeros(nb + 1, dtype=torch.int64, device="cuda")
    amd.frame_offsets(csz, off)
    torch.cuda.synchronize()
    c = csz.cpu().numpy().astype(np.int64)
    assert (c > 0).all()
    want = np.concatenate([[0], np.cumsum(4 + c)])
    assert off.cpu().numpy().tolist() == want.tolist()
    frames = torch.zeros(int(want[-1]) + 64, dtype=torch.uint8, device="cuda")
    amd.frame_pack(comp, csz, off, frames)
    torch.cuda.synchronize()
    fh = frames.cpu().numpy().tobytes()
    ch = comp.cpu().numpy()
    # host-side parse of the stream, as a receiver would
    pos = 0
    for i in range(nb):
        n = int.from_bytes(fh[pos:pos + 4], "little")
        assert n == c[i]
        assert fh[pos + 4:pos + 4 + n] == ch[i, :n].tobytes()
        pos += 4 + n
    assert pos == want[-1]
    # decode straight out of the stream
    out = torch.zeros((nb, S), dtype=torch.uint8, device="cuda")
    res = torch.zeros(nb, dtype=torch.int32, device="cuda")
    amd.decompress_frames(frames, off, out, res, dst_caps=sizes)
    out2 = torch.zeros((nb, S), dtype=torch.uint8, device="cuda")
    res2 = torch.zeros(nb, dtype=torch.int32, device="cuda")
    amd.decompress_batch(comp, csz, out2, res2, dst_caps=sizes)
    torch.cuda.synchronize()
    assert res.cpu().tolist() == [len(s) for s in srcs]
    assert res.cpu().tolist() == res2.cpu().tolist()
    oh = out.cpu().numpy()
    for i in range(0, nb, max(1, nb // 50)):
        assert oh[i, :len(srcs[i])].tobytes() == srcs[i]
        r, o = orc_decompress(oracle, ch[i, :c[i]].tobytes(), len(srcs[i]))
        assert r == len(srcs[i]) and o == srcs[i]
    assert torch.equal(out, out2)


def test_frames_malformed_block_reports_like_decompress_safe(cuda, product):
    """A corrupted block inside the stream returns the same -(consumed)-1 as the
    row-form decoder (the frame header supplies the size)."""
    torch = cuda
    amd = product
    srcs = [I.make("comp", 4096, seed=s) for s in range(3)]
    host = np.zeros((3, 4096), dtype=np.uint8)
    for i, s in enumerate(srcs):
        host[i] = np.frombuffer(s, dtype=np.uint8)
    src = torch.from_numpy(host).cuda()
    sizes = torch.full((3,), 4096, dtype=torch.int32, device="cuda")
    slot = (amd.compressBound(4096) + 15) // 16 * 16
    comp = torch.zeros((3, slot), dtype=torch.uint8, device="cuda")
    csz = torch.zeros(3, dtype=torch.int32, device="cuda")
    amd.compress_batch(src, sizes, comp, csz)
    torch.cuda.synchronize()
    comp[1, 0] = 0xFF      # literal length chain runs off the block
    comp[1, 1:40] = 0xFF
    off = torch.zeros(4, dtype=torch.int64, device="cuda")
    amd.frame_offsets(csz, off)
    frames = torch.zeros(int(off[-1].item()) + 64, dtype=torch.uint8, device="cuda")
    amd.frame_pack(comp, csz, off, frames)
    out = torch.zeros((3, 4096), dtype=torch.uint8, device="cuda")
    res = torch.zeros(3, dtype=torch.int32, device="cuda")
    amd.decompress_frames(frames, off, out, res, dst_caps=sizes)
    res2 = torch.zeros(3, dtype=torch.int32, device="cuda")
    amd.decompress_batch(comp, csz, out.clone(), res2, dst_caps=sizes)
    torch.cuda.synchronize()
    r = res.cpu().tolist()
    assert r == res2.cpu().tolist()
    assert r[0] == 4096 and r[2] == 4096 and r[1] < 0


def test_frames_corrupt_header_is_rejected(cuda, product):
    """a frame header claiming more bytes than its frame holds (or a negative
    size) is rejected with -1 before anything is read past the frame or written; the
    neighbouring frames decode normally (ref src/ape_socket.c:1382-1384 rejects a size
    above the data it has)."""
    torch = cuda
    amd = product
    nb, n = 6, 4096
    srcs = [I.make("comp", n, seed=40 + s) for s in range(nb)]
    host = np.stack([np.frombuffer(s, dtype=np.uint8) for s in srcs])
    src = torch.from_numpy(host).cuda()
    sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
    slot = (amd.compressBound(n) + 15) // 16 * 16
    comp = torch.zeros((nb, slot), dtype=torch.uint8, device="cuda")
    csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
    amd.compress_batch(src, sizes, comp, csz)
    off = torch.zeros(nb + 1, dtype=torch.int64, device="cuda")
    amd.frame_offsets(csz, off)
    frames = torch.zeros(int(off[-1].item()) + 64, dtype=torch.uint8, device="cuda")
    amd.frame_pack(comp, csz, off, frames)
    torch.cuda.synchronize()
    o = off.cpu().tolist()
    fh = frames.cpu().numpy()
    big = (int(csz[1].item()) + 1).to_bytes(4, "little")        # one byte past its frame
    fh[o[1]:o[1] + 4] = np.frombuffer(big, dtype=np.uint8)
    fh[o[3]:o[3] + 4] = np.frombuffer((0x80000001).to_bytes(4, "little"), dtype=np.uint8)
    fh[o[4]:o[4] + 4] = np.frombuffer((0x7FFFFFF0).to_bytes(4, "little"), dtype=np.uint8)
    frames = torch.from_numpy(fh).cuda()
    out = torch.full((nb, n), 0xCB, dtype=torch.uint8, device="cuda")
    res = torch.zeros(nb, dtype=torch.int32, device="cuda")
    amd.decompress_frames(frames, off, out, res, dst_caps=sizes)
    torch.cuda.synchronize()
    r = res.cpu().tolist()
    assert r == [n, -1, n, -1, -1, n], r
    oh = out.cpu().numpy()
    for i in (1, 3, 4):
        assert (oh[i] == 0xCB).all(), i
    for i in (0, 2, 5):
        assert oh[i].tobytes() == srcs[i]
