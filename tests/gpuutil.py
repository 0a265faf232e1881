"""Device-batch packing helpers for the GPU tests (torch is only plumbing here).

Every output buffer made by alloc_out() is filled with a canary byte and registered;
tests/conftest.py checks after each GPU test that no byte outside the slots
[off, off + max(cap, 0)) changed -- the reference's guarantee that a codec call never
writes outside dst[0:cap) (ref src/ape_lz4.h:94-95, 115-116)."""
import numpy as np

CANARY = 0xCB
_REGISTERED = []   # (device tensor, [(off, writable bytes)])


def pack(torch, blobs, align=16, misalign=None, min_len=1, extra=64):
    """Copy byte strings into one CUDA buffer; returns (buffer, int64 ptr tensor, offsets).

    misalign: optional list of byte offsets (0..15) added to each blob start."""
    offs, pos = [], 0
    for i, b in enumerate(blobs):
        pos = (pos + align - 1) // align * align
        if misalign is not None:
            pos += misalign[i]
        offs.append(pos)
        pos += max(len(b), min_len) + extra
    host = np.full(pos + 64, CANARY, dtype=np.uint8)
    for o, b in zip(offs, blobs):
        if len(b):
            host[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    ptrs = torch.tensor([dev.data_ptr() + o for o in offs], dtype=torch.int64, device="cuda")
    return dev, ptrs, offs


def alloc_out(torch, caps, misalign=None, extra=64):
    """Output slots of max(cap, 1) + extra bytes, canary-filled; only [off, off + cap) may
    be written (checked after the test)."""
    offs, pos = [], 0
    for i, c in enumerate(caps):
        pos = (pos + 15) // 16 * 16
        if misalign is not None:
            pos += misalign[i]
        offs.append(pos)
        pos += max(c, 1) + extra
    dev = torch.full((pos + 64,), CANARY, dtype=torch.uint8, device="cuda")
    ptrs = torch.tensor([dev.data_ptr() + o for o in offs], dtype=torch.int64, device="cuda")
    _REGISTERED.append((dev, [(o, max(int(c), 0)) for o, c in zip(offs, caps)]))
    return dev, ptrs, offs


def check_canaries():
    """Raise AssertionError naming the first slot whose canary was overwritten."""
    try:
        for dev, slots in _REGISTERED:
            host = dev.cpu().numpy()
            keep = np.ones(host.shape[0], dtype=bool)
            for o, c in slots:
                keep[o:o + c] = False
            bad = np.nonzero(keep & (host != CANARY))[0]
            if bad.size:
                at = int(bad[0])
                owner = max((i for i, (o, _) in enumerate(slots) if o <= at), default=-1)
                raise AssertionError(
                    "write outside dst[0:cap): byte %d (%d bytes in all) after slot %d %s" %
                    (at, bad.size, owner, slots[owner] if owner >= 0 else None))
    finally:
        _REGISTERED.clear()


def ints(torch, xs):
    return torch.tensor(list(xs), dtype=torch.int32, device="cuda")


def fetch(dev, off, n):
    return bytes(dev[off:off + n].cpu().numpy().tobytes()) if n > 0 else b""
