"""Device-batch packing helpers for the GPU tests (torch is only plumbing here)."""
import numpy as np


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
    host = np.zeros(pos + 64, dtype=np.uint8)
    for o, b in zip(offs, blobs):
        if len(b):
            host[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    ptrs = torch.tensor([dev.data_ptr() + o for o in offs], dtype=torch.int64, device="cuda")
    return dev, ptrs, offs


def alloc_out(torch, caps, misalign=None, extra=64):
    offs, pos = [], 0
    for i, c in enumerate(caps):
        pos = (pos + 15) // 16 * 16
        if misalign is not None:
            pos += misalign[i]
        offs.append(pos)
        pos += max(c, 1) + extra
    dev = torch.zeros(pos + 64, dtype=torch.uint8, device="cuda")
    ptrs = torch.tensor([dev.data_ptr() + o for o in offs], dtype=torch.int64, device="cuda")
    return dev, ptrs, offs


def ints(torch, xs):
    return torch.tensor(list(xs), dtype=torch.int32, device="cuda")


def fetch(dev, off, n):
    return bytes(dev[off:off + n].cpu().numpy().tobytes()) if n > 0 else b""
