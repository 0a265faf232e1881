#!/usr/bin/env python3
"""Probe (diagnostic): compress+decompress of N x 64 KiB blocks, sequential (encode all,
then decode all, one stream) vs pipelined (sub-batches: encode of sub-batch i+1 on one stream
overlapping decode of sub-batch i on another).  usage: overlap_probe.py [nblocks] [subs]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import libapenetwork_amd as amd
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    subs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    n = 65536
    slot = (amd.compressBound(n) + 15) // 16 * 16
    src = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    for b0 in range(0, nb, 1 << 16):
        amd.synth_blocks(src[b0:b0 + (1 << 16)], n, b0, 1)
    comp = torch.empty((nb, slot), dtype=torch.uint8, device="cuda")
    out = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
    csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
    dres = torch.zeros(nb, dtype=torch.int32, device="cuda")
    sa = torch.cuda.current_stream()
    sb = torch.cuda.Stream()

    def seq():
        amd.compress_batch(src, sizes, comp, csz, stream=sa)
        amd.decompress_batch(comp, csz, out, dres, dst_caps=sizes, stream=sa)

    def pipe():
        q = nb // subs
        for i in range(subs):
            s = slice(i * q, (i + 1) * q)
            amd.compress_batch(src[s], sizes[s], comp[s], csz[s], stream=sa)
            ev = torch.cuda.Event()
            ev.record(sa)
            sb.wait_event(ev)
            amd.decompress_batch(comp[s], csz[s], out[s], dres[s], dst_caps=sizes[s], stream=sb)
        ev = torch.cuda.Event()
        ev.record(sb)
        sa.wait_event(ev)

    for name, fn in (("seq", seq), ("pipe", pipe), ("seq", seq), ("pipe", pipe)):
        fn()
        torch.cuda.synchronize()
        dres.zero_()
        t = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 3
        ok = bool((dres == n).all()) and bool(torch.equal(out[:1024], src[:1024]))
        print("%-5s %.2f ms  %.2f GiB/s  ok %s" % (name, dt * 1e3, nb * n / dt / 2**30, ok), flush=True)


if __name__ == "__main__":
    main()
