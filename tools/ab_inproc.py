#!/usr/bin/env python3
"""Interleaved in-process kernel-time A/B of library variants (DIAGNOSTIC).

Every variant (libapenetwork_amd/libape_lz4_amd_<v>.so, "base" = the product library) is
loaded into ONE process; the same device-resident App. C blocks are encoded and decoded by
each variant in turn, ROUNDS times, timed with HIP events on one stream; prints the median
encode / decode times and checks each variant's round trip (decode == input, and the
encoded bytes decoded by the base library's decoder) and whether each variant's compressed bytes
equal the first variant's (sizes of every block, bytes of 256 sampled blocks).
usage: ab_inproc.py NBLOCKS ROUNDS v1 v2 ..."""
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import libapenetwork_amd as amd
    nb, rounds, names = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3:]
    n = 65536
    slot = (amd.compressBound(n) + 15) // 16 * 16
    src = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    amd.synth_blocks(src, n, 0, 1)
    comp = torch.empty((nb, slot), dtype=torch.uint8, device="cuda")
    out = torch.empty((nb, n), dtype=torch.uint8, device="cuda")
    sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
    csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
    dres = torch.zeros(nb, dtype=torch.int32, device="cuda")
    libs = {}
    for v in names:
        p = os.path.join(ROOT, "libapenetwork_amd",
                         "libape_lz4_amd.so" if v == "base" else "libape_lz4_amd_%s.so" % v)
        L = C.CDLL(p)
        for f in ("APE_LZ4_compress_batch_strided_dev", "APE_LZ4_decompress_safe_batch_strided_dev"):
            getattr(L, f).argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t,
                                      C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        libs[v] = L
    st = torch.cuda.current_stream()
    sp = C.c_void_p(st.cuda_stream)

    def enc(L):
        L.APE_LZ4_compress_batch_strided_dev(src.data_ptr(), n, sizes.data_ptr(), comp.data_ptr(),
                                             slot, None, csz.data_ptr(), nb, sp)

    def dec(L):
        L.APE_LZ4_decompress_safe_batch_strided_dev(comp.data_ptr(), slot, csz.data_ptr(),
                                                    out.data_ptr(), n, sizes.data_ptr(),
                                                    dres.data_ptr(), nb, sp)

    t = {v: ([], []) for v in names}
    ok = {}
    ref = None   # the first variant's compressed bytes: the others are compared with them
    for v in names:   # warm-up + check
        enc(libs[v]); torch.cuda.synchronize()
        same = None
        if ref is None:
            ref = (comp.clone(), csz.clone())
        else:
            same = bool(torch.equal(csz, ref[1])) and all(
                bool(torch.equal(comp[i, :int(csz[i])], ref[0][i, :int(csz[i])]))
                for i in range(0, nb, max(1, nb // 256)))
        dec(libs[v]); torch.cuda.synchronize()
        ok[v] = bool((dres == n).all()) and bool(torch.equal(out, src))
        ratio = nb * n / int(csz.sum())
        dec(libs[names[0]]); torch.cuda.synchronize()
        ok[v] = ok[v] and bool((dres == n).all()) and bool(torch.equal(out, src))
        print("%-12s ok %s ratio %.4f%s" % (v, ok[v], ratio, "" if same is None else
                                             "  bytes %s the first variant's (256 sampled blocks)"
                                             % ("identical to" if same else "DIFFER from")),
              flush=True)
    for r in range(rounds):
        for v in names:
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(st); enc(libs[v]); e[1].record(st); dec(libs[v]); e[2].record(st)
            torch.cuda.synchronize()
            t[v][0].append(e[0].elapsed_time(e[1]))
            t[v][1].append(e[1].elapsed_time(e[2]))
    base = statistics.median(t[names[0]][0])
    for v in names:
        me, md = statistics.median(t[v][0]), statistics.median(t[v][1])
        print("%-12s enc %.3f ms (min %.3f, %+.1f%%)  dec %.3f ms (min %.3f)" % (
            v, me, min(t[v][0]), 100 * (me / base - 1), md, min(t[v][1])), flush=True)


if __name__ == "__main__":
    main()
