#!/usr/bin/env python3
"""Compression ratio of library variants on real files of this image (DIAGNOSTIC).

Datasets (64 x 64 KiB blocks each, built at run time from files the image ships): the
concatenated Python 3.10 standard-library sources ("pysrc"), a 4 MiB slice of the largest
shared library under torch/lib ("sobin"), and SURVEY App. C blocks ("appC").  Every variant's
blocks are decoded by the product library and compared; the reference's own ratio
(oracle/_ref, when built) is printed beside them.
usage: ratio_files.py v1 v2 ...   ("base" = the product library)"""
import ctypes as C
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
N = 65536


def datasets():
    import torch
    py = b"".join(open(f, "rb").read() for f in sorted(glob.glob("/usr/lib/python3.10/*.py")))
    so = os.path.join(os.path.dirname(torch.__file__), "lib")
    big = sorted(glob.glob(so + "/*.so"), key=os.path.getsize)[-1]
    with open(big, "rb") as f:
        f.seek(50 << 20)
        sob = f.read(64 * N)
    return {"pysrc": py[:64 * N], "sobin": sob}


def main():
    import torch
    import libapenetwork_amd as amd
    names = sys.argv[1:]
    ds = datasets()
    nb = 64
    src = torch.empty((nb, N), dtype=torch.uint8, device="cuda")
    amd.synth_blocks(src, N, 0, 1)
    data = {"appC": src.cpu().numpy().tobytes()}
    data.update(ds)
    slot = (amd.compressBound(N) + 15) // 16 * 16
    comp = torch.empty((nb, slot), dtype=torch.uint8, device="cuda")
    out = torch.empty((nb, N), dtype=torch.uint8, device="cuda")
    sizes = torch.full((nb,), N, dtype=torch.int32, device="cuda")
    csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
    dres = torch.zeros(nb, dtype=torch.int32, device="cuda")
    refp = os.path.join(ROOT, "oracle", "_ref", "libape_lz4_ref.so")
    ref = C.CDLL(refp) if os.path.exists(refp) else None
    print("%-8s" % "variant" + "".join("%10s" % k for k in data))
    if ref is not None:
        row = []
        for k, d in data.items():
            tot = 0
            for i in range(nb):
                o = C.create_string_buffer(slot)
                tot += ref.APE_LZ4_compress_default(d[i * N:(i + 1) * N], o, N, slot)
            row.append(nb * N / tot)
        print("%-8s" % "ref" + "".join("%10.4f" % r for r in row))
    for v in names:
        p = os.path.join(ROOT, "libapenetwork_amd",
                         "libape_lz4_amd.so" if v == "base" else "libape_lz4_amd_%s.so" % v)
        L = C.CDLL(p)
        f = L.APE_LZ4_compress_batch_strided_dev
        f.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                      C.c_void_p, C.c_int, C.c_void_p]
        row, tms = [], []
        for k, d in data.items():
            import numpy as np
            src.copy_(torch.from_numpy(np.frombuffer(d, dtype=np.uint8).reshape(nb, N).copy()))
            ts = []
            for _ in range(5):   # encode time of the 64 blocks (median of 5, HIP events)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f(src.data_ptr(), N, sizes.data_ptr(), comp.data_ptr(), slot, None, csz.data_ptr(),
                  nb, C.c_void_p(torch.cuda.current_stream().cuda_stream))
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            tms.append(sorted(ts)[2])
            amd.decompress_batch(comp, csz, out, dres, dst_caps=sizes)
            torch.cuda.synchronize()
            ok = bool((dres == N).all()) and bool(torch.equal(out, src))
            row.append(nb * N / int(csz.sum()) if ok else float("nan"))
        print("%-8s" % v + "".join("%10.4f" % r for r in row) +
              "   encode ms (64 blocks): " + " ".join("%.3f" % t for t in tms), flush=True)


if __name__ == "__main__":
    main()
