"""Child process of tests/test_gpu_encode_seg.py (not collected by pytest): the opt-in
segment encoder (APE_LZ4_ENCODER=seg, read once per process by libape_lz4_amd.so) on the
encoder suite's inputs.  Every block must decode back with the oracle restatement and with
the reference library itself (oracle/_ref, when present) at cap = n, fail the same way at
n - 1, stay within compressBound, give limitedOutput's 0 below its size, be deterministic,
and the App. C ratio is printed beside the reference's.  Prints one JSON line; exit 1 on
any failure."""
import ctypes as C
import json
import os
import random
import sys

os.environ["APE_LZ4_ENCODER"] = "seg"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, HERE, os.path.join(HERE, "golden")]

import torch  # noqa: E402  (torch's HIP runtime first, as in conftest.py)

import libapenetwork_amd as amd  # noqa: E402
from gpuutil import alloc_out, fetch, ints, pack  # noqa: E402
from lz4util import I, buf, orc_compress, orc_decompress, ref_lib  # noqa: E402


def encode(srcs, caps=None, in_mis=None, out_mis=None):
    caps = [amd.compressBound(len(s)) for s in srcs] if caps is None else caps
    src, sptr, _ = pack(torch, srcs, misalign=in_mis)
    dst, dptr, doffs = alloc_out(torch, caps, misalign=out_mis)
    res = ints(torch, [-99] * len(srcs))
    sizes, capt = ints(torch, map(len, srcs)), ints(torch, caps)
    rc = amd.lib().APE_LZ4_compress_batch_dev(sptr.data_ptr(), sizes.data_ptr(), dptr.data_ptr(),
                                              capt.data_ptr(), res.data_ptr(), len(srcs), None)
    assert rc == 0, amd.gpu_last_error()
    torch.cuda.synchronize()
    rs = res.cpu().tolist()
    return rs, [fetch(dst, o, r) for o, r in zip(doffs, rs)]


def main():
    import gpuutil
    orc = C.CDLL(os.path.join(ROOT, "oracle", "liblz4_oracle.so"))
    ref = ref_lib()
    rng = random.Random(11)
    srcs = [I.synth_comp(65536, b) for b in range(64)] + \
           [I.synth_rand(4096, b) for b in range(32)] + \
           [I.synth_comp(4096, b) for b in range(32)] + \
           [I.make(c, n) for c in I.ENC_CONTENTS for n in I.ENC_SIZES if n <= 65536] + \
           [bytes(65536), b"\xab" * 65536, (b"xyz" * 30000)[:65536]] + \
           [I.make(rng.choice(["comp", "text", "rand", "zeros", "period7"]),
                   rng.randrange(0, 65537), seed=i) for i in range(48)]
    mis_in = [rng.randrange(16) for _ in srcs]
    mis_out = [rng.randrange(16) for _ in srcs]
    rs, comps = encode(srcs, in_mis=mis_in, out_mis=mis_out)
    bad = []
    for i, (s, r, c) in enumerate(zip(srcs, rs, comps)):
        n = len(s)
        if not 0 < r <= amd.compressBound(n):
            bad.append((i, "size", r))
            continue
        if orc_decompress(orc, c, n) != (n, s):
            bad.append((i, "oracle decode"))
        if ref is not None:
            o = C.create_string_buffer(n + 64)
            if ref.APE_LZ4_decompress_safe(buf(c), o, len(c), n) != n or o.raw[:n] != s:
                bad.append((i, "reference decode"))
            if n:
                rr = ref.APE_LZ4_decompress_safe(buf(c), o, len(c), n - 1)
                if rr >= 0 or rr != orc_decompress(orc, c, n - 1)[0]:
                    bad.append((i, "n-1", rr))
    # limitedOutput: cap = its size gives the same bytes, one less gives 0
    rs2, comps2 = encode(srcs, caps=rs)
    if rs2 != rs or comps2 != comps:
        bad.append(("limited at size",))
    rs3, _ = encode(srcs, caps=[max(r - 1, 0) for r in rs])
    if rs3 != [0] * len(srcs):
        bad.append(("limited below size", [i for i, r in enumerate(rs3) if r]))
    # deterministic
    if encode(srcs) != (rs, comps):
        bad.append(("nondeterministic",))
    try:
        gpuutil.check_canaries()
    except AssertionError as e:
        bad.append(("canary", str(e)))
    ratio = 64 * 65536 / sum(rs[:64])
    ref_ratio = 64 * 65536 / sum(orc_compress(orc, s)[0] for s in srcs[:64])
    print(json.dumps({"blocks": len(srcs), "bad": bad[:10], "nbad": len(bad),
                      "ratio": round(ratio, 4), "ref_ratio": round(ref_ratio, 4),
                      "reference_decoder": ref is not None}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
