"""DIAGNOSTIC (GPU box): one compress_batch call of the segment encoder on a chosen input,
printing the per-block results (a guarded build marks loops that ran past their bound)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import torch
import inputs as I
import libapenetwork_amd as amd

kind, nb = sys.argv[1], int(sys.argv[2])
n = 65536
if kind == "zeros":
    srcs = [bytes(n)] * nb
elif kind == "comp":
    srcs = [I.synth_comp(n, b) for b in range(nb)]
elif kind == "runs":
    srcs = [b"\xab" * n, (b"xyz" * 30000)[:n], bytes(1000) + I.synth_rand(2000, 1) + bytes(62536),
            bytes(n), I.text(n), (b"abcd" * 20000)[:n], bytes(30000) + I.synth_comp(35536, 3), I.synth_comp(n, 9)][:nb]
else:
    srcs = [I.synth_rand(n, b) for b in range(nb)]
assert amd.gpu_init() == 0, amd.gpu_last_error()
slot = (amd.compressBound(n) + 15) // 16 * 16
src = torch.tensor(bytearray(b"".join(srcs)), dtype=torch.uint8).view(nb, n).cuda()
sizes = torch.full((nb,), n, dtype=torch.int32, device="cuda")
comp = torch.zeros((nb, slot), dtype=torch.uint8, device="cuda")
csz = torch.zeros(nb, dtype=torch.int32, device="cuda")
amd.compress_batch(src, sizes, comp, csz)
torch.cuda.synchronize()
r = csz.cpu().tolist()
print(kind, nb, "results", r[:8], "min", min(r), "ratio", nb * n / max(1, sum(x for x in r if x > 0)))
# every block decodes (the reference's own decoder when oracle/_ref is present, else the oracle)
import ctypes as C
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
refp = os.path.join(root, "oracle", "_ref", "libape_lz4_ref.so")
L = C.CDLL(refp) if os.path.exists(refp) else C.CDLL(os.path.join(root, "oracle", "liblz4_oracle.so"))
dec = L.APE_LZ4_decompress_safe if hasattr(L, "APE_LZ4_decompress_safe") else L.orc_decompress_safe
ch = comp.cpu().numpy()
bad = 0
for i in range(nb):
    if r[i] <= 0:
        bad += 1
        continue
    blk = ch[i, :r[i]].tobytes()
    out = C.create_string_buffer(n + 64)
    if dec(blk, out, r[i], n) != n or out.raw[:n] != srcs[i]:
        bad += 1
print("decode check: %d bad of %d" % (bad, nb))
sys.exit(1 if bad else 0)
