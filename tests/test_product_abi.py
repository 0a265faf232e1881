"""CPU tests of the product library (no GPU compute here).

* libape_lz4_amd.so loads and exports every function include/*.h declares;
* ABI sizes/constants match the reference (ape_lz4.h:52-59, 123-127, 240-253, 317-322);
* the host stream codec (the socket TX/RX path) is bit-exact
  with the reference on the golden stream KATs and with the oracle on dictionary /
  prefix / fast decoding;
* one-shot calls run the host codec by default; with the GPU one-shot path
  selected, and for every batch entry point, no GPU means a loud failure (no CPU fallback).
"""
import base64
import ctypes as C
import os
import random
import re
import subprocess

import pytest

from lz4util import I, buf, orc_compress, sha

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = []
    for h in ("ape_lz4.h", "ape_lz4_gpu.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"#define[^\n]*(\\\n[^\n]*)*", "", src)
        for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", src):
            name = m.group(1)
            if name.startswith(("APE_LZ4_", "LZ4_compress_forceExtDict")):
                names.append(name)
    return sorted(set(names))


def test_exports_everything_declared(product):
    L = product.lib()
    names = declared_functions()
    assert len(names) >= 40 + 12
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", product.LIB_PATH], capture_output=True,
                         text=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if " T " in line)
    assert set(names) <= exported


def test_reference_symbol_set(product):
    """The 40 symbols the reference library exports are all present."""
    ref40 = """versionNumber compress_default decompress_safe compressBound compress_fast
    sizeofState compress_fast_extState compress_destSize decompress_fast decompress_safe_partial
    resetStream createStream freeStream loadDict compress_fast_continue saveDict
    createStreamDecode freeStreamDecode setStreamDecode decompress_safe_continue
    decompress_fast_continue decompress_safe_usingDict decompress_fast_usingDict compress
    compress_limitedOutput compress_withState compress_limitedOutput_withState compress_continue
    compress_limitedOutput_continue create sizeofStreamState resetStreamState slideInputBuffer
    decompress_safe_withPrefix64k decompress_fast_withPrefix64k compress_fast_force
    decompress_safe_forceExtDict uncompress uncompress_unknownOutputSize""".split()
    names = ["APE_LZ4_" + n for n in ref40] + ["LZ4_compress_forceExtDict"]
    assert len(names) == 40
    L = product.lib()
    assert all(hasattr(L, n) for n in names)


def test_constants(product, golden):
    L = product.lib()
    assert product.versionNumber() == golden["version"] == 10701
    assert L.APE_LZ4_sizeofState() == L.APE_LZ4_sizeofStreamState() == 16416
    for n in (0, 1, 255, 4096, 65536, 0x7E000000, 0x7E000001, -1):
        assert product.compressBound(n) == (0 if (n & 0xFFFFFFFF) > 0x7E000000 else n + n // 255 + 16)


def _product_stream_frames(L, st):
    L.APE_LZ4_createStream.restype = C.c_void_p
    msgs = [I.make(st["content"], st["msg_len"], seed=s) for s in st["seeds"]]
    s = C.c_void_p(L.APE_LZ4_createStream())
    dictbuf = C.create_string_buffer(65536)
    frames, keep = [], []
    for msg in msgs:
        mb = buf(msg)
        keep.append(mb)
        pos = 0
        while pos < len(msg):
            ln = min(8192, len(msg) - pos)
            ob = C.create_string_buffer(8240 + 64)
            r = L.APE_LZ4_compress_fast_continue(s, C.byref(mb, pos), ob, ln, 8240, 1)
            frames.append(ob.raw[:r])
            pos += ln
        L.APE_LZ4_saveDict(s, dictbuf, 65536)
    L.APE_LZ4_freeStream(s)
    return frames


@pytest.mark.parametrize("idx", [0, 1, 2])
def test_host_stream_codec_golden(product, golden, idx):
    """Socket-style TX (compress_fast_continue + saveDict) and RX (safe_continue + ring)."""
    L = product.lib()
    st = golden["stream"][idx]
    frames = _product_stream_frames(L, st)
    assert [base64.b64encode(f).decode() for f in frames] == st["frames_b64"]
    L.APE_LZ4_createStreamDecode.restype = C.c_void_p
    ds = C.c_void_p(L.APE_LZ4_createStreamDecode())
    ring = C.create_string_buffer(65536)
    rp, rets, plain = 0, [], b""
    for fr in frames:
        tmp = C.create_string_buffer(8192 + 64)
        r = L.APE_LZ4_decompress_safe_continue(ds, buf(fr), tmp, len(fr), 8192)
        rets.append(r)
        if r <= 0:
            break
        plain += tmp.raw[:r]
        if rp + r > 65536:
            keepn = 65536 - r
            C.memmove(ring, C.byref(ring, rp - keepn), keepn)
            rp = keepn
        C.memmove(C.byref(ring, rp), tmp, r)
        rp += r
        L.APE_LZ4_setStreamDecode(ds, ring, rp)
    L.APE_LZ4_freeStreamDecode(ds)
    assert rets == st["dec_rets"] and sha(plain) == st["plain_sha256"]


def test_host_dict_and_fast_decoders_vs_oracle(product, oracle):
    """usingDict (ext + prefix forms), forceExtDict, withPrefix64k, decompress_fast,
    fast_continue and compress_destSize against the oracle, incl. mutated input."""
    L = product.lib()
    rng = random.Random(77)
    for it in range(120):
        n1 = rng.choice([100, 4096, 8192, 65536])
        msg = I.make(rng.choice(["comp", "text", "rand"]), n1 + 8192, seed=it)
        # chunk 2 compressed against chunk 1 as an external dictionary
        st = C.c_void_p(oracle.orc_createStream())
        b1, b2 = buf(msg[:n1]), buf(msg[n1:])
        c1 = C.create_string_buffer(n1 + n1 // 255 + 80)
        oracle.orc_compress_fast_continue(st, b1, c1, n1, n1 + n1 // 255 + 16, 1)
        c2 = C.create_string_buffer(8300)
        k = oracle.orc_compress_fast_continue(st, b2, c2, 8192, 8240, 1)
        comp = bytearray(c2.raw[:k])
        if it % 3 == 2:
            comp[rng.randrange(len(comp))] = rng.randrange(256)
        comp = bytes(comp)
        for name, call in (
            ("safe_usingDict_ext", lambda lib, p, o: getattr(lib, p + "decompress_safe_usingDict")(
                buf(comp), o, len(comp), 8192, b1, n1)),
            ("safe_forceExtDict", lambda lib, p, o: getattr(lib, p + "decompress_safe_forceExtDict")(
                buf(comp), o, len(comp), 8192, b1, n1)),
        ):
            outs = []
            for lib, p in ((L, "APE_LZ4_"), (oracle, "orc_")):
                o = C.create_string_buffer(8192 + 64)
                r = call(lib, p, o)
                outs.append((r, o.raw[:max(r, 0)]))
            assert outs[0] == outs[1], (name, it)
        # prefix form: dictionary immediately precedes dst
        outs = []
        for lib, p in ((L, "APE_LZ4_"), (oracle, "orc_")):
            pre = buf(msg[:n1] + b"\0" * 8300)
            r = getattr(lib, p + "decompress_safe_usingDict")(buf(comp), C.byref(pre, n1),
                                                              len(comp), 8192, pre, n1)
            outs.append((r, pre.raw[n1:n1 + max(r, 0)]))
        assert outs[0] == outs[1]
    # one-shot fast decoders and destSize
    for it in range(200):
        src = I.make(rng.choice(["comp", "text", "rand", "zeros"]), rng.randrange(1, 70000), seed=it)
        _, comp = orc_compress(oracle, src)
        tgt = rng.randrange(1, len(comp) + 20)
        outs = []
        for lib, p in ((L, "APE_LZ4_"), (oracle, "orc_")):
            pad = C.create_string_buffer(65536 + len(src) + 64)
            r1 = getattr(lib, p + "decompress_fast")(buf(comp), C.byref(pad, 65536), len(src))
            r2 = getattr(lib, p + "decompress_safe_withPrefix64k")(buf(comp), C.byref(pad, 65536),
                                                                    len(comp), len(src))
            sz = C.c_int(len(src))
            d = C.create_string_buffer(tgt + 64)
            r3 = getattr(lib, p + "compress_destSize")(buf(src), d, C.byref(sz), tgt)
            outs.append((r1, r2, pad.raw[65536:65536 + len(src)], r3, sz.value, d.raw[:max(r3, 0)]))
        assert outs[0] == outs[1], it


def test_no_gpu_fails_loudly(product):
    """Without a device the GPU entry points report failure; nothing falls back to CPU.
    One-shot calls take the host codec by default; once the GPU one-shot
    path is selected they fail too."""
    L = product.lib()
    if L.APE_LZ4_gpu_device_count() > 0:
        pytest.skip("a GPU is visible here; covered by the -m gpu suite")
    assert product.gpu_init() == -1
    assert "no HIP device" in product.gpu_last_error()
    r, comp = product.compress_default(b"hello hello hello hello hello")   # default: host
    assert r > 0 and product.decompress_safe(comp, 29) == (29, b"hello hello hello hello hello")
    with product.oneshot_on_gpu():
        r, _ = product.compress_default(b"hello hello hello hello hello")
        assert r == 0
        r, _ = product.decompress_safe(b"\x50hello", 5)
        assert r < 0
    # the batch API has no host path at all
    z = C.c_void_p(0)
    assert L.APE_LZ4_compress_batch_dev(z, z, z, z, z, 1, z) != 0
    # argument checks come before the device check (EINVAL = -2), then ENODEV (-1)
    assert L.APE_LZ4_compress_exact_batch_dev(z, z, z, z, z, -1, 1, z) == -2
    assert L.APE_LZ4_compress_exact_batch_dev(z, z, z, z, z, 3, 1, z) == -2
    p = C.c_void_p(8)   # never dereferenced: no device
    assert L.APE_LZ4_compress_exact_batch_dev(p, p, p, p, p, 3, 1, z) == -1


def test_one_shot_compress_above_gpu_block(product, golden, oracle):
    """compress_default / compress_fast / _extState on inputs above the GPU block limit
    (65536 < n <= LZ4_MAX_INPUT_SIZE) run the host codec and return the reference's exact
    block (ref src/ape_lz4.c:766-769 byU32 path), GPU or not."""
    from lz4util import blob_matches
    import base64
    L = product.lib()
    kats = [e for e in golden["encode"] if e["n"] > 65536]
    assert {e["n"] for e in kats} == {65546, 65547}
    for e in kats:
        src = I.make(e["content"], e["n"])
        assert sha(src) == e["in_sha256"]
        out = C.create_string_buffer(e["bound"] + 64)
        r = L.APE_LZ4_compress_default(buf(src), out, e["n"], e["bound"])
        assert r == e["clen"] and blob_matches(e["comp"], out.raw[:r]), (e["content"], e["n"])
        for lim in e["limited"]:
            o2 = C.create_string_buffer(max(lim["cap"], 1) + 64)
            assert L.APE_LZ4_compress_default(buf(src), o2, e["n"], lim["cap"]) == lim["ret"]
        for ac in e["accel"]:
            o3 = C.create_string_buffer(e["bound"] + 64)
            r3 = L.APE_LZ4_compress_fast(buf(src), o3, e["n"], e["bound"], ac["accel"])
            assert r3 == ac["ret"] and sha(o3.raw[:r3]) == ac["sha256"]
    # 65537 and 1 MiB against the oracle (pinned by the KATs above)
    state = C.create_string_buffer(16416)
    for n, content in ((65537, "comp"), (65537, "text"), (1 << 20, "comp"), (1 << 20, "rand"),
                       (300000, "zeros")):
        src = I.make(content, n, seed=n)
        bound = product.compressBound(n)
        er, eout = orc_compress(oracle, src)
        out = C.create_string_buffer(bound + 64)
        assert L.APE_LZ4_compress_default(buf(src), out, n, bound) == er
        assert out.raw[:er] == eout, (n, content)
        out2 = C.create_string_buffer(bound + 64)
        assert L.APE_LZ4_compress_fast_extState(state, buf(src), out2, n, bound, 1) == er
        assert out2.raw[:er] == eout


def test_oneshot_host_routing_threshold(product, golden):
    """APE_LZ4_gpu_set_oneshot_host_below (latency routing): below the
    threshold the one-shot calls run the host codec and return the reference's exact
    results -- compress bytes, decompress_safe and _partial return values and bytes --
    GPU or not; the default (0x7FFFFFFF) keeps every one-shot call on the host."""
    import base64
    from lz4util import blob_matches
    L = product.lib()
    L.APE_LZ4_gpu_set_oneshot_host_below.restype = C.c_int
    L.APE_LZ4_gpu_set_oneshot_host_below.argtypes = [C.c_int]
    prev = L.APE_LZ4_gpu_set_oneshot_host_below(1 << 30)
    try:
        env = os.environ.get("APE_LZ4_ONESHOT_HOST_BELOW")
        assert prev == (int(env) if env else product.ONESHOT_HOST_ALL)
        for e in golden["encode"]:
            if e["n"] > 65536:
                continue
            src = I.make(e["content"], e["n"])
            out = C.create_string_buffer(e["bound"] + 64)
            r = L.APE_LZ4_compress_default(buf(src), out, e["n"], e["bound"])
            assert r == e["clen"] and blob_matches(e["comp"], out.raw[:r]), (e["content"], e["n"])
        for d in golden["decode"]:
            comp = base64.b64decode(d["comp_b64"])
            r, out = product.decompress_safe(comp, d["cap"])
            assert r == d["ret"], d["name"]
            if r > 0 and not d["has_offset0"]:
                assert sha(out) == d["out_sha256"], d["name"]
            pr, _ = product.decompress_safe_partial(comp, d["partial"]["target"], d["cap"])
            assert pr == d["partial"]["ret"], d["name"]
    finally:
        assert L.APE_LZ4_gpu_set_oneshot_host_below(prev) == 1 << 30
    if L.APE_LZ4_gpu_device_count() == 0:   # the GPU one-shot path fails loudly here
        with product.oneshot_on_gpu():
            assert product.compress_default(b"hello hello hello hello hello")[0] == 0


def test_c_caller_links_like_ape_socket(product, golden, tmp_path):
    """The C boundary with a compiled caller: tests/c/ape_socket_caller.c
    uses include/ape_lz4.h as src/ape_socket.c does -- APE_LZ4_COMPRESSBOUND in a constant
    expression, create/free stream and decode stream, 8 KiB compress_fast_continue frames +
    saveDict, decompress_safe_continue with the 64 KiB dictionary ring + setStreamDecode, and
    a stack APE_LZ4_streamDecode_t -- built with gcc -Wall -Werror against the header and
    linked with -lape_lz4_amd.  Its frames must equal the reference's golden socket-stream
    KATs byte for byte, and both RX passes must restore the messages."""
    import base64
    libdir = os.path.join(ROOT, "libapenetwork_amd")
    exe = str(tmp_path / "ape_socket_caller")
    cc = subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror",
                         "-I", os.path.join(ROOT, "include"),
                         os.path.join(ROOT, "tests", "c", "ape_socket_caller.c"),
                         "-L", libdir, "-lape_lz4_amd", "-Wl,-rpath," + libdir, "-o", exe],
                        capture_output=True, text=True)
    assert cc.returncode == 0, cc.stderr
    for kat in golden["stream"]:
        msgs = b"".join(I.make(kat["content"], kat["msg_len"], seed=s) for s in kat["seeds"])
        r = subprocess.run([exe, str(kat["msg_len"])], input=msgs, capture_output=True,
                           timeout=120)
        assert r.returncode == 0, (kat["content"], r.returncode, r.stderr[-500:])
        out = r.stdout
        fb = int.from_bytes(out[:4], "little")
        frames = out[4:4 + fb]
        want = b""
        for f in kat["frames_b64"]:
            blk = base64.b64decode(f)
            want += len(blk).to_bytes(4, "little") + blk
        assert frames == want, kat["content"]
        n = len(msgs)
        assert out[4 + fb:4 + fb + n] == msgs and out[4 + fb + n:] == msgs


def test_encoder_m0_only_in_hop_chain(tmp_path):
    """The walker's hop chain (lz4_encode.hip hop_chain_pm) passes its lane select through m0
    and declares m0 clobbered, which clang accepts for a reserved register without preserving
    it: the kernel is correct only while nothing else in it keeps a value in m0.  Compile the
    encoder as the Makefile does and check every m0 reference in the ISA is the chain's own."""
    import shutil
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc absent")
    csrc = os.path.join(ROOT, "libapenetwork_amd", "csrc")
    out = tmp_path / "enc.s"
    subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                    "-mllvm", "-amdgpu-sched-strategy=max-ilp", "-I" + csrc,
                    "-I" + os.path.join(ROOT, "include"), "-S", "--cuda-device-only",
                    os.path.join(csrc, "lz4_encode.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    uses = [ln.split(";")[0].strip() for ln in out.read_text().splitlines()
            if "m0" in ln.split(";")[0] and not ln.lstrip().startswith((".", ";"))]
    assert uses, "the hop chain's m0 moves are gone: update this test with the asm"
    bad = [u for u in uses if not (u.startswith("s_mov_b32 m0,") or
                                   (u.startswith("v_writelane_b32") and u.endswith(", m0")))]
    assert not bad, bad
