#!/usr/bin/env python3
"""Generate tests/golden/lz4_golden.json from the REFERENCE codec itself.

Runs the reference /root/reference/src/ape_lz4.c compiled by oracle/Makefile into
oracle/_ref/libape_lz4_ref.so (this container only; the GPU box never sees the
reference).  The fixtures are data: inputs are rebuilt from (content, n, seed)
by tests/golden/inputs.py and pinned by sha256; expected outputs are the
reference's bytes (base64 when <= 8 KiB, sha256 otherwise) and return codes.

Usage:  make -C oracle && python3 tests/golden/gen_golden.py
"""
import base64
import ctypes as C
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import inputs as I  # noqa: E402

REF = os.path.join(HERE, "..", "..", "oracle", "_ref", "libape_lz4_ref.so")
ref = C.CDLL(REF)
for f in ("createStream", "createStreamDecode"):
    getattr(ref, "APE_LZ4_" + f).restype = C.c_void_p
F = lambda name: getattr(ref, "APE_LZ4_" + name)  # noqa: E731
B64_MAX = 8192


def enc_blob(b):
    if len(b) <= B64_MAX:
        return {"b64": base64.b64encode(b).decode()}
    return {"len": len(b), "sha256": I.sha(b)}


def cbuf(b, pad=64):
    return C.create_string_buffer(b + b"\0" * pad, len(b) + pad)


def compress(src, cap, accel=None):
    n = len(src)
    out = C.create_string_buffer(max(cap, 1) + 64)
    if accel is None:
        r = F("compress_default")(cbuf(src), out, n, cap)
    else:
        r = F("compress_fast")(cbuf(src), out, n, cap, accel)
    return r, out.raw[:max(r, 0)]


def decompress(comp, cap, partial_target=None):
    out = C.create_string_buffer(cap + 64)
    if partial_target is None:
        r = F("decompress_safe")(cbuf(comp), out, len(comp), cap)
    else:
        r = F("decompress_safe_partial")(cbuf(comp), out, len(comp), partial_target, cap)
    return r, out.raw[:max(r, 0)]


def dec_case(name, comp, cap, rng=None, partial=True):
    r, out = decompress(comp, cap)
    case = {"name": name, "comp_b64": base64.b64encode(comp).decode(), "cap": cap, "ret": r}
    if r > 0:
        case["out_sha256"] = I.sha(out)
    # offset-0 streams write bytes that depend on prior dst contents
    case["has_offset0"] = has_offset0(comp)
    if partial:
        tgt = (rng.randrange(0, cap + 8) if rng else cap // 2)
        pr, pout = decompress(comp, cap, tgt)
        case["partial"] = {"target": tgt, "ret": pr}
        if pr > 0:
            case["partial"]["out_sha256"] = I.sha(pout)
    return case


def has_offset0(comp):
    """Walk the token chain leniently; True if any match offset is 0."""
    ip, n = 0, len(comp)
    while ip < n:
        tok = comp[ip]; ip += 1
        ln = tok >> 4
        if ln == 15:
            while ip < n:
                s = comp[ip]; ip += 1; ln += s
                if s != 255:
                    break
        ip += ln
        if ip + 2 > n:
            return False
        if comp[ip] == 0 and comp[ip + 1] == 0:
            return True
        ip += 2
        if tok & 15 == 15:
            while ip < n:
                s = comp[ip]; ip += 1
                if s != 255:
                    break
    return False


def main():
    rng = random.Random(20261015)
    fx = {"generator": "tests/golden/gen_golden.py", "reference": "src/ape_lz4.c (LZ4 v1.7.1)",
          "version": F("versionNumber")(), "sizeofState": F("sizeofState")(),
          "encode": [], "decode": [], "stream": []}
    # 1. encode KATs (App. D.1)
    for content in I.ENC_CONTENTS:
        for n in I.ENC_SIZES:
            src = I.make(content, n)
            bound = F("compressBound")(n)
            r, comp = compress(src, bound)
            e = {"content": content, "n": n, "in_sha256": I.sha(src), "bound": bound,
                 "clen": r, "comp": enc_blob(comp)}
            # limited-output variants: exact size fits; one byte short fails (0)
            e["limited"] = []
            for cap in sorted({r, r - 1, max(r - 17, 0), bound - 1}):
                if cap < 0:
                    continue
                lr, lcomp = compress(src, cap)
                e["limited"].append({"cap": cap, "ret": lr, "sha256": I.sha(lcomp)})
            e["accel"] = []
            for acc in (2, 9):
                ar, acomp = compress(src, bound, acc)
                e["accel"].append({"accel": acc, "ret": ar, "sha256": I.sha(acomp)})
            fx["encode"].append(e)
            # round-trip decode KATs at cap = n, n - 1, n + 7
            if n <= 8192:
                for cap in sorted({n, max(n - 1, 0), n + 7}):
                    case = dec_case("rt_%s_%d_cap%d" % (content, n, cap), comp, cap, rng)
                    # decompress_fast (:1489) with originalSize = cap <= n: the reference
                    # stays inside the stream (a larger size would read past it)
                    if cap <= n:
                        fo = C.create_string_buffer(max(cap, 1) + 64)
                        fr = F("decompress_fast")(cbuf(comp), fo, cap)
                        case["fast"] = {"osize": cap, "ret": fr}
                        if fr > 0:
                            case["fast"]["out_sha256"] = I.sha(fo.raw[:cap])
                    fx["decode"].append(case)
    # 2. crafted malformed streams (App. D.2)
    crafted = {
        "empty_src_cap8_tok00": (b"", 8),
        "cap0_single_zero": (b"\x00", 0),
        "cap0_single_nonzero": (b"\x10", 0),
        "cap0_two_bytes": (b"\x00\x00", 0),
        "truncated_token_lit15": (b"\xf0", 64),
        "truncated_length_chain": (b"\xf0\xff\xff", 64),
        "offset_beyond_output": (b"\x40abcd\x10\x00" + b"\x50hello", 64),
        "offset_zero": (b"\x40abcd\x00\x00" + b"\x50hello", 64),
        "match_into_last5": (b"\x40abcd\x04\x00" + b"\x30xyz", 12),
        "final_literals_short": (b"\x50abcd", 64),
        "final_literals_long": (b"\x30abcdef", 64),
        "valid_13": (b"\x40abcd\x04\x00\x50hello", 64),
        "valid_13_cap13": (b"\x40abcd\x04\x00\x50hello", 13),
        "valid_13_cap17": (b"\x40abcd\x04\x00\x50hello", 17),
        "match_len_chain_trunc": (b"\x4fabcd\x04\x00\xff\xff", 600),
        "lit_only_exact": (b"\x20hi", 2),
        "lit_only_cap1": (b"\x20hi", 1),
        "overlap_offset1_long": (b"\x1fA\x01\x00\xff\x10" + b"\x50ZZZZZ", 1024),
        "overlap_offset3": (b"\x3fABC\x03\x00\x20" + b"\x50WXYZQ", 256),
    }
    for name, (comp, cap) in crafted.items():
        fx["decode"].append(dec_case("crafted_" + name, comp, cap, rng))
    # 3. mutated valid streams (fuzz KATs: return-code parity on malformed input)
    for k in range(400):
        content = rng.choice(["comp", "text", "rand", "period3", "zeros"])
        n = rng.choice([64, 300, 1000, 4096, 8192])
        src = I.make(content, n, seed=k)
        _, comp = compress(src, F("compressBound")(n))
        c = bytearray(comp)
        for _ in range(rng.randrange(1, 4)):
            if c:
                c[rng.randrange(len(c))] = rng.randrange(256)
        if rng.random() < 0.25:
            c = c[: rng.randrange(len(c) + 1)]
        cap = rng.choice([n, n - 1, n + rng.randrange(64), rng.randrange(n + 1)])
        fx["decode"].append(dec_case("mut_%03d_%s_%d" % (k, content, n), bytes(c), max(cap, 0),
                                     rng))
    # 4. socket-style stream KATs (App. D.3): 8 KiB chunks, saveDict after each message
    for si, content in enumerate(["comp", "text", "rand"]):
        msgs = [I.make(content, 3 * 8192 + 1000, seed=si * 10 + m) for m in range(3)]
        st = C.c_void_p(F("createStream")())
        dictbuf = C.create_string_buffer(65536)
        frames = []
        keep = []
        for msg in msgs:
            mb = cbuf(msg)
            keep.append(mb)
            pos = 0
            while pos < len(msg):
                ln = min(8192, len(msg) - pos)
                ob = C.create_string_buffer(8240 + 64)
                r = F("compress_fast_continue")(st, C.byref(mb, pos), ob, ln, 8240, 1)
                frames.append(ob.raw[:r])
                pos += ln
            F("saveDict")(st, dictbuf, 65536)
        # RX replay: decompress_safe_continue into a 64 KiB ring with setStreamDecode
        ds = C.c_void_p(F("createStreamDecode")())
        ring = C.create_string_buffer(65536)
        rp, rets, plain = 0, [], b""
        for fr in frames:
            tmp = C.create_string_buffer(8192 + 64)
            r = F("decompress_safe_continue")(ds, cbuf(fr), tmp, len(fr), 8192)
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
            F("setStreamDecode")(ds, ring, rp)
        fx["stream"].append({"content": content, "msg_len": 3 * 8192 + 1000, "seeds":
                             [si * 10 + m for m in range(3)],
                             "frames_b64": [base64.b64encode(f).decode() for f in frames],
                             "dec_rets": rets, "plain_sha256": I.sha(plain),
                             "plain_ok": plain == b"".join(msgs)})
    # 5. benchmark-size decode KATs (pin 64 KiB decode parity on reference
    #    output, not only on the restatement): BASELINE config 3 blocks (App. C gen_comp,
    #    65536 B) and config 2 blocks (gen_rand, 4096 B), compressed by the reference
    brng = random.Random(20261016)
    for bid in (0, 1, 777, 65535, 524287, 1048575):
        src = I.synth_comp(65536, bid)
        _, comp = compress(src, F("compressBound")(65536))
        for cap in (65536, 65535):
            fx["decode"].append(dec_case("bench_comp64k_%d_cap%d" % (bid, cap), comp, cap, brng))
    for bid in (0, 1, 4242, 262143):
        src = I.synth_rand(4096, bid)
        _, comp = compress(src, F("compressBound")(4096))
        assert len(comp) == 4114
        for cap in (4096, 4095):
            fx["decode"].append(dec_case("bench_rand4k_%d_cap%d" % (bid, cap), comp, cap, brng))
    out = os.path.join(HERE, "lz4_golden.json")
    with open(out, "w") as f:
        json.dump(fx, f, separators=(",", ":"))
    print("wrote", out, os.path.getsize(out), "bytes;", len(fx["encode"]), "encode,",
          len(fx["decode"]), "decode,", len(fx["stream"]), "stream KATs")


if __name__ == "__main__":
    main()
