"""Memory safety of the product's host codec (SURVEY.md App. D item 4, section 5 sanitizers).

The host codec (libapenetwork_amd/csrc/ape_lz4_host.c) is what every one-shot and stream call
of ape_lz4.h runs by default -- what ape_socket.c:832-857 / :1386-1421 would run on network
input.  tests/fuzz/fuzz_host_codec.c compiles it with ASan + UBSan and compares it, return
value and bytes, against the reference compiled from its own source (oracle/_ref) on mutated
blocks and streams; exact-size buffers make any read past src or write past dst a report.
"""
import ctypes as C
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "libape_lz4_ref.so")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref not built (reference sources absent)")
    out = tmp_path_factory.mktemp("fuzz")
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "fuzz"), "OUT=%s" % out],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    exe = os.path.join(out, "fuzz_host_codec")
    nm = subprocess.run(["nm", "-D", exe], capture_output=True, text=True).stdout
    assert "APE_LZ4_" not in nm, "product symbols exported: the reference could bind to them"
    return exe


@pytest.mark.parametrize("seed", [1, 7])
def test_host_codec_sanitized_fuzz_vs_reference(harness, seed):
    """~25k mutated cases per seed over every host entry point (decoders at random caps,
    targets and dictionaries; the 64 KiB-ring RX stream; compress_default / limitedOutput /
    fast / destSize; the 8 KiB-chunk TX stream with saveDict): no sanitizer report, every
    return value and every produced byte equal to the reference's."""
    env = dict(os.environ, APE_REF_LIB=REF, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([harness, "25000", str(seed), "120"], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-4000:])
    assert "0 mismatches" in r.stdout, r.stdout


def test_final_token_literal_run_reads_nothing_past_src():
    """`[0xFF]`, csize 1 -- a token with literal length 15 as the last input byte.
    The reference reads src[1] (ref src/ape_lz4.c:1330-1337); the product returns the same
    -3 without touching it.  The byte sits at the end of a page followed by a PROT_NONE page,
    so any read past src faults (run in a child process)."""
    code = textwrap.dedent("""
        import ctypes as C, mmap, sys
        sys.path.insert(0, %r)
        import libapenetwork_amd as amd
        L = amd.lib()
        libc = C.CDLL(None)
        libc.mmap.restype = C.c_void_p
        libc.mmap.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_long]
        libc.mprotect.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
        pg = mmap.PAGESIZE
        base = libc.mmap(None, 2 * pg, 3, 0x22, -1, 0)
        assert libc.mprotect(base + pg, pg, 0) == 0
        out = C.create_string_buffer(256)
        res = []
        for tok in (0xFF, 0xF0, 0xF5):
            C.memmove(base + pg - 1, bytes([tok]), 1)
            p = C.c_char_p(base + pg - 1)
            for cap in (64, 1, 255):
                res.append(L.APE_LZ4_decompress_safe(p, out, 1, cap))
                res.append(L.APE_LZ4_decompress_safe_partial(p, out, 1, 10, cap))
                res.append(L.APE_LZ4_decompress_safe_usingDict(p, out, 1, cap, out, 16))
        # a literal followed by such a token (fails earlier, at the first sequence's checks)
        C.memmove(base + pg - 3, b"\\x10a\\xf0", 3)
        res.append(L.APE_LZ4_decompress_safe(C.c_char_p(base + pg - 3), out, 3, 64))
        print(res)
    """ % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    res = eval(r.stdout.strip().splitlines()[-1])
    assert res[:-1] == [-3] * (len(res) - 1), res
    ref = C.CDLL(REF) if os.path.exists(REF) else None
    if ref is not None:   # the reference's own return on the same bytes (padded buffer)
        out = C.create_string_buffer(256)
        assert ref.APE_LZ4_decompress_safe(C.create_string_buffer(b"\xff" + b"\0" * 15), out,
                                           1, 64) == -3
        assert ref.APE_LZ4_decompress_safe(C.create_string_buffer(b"\x10a\xf0" + b"\0" * 13),
                                           out, 3, 64) == res[-1]
