"""The drop-in against the reference's own caller (CPU only).

oracle/ref_net.sh compiles the reference's socket stack -- every /root/reference/src/*.c except
ape_lz4.c, with gcc, against the reference's own headers -- and links it with
tests/c/ref_socket_lz4.c against libape_lz4_amd.so in place of the reference's ape_lz4.o.  The
driver runs one APE_socket pair over 127.0.0.1 with APE_socket_enable_lz4(TX|RX) on both ends
(ref src/ape_socket.c:105-141, :811-871, :1333-1467): 14 messages of 1 B .. 64 KiB, compressible
and random, sent by the client, checked and echoed by the server, checked by the client.
Skipped where the reference sources are absent (the GPU box); nothing from the reference is
committed or sent there (oracle/_ref/net is git- and gpurun-ignored)."""
import os
import socket
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF_SRC = os.environ.get("APE_REF_SRC", "/root/reference/src")
EXE = os.path.join(ROOT, "oracle", "_ref", "net", "ref_socket_lz4")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference sources absent")
def test_reference_socket_stack_on_product_library():
    b = subprocess.run(["bash", os.path.join(ROOT, "oracle", "ref_net.sh")], capture_output=True,
                       text=True, timeout=300)
    if b.returncode == 2:
        pytest.skip("reference socket stack unbuildable here: " + b.stdout.strip())
    assert b.returncode == 0, b.stdout + b.stderr
    # the codec symbols the reference's socket code calls resolve to the product library
    nm = subprocess.run(["nm", "-D", "--undefined-only", EXE], capture_output=True, text=True).stdout
    need = {"APE_LZ4_createStream", "APE_LZ4_createStreamDecode", "APE_LZ4_compress_fast_continue",
            "APE_LZ4_saveDict", "APE_LZ4_decompress_safe_continue", "APE_LZ4_setStreamDecode",
            "APE_LZ4_freeStream", "APE_LZ4_freeStreamDecode"}
    assert need <= {ln.split()[-1] for ln in nm.splitlines() if ln.strip()}
    ldd = subprocess.run(["ldd", EXE], capture_output=True, text=True).stdout
    assert os.path.join(ROOT, "libapenetwork_amd", "libape_lz4_amd.so") in ldd
    r = subprocess.run([EXE, str(_free_port())], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "14 messages" in r.stdout and "identical" in r.stdout
