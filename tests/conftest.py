import ctypes
import json
import os
import subprocess
import sys

import pytest

# torch first: its wheel carries its own HIP runtime, and loading /opt/rocm's (through
# libape_lz4_amd.so) before it leaves torch.cuda unavailable in that process (the
# library works either way).  Plumbing only: no test needs torch on CPU.
try:
    import torch  # noqa: F401
except ImportError:
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def _ensure(path, make_dir):
    if not os.path.exists(path):
        subprocess.run(["make", "-C", make_dir], check=True, capture_output=True)
    return path


@pytest.fixture(scope="session")
def oracle():
    """The CPU restatement (TEST INFRASTRUCTURE) -- the checker."""
    p = _ensure(os.path.join(ROOT, "oracle", "liblz4_oracle.so"), os.path.join(ROOT, "oracle"))
    L = ctypes.CDLL(p)
    for f in ("orc_createStream", "orc_createStreamDecode"):
        getattr(L, f).restype = ctypes.c_void_p
    return L


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "lz4_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def product():
    _ensure(os.path.join(ROOT, "libapenetwork_amd", "libape_lz4_amd.so"),
            os.path.join(ROOT, "libapenetwork_amd", "csrc"))
    import libapenetwork_amd as amd
    return amd


@pytest.fixture(autouse=True)
def _dst_canaries(request):
    """After every GPU test: nothing was written outside any alloc_out() slot."""
    yield
    if request.node.get_closest_marker("gpu") is not None:
        import gpuutil
        gpuutil.check_canaries()


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda is not available")
    return torch
