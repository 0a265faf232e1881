"""The opt-in segment-parallel encoder (APE_LZ4_ENCODER=seg, lz4_encode_seg.hip; DESIGN.md
3.1.2).  The library reads the variable once per process, so the checks run in one child
process (tests/seg_check.py): valid blocks decoded by the oracle and by the reference
library itself, limitedOutput, determinism and dst canaries on the encoder suite's inputs,
and the App. C ratio at least the reference's."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_segment_encoder_blocks_valid(cuda, product, oracle):
    env = dict(os.environ, APE_LZ4_ENCODER="seg")
    p = subprocess.run([sys.executable, os.path.join(HERE, "seg_check.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    r = json.loads(lines[-1])
    print("segment encoder:", r)
    assert p.returncode == 0 and r["nbad"] == 0, r
    assert r["ratio"] >= r["ref_ratio"], r
