"""The host program without a GPU (CPU suite): the devices open on their own
thread while step 0 reads the first chunk, and a failure there ends the
process loudly before any output -- no CPU fallback, no hang on a reader
still holding the input."""
import os
import subprocess

import pytest

from tools.gen_synth import write

BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ccsx_amd", "bin", "ccsx")


def _gpu_visible():
    return os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK | os.W_OK)


@pytest.mark.skipif(not os.path.exists(BIN), reason="host program not built")
@pytest.mark.skipif(_gpu_visible(), reason="a GPU is visible")
@pytest.mark.parametrize("from_stdin", [False, True])
def test_cli_without_gpu_fails_loudly(tmp_path, from_stdin):
    fa = str(tmp_path / "in.fa")
    write(fa, 40, 1500, 7)
    out = str(tmp_path / "out.fa")
    if from_stdin:
        with open(fa, "rb") as f:
            r = subprocess.run([BIN, "-A", "-j", "2", "-", out], stdin=f, capture_output=True, timeout=120)
    else:
        r = subprocess.run([BIN, "-A", "-j", "2", fa, out], capture_output=True, timeout=120)
    assert r.returncode == 1
    assert b"no HIP device" in r.stderr
    assert os.path.getsize(out) == 0
