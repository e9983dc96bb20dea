"""The experimental frame-resident executor K4F (zd_k_execute_lds, DESIGN.md
§4) is routed by ZD_K4F=1, read once per process: the GPU parity suite runs
again in a child process with it on (frames up to 128 KiB take K4F)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_gpu_parity_suite_on_k4f():
    env = dict(os.environ, ZD_K4F="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_parity.py")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
