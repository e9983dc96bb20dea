"""The experimental frame-resident executor K4F (zd_k_execute_lds, DESIGN.md
§4) is routed by ZD_K4F=1, read once per process: the GPU parity suite runs
again in a child process with it on (frames up to 128 KiB take K4F).  The
child's progress goes to gpurun_out/k4f_suite.log as it runs (a GPU box
takes a command that stays silent for minutes to be hung)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_gpu_parity_suite_on_k4f():
    env = dict(os.environ, ZD_K4F="1")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    log = os.path.join(ROOT, "gpurun_out", "k4f_suite.log")
    with open(log, "w") as f:
        r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-v", "-m", "gpu", "-p", "no:cacheprovider",
                            os.path.join(ROOT, "tests", "test_gpu_parity.py")],
                           cwd=ROOT, env=env, stdout=f, stderr=subprocess.STDOUT, text=True, timeout=900)
    assert r.returncode == 0, open(log).read()[-3000:]
