"""Host unit test of the arithmetic the kernels share with the host
(zd_common.h): sequence-code baselines, 16-bit FSE entries, packed sequence
records, K3 chain entries and K4's repeat-offset batch walk vs decode_offset
(decoding_context.rs:50-75).
Compiled with g++ from tests/native/test_common.cpp; no GPU needed."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_common_arithmetic(tmp_path):
    exe = tmp_path / "test_common"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-Wall", "-o", str(exe),
                           os.path.join(ROOT, "tests", "native", "test_common.cpp")])
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("ok")
