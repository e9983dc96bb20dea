"""The LDS write-ordering property the streaming executor's pass 0 relies on
(zd_kernels.hip k4_body, ZD_K4_OVS): when lanes of one wave's ds_write_b128 /
ds_write_b64 write overlapping byte-unaligned ranges, every byte ends up with
the value of the highest lane that wrote it.  tools/lds_order_check runs
random overlap patterns (sequence-length-like gaps, inactive lanes, four
waves per workgroup) and compares every byte with that rule."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_lds_write_order_highest_lane_wins():
    exe = os.path.join(ROOT, "tools", "lds_order_check")
    assert os.path.exists(exe), "build it: make -C zstd-decompressor_amd (tools/lds_order_check)"
    r = subprocess.run([exe, "2048", "128"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("ok"), r.stdout
