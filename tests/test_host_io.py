"""The drop-in's host-in / host-out path and process plumbing, on the GPU:
zd_plan_decompress (the INTEGRATION.md decompress(): pinned chunks, plan-owned
device buffers, io_*_ns phase times), the one-HIP-runtime rule of _lib when
libzd is loaded before torch, and plans destroyed on another device than
their own."""
import ctypes as C
import os
import subprocess
import sys

import pytest

from corpus import gen
from oracle import oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_decompress_large_repeated():
    """A plan reused three times on a 96 MB many-frame input (several pinned
    chunks each way, an odd tail chunk), and on a frame whose output is
    shorter than dst: bit-exact every time, phase times reported."""
    from zstd_decompressor import _lib
    from zstd_decompressor.batch import Plan
    src = gen.text((96 << 20) + 12345, seed=44)
    data = gen.frames(src, 128 << 10, 3)
    plan = Plan(data)
    cap = plan.info.out_bytes
    assert cap == len(src)
    buf = (C.c_uint8 * (cap + 7))()
    n = C.c_size_t()
    p, nb, keep = _lib.buf(data)
    for _ in range(3):
        C.memset(buf, 0, cap)
        st = _lib.lib().zd_plan_decompress(plan._h, p, nb, buf, cap + 7, C.byref(n))
        assert st == 0 and n.value == len(src)
        assert bytes(buf[: n.value]) == src
        info = _lib.PlanInfo()
        _lib.check(_lib.lib().zd_plan_info_get(plan._h, C.byref(info)))
        assert info.io_h2d_ns > 0 and info.io_decode_ns > 0 and info.io_d2h_ns > 0
    # dst too small: DstTooSmall, the bytes that fit copied
    small = (C.c_uint8 * 1000)()
    st = _lib.lib().zd_plan_decompress(plan._h, p, nb, small, 1000, C.byref(n))
    assert st == _lib.DST_TOO_SMALL and n.value == len(src) and bytes(small) == src[:1000]
    plan.close()


def test_decompress_matches_oracle_on_resources(resources):
    from zstd_decompressor.batch import decompress_status
    for name, data in resources.items():
        assert decompress_status(data) == oracle.decompress_status(data), name


_LIB_FIRST = r"""
import sys
sys.path[:0] = [{root!r}, {pkg!r}]
from zstd_decompressor import _lib
L = _lib.lib()                      # libzd first: torch's runtime goes in by path
assert "torch" not in sys.modules
import torch                        # then torch, sharing that runtime
from zstd_decompressor.batch import Plan
data = open({path!r}, "rb").read()
plan = Plan(data)
dev = torch.device("cuda", 0)
d_src = torch.zeros(len(data) + 64, dtype=torch.uint8, device=dev)
d_src[: len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
d_dst = torch.zeros(plan.info.out_bytes + 64, dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), plan.info.out_bytes, s)
st, total, _, _, _ = plan.results(d_dst.data_ptr(), s)
sys.stdout.buffer.write(bytes([st & 255]) + bytes(d_dst[:total].cpu().numpy().tobytes()))
"""


def test_libzd_loaded_before_torch():
    """_lib loads torch's HIP runtime by path before libzd without importing
    torch; a later `import torch` shares it, so torch tensors' device pointers
    work in libzd."""
    path = os.path.join(ROOT, "tests", "golden", "resources", "moby-dick.txt.zst")
    code = _LIB_FIRST.format(root=ROOT, pkg=os.path.join(ROOT, "zstd-decompressor_amd"), path=path)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=300)
    assert out.returncode == 0, out.stderr.decode()[-2000:]
    assert out.stdout[0] == 0
    assert out.stdout[1:] == oracle.decompress(open(path, "rb").read())


def test_plan_destroyed_on_another_device():
    """A plan made on GPU 0 and destroyed while GPU 1 is current returns its
    workspace and aux stream to GPU 0's cache: the next plan
    on GPU 1 decodes correctly on its own memory and stream."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    from zstd_decompressor.batch import Plan
    src = gen.text(4 << 20, seed=45)
    data = gen.frames(src, 128 << 10, 3)
    torch.cuda.set_device(0)
    p0 = Plan(data)
    torch.cuda.set_device(1)
    p0.close()
    p1 = Plan(data)
    dev = torch.device("cuda", 1)
    d_src = torch.zeros(len(data) + 64, dtype=torch.uint8, device=dev)
    d_src[: len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    d_dst = torch.zeros(len(src) + 64, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    p1.decode_async(d_src.data_ptr(), d_dst.data_ptr(), len(src), s)
    st, total, _, _, _ = p1.results(d_dst.data_ptr(), s)
    assert st == 0 and bytes(d_dst[:total].cpu().numpy().tobytes()) == src
    p1.close()
    torch.cuda.set_device(0)
