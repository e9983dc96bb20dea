"""K1 phase cycles (ZD_K1_PROF variant): decode C3-shaped and C4-shaped plans
and print the summed s_memtime cycles per phase per K1 lane.
usage: ZD_LIB_PATH=.../libzd_k1prof.so python scripts/k1prof.py"""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zstd-decompressor_amd")]
import torch  # noqa: E402
from corpus import gen  # noqa: E402
from zstd_decompressor import _lib  # noqa: E402
from zstd_decompressor.batch import Plan  # noqa: E402

L = _lib.lib()
L.zd_debug_k1_prof.argtypes = [C.POINTER(C.c_uint64), C.c_int]
names = ["spread", "fse table", "ncount parse", "huf weights", "huf widths+holes", "huf LUT fill", "kernel (lane)", "lanes"]
for what, n in (("C3-shaped 763 frames", 763), ("8192 frames", 8192)):
    src = gen.text(min(n, 1024) * (128 << 10), seed=5)
    data = gen.frames(src, 128 << 10, 3)
    data = data * (n // min(n, 1024))
    plan = Plan(data)
    d_src = torch.frombuffer(bytearray(data + bytes(64)), dtype=torch.uint8).cuda()
    d_dst = torch.empty(plan.info.out_bytes + 64, dtype=torch.uint8, device="cuda")
    buf = (C.c_uint64 * 8)()
    for it in range(3):
        L.zd_debug_k1_prof(buf, 1)
        plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), d_dst.numel())
        torch.cuda.synchronize()
        L.zd_debug_k1_prof(buf, 0)
    lanes = max(buf[7], 1)
    print(what, {names[i]: round(buf[i] / lanes) for i in range(7)}, "lanes", buf[7])
