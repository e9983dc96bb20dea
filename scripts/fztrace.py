"""zd_k_fused timeline on the C3 corpus (ZD_FZ_TRACE variant): per-frame
times (us) from the kernel's first start to tables ready, chain start,
chain end, K4's waits over and K4 end, plus K2's end.
usage: ZD_LIB_PATH=.../libzd_fztrace.so python scripts/fztrace.py"""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zstd-decompressor_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from zstd_decompressor import _lib  # noqa: E402
from zstd_decompressor.batch import Plan  # noqa: E402

L = _lib.lib()
L.zd_debug_fz_trace.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
data, src, reps, meta, tgen = bench.make_corpus("c3", 100 << 20, 0x5EED, 3)
plan = Plan(data)
nf = plan.info.nframes
d_src = torch.frombuffer(bytearray(data + bytes(64)), dtype=torch.uint8).cuda()
d_dst = torch.empty(plan.info.out_bytes + 64, dtype=torch.uint8, device="cuda")
buf = (C.c_uint64 * (1024 * 16))()
k2 = C.c_uint64()
names = ["start", "tables", "chain end", "K4 waits over", "K4 end", "chain start", "parsed", "built", "K4 start", "parse start"]
for it in range(4):
    plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), d_dst.numel())
    torch.cuda.synchronize()
    L.zd_debug_fz_trace(buf, C.byref(k2))
    t = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16)[:min(nf, 1024), :10].astype(np.int64)
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0                     # s_memrealtime: 100 MHz
    row = {names[i]: (round(float(np.median(us[:, i])), 1), round(float(us[:, i].max()), 1)) for i in range(10)}
    k2us = (int(k2.value) - t0) / 100.0
    lag = us[:, 4] - us[:, 2]
    print(f"iter {it}: (median, max) us {row}; K2 end {k2us:.1f}; K4 end - chain end median {np.median(lag):.1f} max {lag.max():.1f}",
          flush=True)
