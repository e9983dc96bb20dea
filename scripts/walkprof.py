"""Device header walk vs host walk plan times on a 1 GiB C4-shaped input.
Per-range scan / walk cycles: build `make -C zstd-decompressor_amd variant
NAME=walkprof DEFS=-DZD_WALK_PROF` and run with
ZD_LIB_PATH=zstd-decompressor_amd/lib/variants/libzd_walkprof.so (and
ZD_PLAN_TIMES=1 for the planner phases)."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zstd-decompressor_amd")]
import torch
from corpus import gen
from zstd_decompressor.batch import Plan
src = gen.text(256 << 20, seed=5)
data = gen.frames(src, 128 << 10, 3) * 4
dev = torch.device("cuda", 0)
d = torch.empty(len(data) + 64, dtype=torch.uint8, device=dev)
d[:len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
torch.cuda.synchronize()
for i in range(2):
    t = time.time(); p = Plan.from_device(d.data_ptr(), len(data)); torch.cuda.synchronize()
    print("device plan ms", (time.time() - t) * 1e3, p.info.nframes, flush=True); p.close()
t = time.time(); p = Plan(data); print("host plan ms", (time.time() - t) * 1e3, flush=True)
