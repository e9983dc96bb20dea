import os, sys, time
sys.path[:0] = ["/root/repo", "/root/repo/zstd-decompressor_amd"]
os.environ.setdefault("ZD_LIB_PATH", "zstd-decompressor_amd/lib/variants/libzd_walkprof.so")
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
