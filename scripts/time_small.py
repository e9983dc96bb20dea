"""Few-frames plans on one GPU: the reference's resources and single multi-block
frames, decoded through each executor (automatic / streaming K4 / K4J), warm,
median wall time of decode_async + results and the per-kernel event times.
usage: python scripts/time_small.py > gpurun_out/small.json"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zstd-decompressor_amd")]
import torch  # noqa: E402

from corpus import gen, libzstd  # noqa: E402
from zstd_decompressor import _lib  # noqa: E402
from zstd_decompressor.batch import Plan  # noqa: E402

dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
inputs = {
    "moby-dick": open(os.path.join(ROOT, "tests", "golden", "resources", "moby-dick.txt.zst"), "rb").read(),
    "text 1 MiB L3 (8 blocks)": libzstd.compress(gen.text(1 << 20, seed=5), 3),
    "text 8 MiB L3 (64 blocks)": libzstd.compress(gen.text(8 << 20, seed=6), 3),
    "xml 4 MiB L19": libzstd.compress(gen.xml(4 << 20, seed=7), 19),
}
res = {}
for name, data in inputs.items():
    d_src = torch.zeros(len(data) + 64, dtype=torch.uint8, device=dev)
    d_src[: len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    for mode, flags in (("auto", 0), ("K4", _lib.F_FRAME_SERIAL), ("K4J", _lib.F_BLOCK_PARALLEL)):
        plan = Plan(data, False, flags)
        n = plan.info.out_bytes
        d_dst = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
        ts = []
        for it in range(7):
            torch.cuda.synchronize(dev)
            t0 = time.time()
            plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), n, s)
            st, total, _, _, _ = plan.results(d_dst.data_ptr(), s)
            ts.append(time.time() - t0)
        plan.set_profiling(True)
        plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), n, s)
        kt = plan.kernel_times()
        plan.results(d_dst.data_ptr(), s)
        plan.close()
        ts.sort()
        res[f"{name} / {mode}"] = {"status": st, "bytes": total, "ms": round(ts[3] * 1e3, 3),
                                   "MBps": round(total / ts[3] / 1e6, 1), "kernel_ms": {k: round(v, 3) for k, v in kt.items()}}
        print(name, mode, res[f"{name} / {mode}"], file=sys.stderr, flush=True)
print(json.dumps(res))
