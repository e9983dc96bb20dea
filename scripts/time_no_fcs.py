"""Times a resident decode of 256 MiB of 128 KiB frames without
Frame_Content_Size (the staging layout + compaction path, zd_k_compact)
against the same frames with it; checks both bit-exact.
usage: python scripts/time_no_fcs.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zstd-decompressor_amd")]
import torch  # noqa: E402
from corpus import gen  # noqa: E402
from zstd_decompressor.batch import Plan  # noqa: E402

src = gen.text(256 << 20, seed=0x5EED)[: 256 << 20]
for fcs in (True, False):
    data = gen.frames(src, 128 << 10, 3, content_size=fcs)
    d_in = torch.empty(len(data) + 16, dtype=torch.uint8, device="cuda")
    d_in[: len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    plan = Plan(data)
    cap = max(plan.info.out_bytes, 1)
    d_out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    ts = []
    for it in range(6):
        torch.cuda.synchronize()
        t0 = time.time()
        plan.decode_async(d_in.data_ptr(), d_out.data_ptr(), cap)
        r = plan.results(d_out.data_ptr())
        torch.cuda.synchronize()
        ts.append(time.time() - t0)
    total = r[2] if isinstance(r, tuple) else None
    ok = bytes(d_out[: len(src)].cpu().numpy()) == src
    print("fcs", fcs, "bytes", len(data), "exact", plan.info.out_exact, "bit_exact", ok,
          "ms", [round(t * 1e3, 2) for t in ts], flush=True)
    plan.close()
