"""Debug zd_k_fused on the C3 corpus: decode fused / two-launch / profiled and
compare each frame with the source."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zstd-decompressor_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from zstd_decompressor import _lib  # noqa: E402
from zstd_decompressor.batch import Plan  # noqa: E402

data, src, reps, meta, tgen = bench.make_corpus("c3", 100 << 20, 0x5EED, 3)
n = int(os.environ.get("NFR", "0"))
print("corpus", len(data), len(src), reps, flush=True)
d_src = torch.frombuffer(bytearray(data + bytes(64)), dtype=torch.uint8).cuda()
ref = np.frombuffer(src, dtype=np.uint8)
cases = {"all": (("fused", 0, False), ("nofuse", _lib.F_NO_FUSE, False), ("fused-prof", 0, True)),
         "plain": (("nofuse", _lib.F_NO_FUSE, False), ("nofuse-prof", _lib.F_NO_FUSE, True))}
for name, flags, prof in cases[os.environ.get("CASES", "all")]:
    plan = Plan(data, flags=flags)
    d_dst = torch.zeros(plan.info.out_bytes + 64, dtype=torch.uint8, device="cuda")
    if prof:
        plan.set_profiling(True)
    for it in range(2):
        plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), plan.info.out_bytes)
        torch.cuda.synchronize()
        st, total, sts, lens, first = plan.results(d_dst.data_ptr())
        out = d_dst[:total].cpu().numpy()
        bad = np.nonzero(out[: len(ref)] != ref[: len(out)])[0] if total == len(ref) else None
        nb = None if bad is None else len(bad)
        msg = f"{name} iter {it}: st {st} total {total} bad bytes {nb}"
        if nb:
            fr = sorted(set((bad // (128 << 10)).tolist()))
            msg += f" frames {fr[:12]} (of {len(fr)}), first byte {bad[0]}"
        print(msg, flush=True)
    plan.close()
