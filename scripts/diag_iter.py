"""Progress-printing run of the frame-iterator cases (diagnostics on the GPU box)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zstd-decompressor_amd"), os.path.join(ROOT, "tests")]
import test_frame_iterator as T
from zstd_decompressor import ForwardByteParser, Frame, ZdError
from zstd_decompressor.frame import FrameIterator
t0 = time.time()
cases = T._cases()
print("cases ready", round(time.time() - t0, 1), flush=True)
for name, data in cases.items():
    for batched in (True, False):
        p = ForwardByteParser(data)
        it = FrameIterator(p)
        k = 0
        while not p.is_empty() and k < 50:
            t1 = time.time()
            try:
                f = next(it) if batched else Frame.parse(p)
            except ZdError as e:
                print(name, batched, k, "parse error", e.code, flush=True)
                break
            try:
                out = f.decode()
                print(name, batched, k, "ok", len(out), round(time.time() - t1, 3), p._pos, flush=True)
            except ZdError as e:
                print(name, batched, k, "decode error", e.code, round(time.time() - t1, 3), flush=True)
            k += 1
print("done", round(time.time() - t0, 1), flush=True)
