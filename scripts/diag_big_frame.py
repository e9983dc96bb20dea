"""Diagnoses a single-frame decode past 2 GiB (tests/test_large_frames.py
test_single_frame_over_2GiB's input): where the GPU output first differs
from the source, and how many bytes differ, without pytest's diff."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zstd-decompressor_amd")]
import numpy as np  # noqa: E402
from corpus import gen, libzstd  # noqa: E402
from zstd_decompressor.batch import decompress_status  # noqa: E402

t0 = time.time()
gib = float(sys.argv[1]) if len(sys.argv) > 1 else 2.25
tile = np.frombuffer(gen.text(256 << 10, seed=10), dtype=np.uint8)
n = int(gib * (1 << 30)) // len(tile)
arr = np.tile(tile, n).reshape(n, len(tile))
arr[:, :4] = np.arange(n, dtype="<u4").view(np.uint8).reshape(n, 4)
src = arr.reshape(-1)
data = libzstd.compress(src.tobytes(), 1)
print("input", len(data), "output", src.size, round(time.time() - t0, 1), flush=True)
st, out = decompress_status(data)
print("status", st, "len", len(out), round(time.time() - t0, 1), flush=True)
g = np.frombuffer(out, dtype=np.uint8)
m = min(g.size, src.size)
bad = np.flatnonzero(g[:m] != src[:m])
print("differing bytes", bad.size, flush=True)
if bad.size:
    f = int(bad[0])
    print("first at", f, "block", f >> 17, "tile", f // len(tile), "last at", int(bad[-1]), flush=True)
    print("gpu", g[f:f + 32].tobytes(), flush=True)
    print("src", src[f:f + 32].tobytes(), flush=True)
    hist = np.bincount((bad >> 28).astype(np.int64))
    print("per 256 MiB", hist.tolist(), flush=True)
if len(sys.argv) > 2:                                # the same frame forced onto the streaming executor
    from zstd_decompressor import _lib
    from zstd_decompressor.batch import Plan
    t1 = time.time()
    p = Plan(data, False, _lib.F_FRAME_SERIAL)
    print("serial plan", round(time.time() - t1, 2), "out_bytes", p.info.out_bytes, flush=True)
    p.close()
    st, out = decompress_status(data, False, _lib.F_FRAME_SERIAL)
    print("serial status", st, "len", len(out), round(time.time() - t1, 2), flush=True)
