"""Writes test_parallel_host_walk's 24 corrupted inputs (tests/test_gpu_parity.py)
to a directory, for tools/decode_file."""
import os
import random
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [root, os.path.join(root, "zstd-decompressor_amd"), os.path.join(root, "tests")]
from corpus import gen  # noqa: E402
from zstd_decompressor.batch import frames_index  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
src = gen.text(1024 * (16 << 10), seed=31)
data = gen.frames(src, 16 << 10, 1)
frames = frames_index(data)[0]
r = random.Random(9)
for it in range(24):
    d = bytearray(data)
    k = [63, 64, 127, 128, 255, 256, 511, 512, 700, 1000][it % 10] + r.randrange(-2, 3)
    f = frames[max(0, min(k, 1023))]
    if it % 3 == 0:
        d[f["src_offset"] + 6 + r.randrange(3)] ^= 1 << r.randrange(8)
    else:
        d[f["src_offset"] + r.randrange(f["src_size"])] = r.randrange(256)
    if it % 8 == 7:
        d = d[: f["src_offset"] + r.randrange(f["src_size"])]
    with open(os.path.join(out, f"pw_{it:02d}.zst"), "wb") as fh:
        fh.write(bytes(d))
