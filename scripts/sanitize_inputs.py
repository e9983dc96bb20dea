"""Inputs for `make sanitize` (tests/native/fuzz_host.cpp): the reference's
resources and seeded libzstd corpora of every frame shape, one large enough
(> 4 MiB) for the parallel host walk.  usage: sanitize_inputs.py OUTDIR"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from corpus import gen, libzstd  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
res = os.path.join(ROOT, "tests", "golden", "resources")
for n in sorted(os.listdir(res)):
    shutil.copy(os.path.join(res, n), os.path.join(out, n))
files = {
    "frames_l3.zst": gen.frames(gen.text(2 << 20, seed=61), 128 << 10, 3),
    "multiblock_l19.zst": gen.frames(gen.text(1 << 20, seed=62), 1 << 20, 19),
    "binary_l1.zst": gen.frames(gen.binary(1 << 20, seed=63), 256 << 10, 1),
    "rawrle.zst": libzstd.compress(gen.binary(300 << 10, seed=64), 1) + libzstd.compress(bytes(500 << 10), 3),
    "parallel_walk.zst": gen.frames(gen.text(12 << 20, seed=65), 32 << 10, 1),
}
for n, d in files.items():
    with open(os.path.join(out, n), "wb") as f:
        f.write(d)
print(out)
