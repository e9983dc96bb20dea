"""Times the crate-mirror loop (src/main.rs:43-53: FrameIterator + Frame.decode
per frame) against decompress() on the C3 shape (100 MB, 763 frames of 128 KiB,
zstd -3), host in / host out; writes one JSON line.
usage: python scripts/time_frame_iterator.py [out.json]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zstd-decompressor_amd")]

from corpus import gen  # noqa: E402
import zstd_decompressor as zd  # noqa: E402
from zstd_decompressor import ForwardByteParser, Frame  # noqa: E402

src = gen.text(100_000_000, seed=0x5EED)[:100_000_000]
data = gen.frames(src, 128 << 10, 3)


def best(f, k=3):
    ts = []
    for _ in range(k):
        t0 = time.time()
        out = f()
        ts.append(time.time() - t0)
    return min(ts), out


t_dec, out1 = best(lambda: zd.decompress(data))
t_it, out2 = best(lambda: b"".join(f.decode() for f in ForwardByteParser(data).iter()))
n_frames = sum(1 for _ in ForwardByteParser(data).iter())


def one_by_one():
    p = ForwardByteParser(data)
    parts = []
    for _ in range(40):                      # the per-frame path, on the first 40 frames
        parts.append(Frame.parse(p).decode())
    return b"".join(parts)


t_one, _ = best(one_by_one, 1)
res = {"workload": "C3: 100,000,000 B, %d frames of 128 KiB, zstd -3, host in / host out" % n_frames,
       "decompress_ms": round(t_dec * 1e3, 1), "frame_iterator_ms": round(t_it * 1e3, 1),
       "ratio": round(t_it / t_dec, 2), "bit_exact": out1 == out2 == src,
       "frame_parse_per_frame_ms": round(t_one * 1e3 / 40, 2),
       "frame_parse_projected_all_ms": round(t_one * 1e3 / 40 * n_frames, 1)}
line = json.dumps(res)
print(line)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(line + "\n")
