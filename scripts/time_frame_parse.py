"""Where Frame.parse's per-frame time goes (the reference's frame-by-frame API,
frame.rs:61-84): the host index, zd_plan_create, zd_plan_decompress and
zd_plan_destroy timed apart over the first frames of the C3 shape (100 MB,
763 frames of 128 KiB, zstd -3).  usage: python scripts/time_frame_parse.py [out.json]"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zstd-decompressor_amd")]

from corpus import gen  # noqa: E402
import zstd_decompressor as zd  # noqa: E402
from zstd_decompressor import _lib, ForwardByteParser, Frame  # noqa: E402
from zstd_decompressor.batch import Plan, run_plan  # noqa: E402

src = gen.text(100_000_000, seed=0x5EED)[:100_000_000]
data = gen.frames(src, 128 << 10, 3)
Frame.parse(ForwardByteParser(data)).decode()       # warm the runtime and caches

N = 40
p = ForwardByteParser(data)
t0 = time.perf_counter()
for _ in range(N):
    Frame.parse(p).decode()
t_parse = (time.perf_counter() - t0) / N

# the same frames, the plan steps apart
p = ForwardByteParser(data)
raws = []
for _ in range(N):
    f = Frame.parse(p)
    raws.append(f.inner._raw)
L = _lib.lib()
tc = td = tx = 0.0
for raw in raws:
    a = time.perf_counter()
    plan = Plan(raw)
    b = time.perf_counter()
    pp, n, keep = _lib.buf(raw)
    st, out = run_plan(plan, pp, n)
    c = time.perf_counter()
    plan.close()
    d = time.perf_counter()
    tc += b - a; td += c - b; tx += d - c
res = {"workload": "C3 frames (128 KiB, zstd -3), the first %d, host in / host out" % N,
       "frame_parse_decode_ms": round(t_parse * 1e3, 3),
       "plan_create_ms": round(tc * 1e3 / N, 3), "plan_decompress_ms": round(td * 1e3 / N, 3),
       "plan_destroy_ms": round(tx * 1e3 / N, 3)}
line = json.dumps(res)
print(line)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(line + "\n")
