"""The host walk (zd_host.cpp plan_index) on CPU: large inputs are cut into
byte ranges whose threads each index the chain of frames from the first
frame magic in their range; the chains are kept from the frame that starts
where the kept frames before them end.  Its result must equal the serial
walk's (one thread, ZD_WALK_THREADS=1) on every input, and its status the
oracle's (FrameIterator + the CLI loop, src/main.rs:43-53), including magic
numbers planted inside compressed data, frames longer than a range, skippable
frames, corruptions and truncations.
"""
import json
import os
import random
import subprocess
import sys

from corpus import gen, libzstd
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAGIC = (0xFD2FB528).to_bytes(4, "little")

_WALK = r"""
import json, sys
sys.path[:0] = [{root!r}, {pkg!r}]
from zstd_decompressor.batch import frames_index
data = open(sys.argv[1], "rb").read()
fr, bl, st, cons = frames_index(data)
print(json.dumps([[(f["src_offset"], f["src_size"], f["num_blocks"]) for f in fr],
                  [(b["src_offset"], b["block_size"], b["type"]) for b in bl], st, cons]))
"""


def _walk(path, threads):
    code = _WALK.format(root=ROOT, pkg=os.path.join(ROOT, "zstd-decompressor_amd"))
    env = dict(os.environ, ZD_WALK_THREADS=str(threads))
    out = subprocess.run([sys.executable, "-c", code, path], env=env, check=True, capture_output=True, text=True)
    return json.loads(out.stdout)


def _inputs():
    r = random.Random(77)
    frames = gen.frames(gen.text(12 << 20, seed=21), 32 << 10, 1)         # ~6 MB, ~400 frames: 6 ranges
    yield "intact", frames
    big = libzstd.compress(gen.text(5 << 20, seed=22), 3)                  # one frame over several ranges
    yield "big frame between", frames[: len(frames) // 2] + big + frames
    skip = (0x184D2A55).to_bytes(4, "little") + (40000).to_bytes(4, "little") + bytes(40000)
    yield "skippable", frames + skip + frames
    d = bytearray(frames * 2)
    for _ in range(200):                                                   # magic numbers inside data
        p = r.randrange(len(d) - 4)
        d[p:p + 4] = MAGIC
    yield "planted magic", bytes(d)
    for i in range(6):
        d = bytearray(frames * 2)
        for _ in range(r.randrange(1, 4)):
            d[r.randrange(len(d))] = r.randrange(256)
        if i % 2:
            d = d[: r.randrange(len(d) // 2, len(d))]
        yield f"corrupt {i}", bytes(d)


def test_parallel_walk_equals_serial(tmp_path):
    for name, data in _inputs():
        assert len(data) >= 4 << 20, name                                   # the parallel walk's threshold
        path = str(tmp_path / "in.zst")
        open(path, "wb").write(data)
        serial = _walk(path, 1)
        par = _walk(path, 8)
        assert par == serial, name
        # the status of the walk is the oracle's unless a failure lies inside a
        # block's entropy-coded content (found on the GPU, after the walk)
        ost, _ = oracle.decompress_status(data)
        if serial[2] != 0:
            assert ost == serial[2], (name, ost, serial[2])


def false_frame_input(threads=None, cut=None):
    """~6 MB of 32 KiB frames with a complete fake frame (magic, header, one
    raw block of 16 bytes) planted inside compressed data as the first magic
    number after byte `cut` (default: range 1 of the host walk on `threads`
    threads): the range's parallel walk indexes it, then fails on the next
    'frame' after it (two frames: not retried as a lone false magic).
    Returns (data, range size, planted offset)."""
    from zstd_decompressor.batch import frames_index
    frames = gen.frames(gen.text(12 << 20, seed=21), 32 << 10, 1)
    n = len(frames)
    if cut is None:
        T = min(threads, n >> 20)
        cut1 = n * 1 // T
    else:
        T, cut1 = n // cut, cut
    _, blocks, st, _ = frames_index(frames)
    assert st == 0
    fake = MAGIC + bytes([0x00, 0x00]) + ((16 << 3) | 1).to_bytes(3, "little") + bytes(range(16))
    for b in blocks:                      # the first compressed block content that holds it after cut1
        lo = max(b["src_offset"] + 64, cut1)
        if b["type"] == 2 and lo + len(fake) + 64 <= b["src_offset"] + b["block_size"]:
            d = bytearray(frames)
            d[lo:lo + len(fake)] = fake
            return bytes(d), n // T, lo
    raise AssertionError("no block to plant into")


def test_false_frame_costs_one_range(tmp_path):
    """A planted magic number that parses as one whole frame makes range 1's
    chain miss the true one.  The stitch walks on serially only until the
    chain meets a later range's (it used to walk the rest of the
    input serially): the serial bytes stay within about two ranges, and the
    frames equal the serial walk's."""
    data, rsize, at = false_frame_input(6)
    path = str(tmp_path / "in.zst")
    open(path, "wb").write(data)
    assert _walk(path, 6) == _walk(path, 1)
    code = _WALK.format(root=ROOT, pkg=os.path.join(ROOT, "zstd-decompressor_amd"))
    env = dict(os.environ, ZD_WALK_THREADS="6", ZD_PLAN_TIMES="1")
    out = subprocess.run([sys.executable, "-c", code, path], env=env, check=True, capture_output=True, text=True)
    line = [x for x in out.stderr.splitlines() if x.startswith("zd walk:")][0]
    serial = int(line.split("serial ")[1].split()[0])
    assert 0 < serial <= 2 * rsize, (serial, rsize, line)
    assert serial < len(data) - at - rsize        # far from the rest of the input
