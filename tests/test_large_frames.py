"""Single frames of many blocks: the block-parallel executor K4J (pointer
jumping, zd_kernels.hip KJ1-KJ4) against the oracle and the streaming
per-frame executor, and frames above 128 MiB.

The reference decodes any frame whose window is at most 8 MiB
(frame.rs:44,167-169,201-206), with the whole frame as history
(decoding_context.rs:29-47, block.rs:90-96).  A stock `zstd` run over a big
file writes exactly one such frame (libzstd level 3: windowLog 21), so the
shapes here are `zstd -3 enwik8` (100 MB, 763 blocks) and a frame past the
128 MiB the GPU path used to refuse.  Same output and the same reference
error variant as the oracle; both executors (plan flags ZD_F_BLOCK_PARALLEL /
ZD_F_FRAME_SERIAL) on the same bytes.
"""
import random

import pytest

from corpus import gen, libzstd
from oracle import oracle

pytestmark = pytest.mark.gpu

OUT_OF_DOMAIN = -91


def _gpu(data, flags=0):
    from zstd_decompressor.batch import decompress_status
    return decompress_status(data, False, flags)


def _flags():
    from zstd_decompressor import _lib
    return _lib.F_BLOCK_PARALLEL, _lib.F_FRAME_SERIAL


def _parity(data, flags, what):
    ost, oout = oracle.decompress_status(data, False)
    gst, gout = _gpu(data, flags)
    assert gst != OUT_OF_DOMAIN, f"{what}: out of the GPU path's domain (oracle status {ost})"
    if ost == 0:
        assert gst == 0, f"{what}: oracle ok, gpu status {gst}"
        assert gout == oout, f"{what}: output differs ({len(gout)} vs {len(oout)} bytes)"
    else:
        assert gst == ost, f"{what}: oracle status {ost}, gpu status {gst}"
        assert gout == oout, f"{what}: partial output differs"
    return ost, gst


@pytest.mark.parametrize("kind", ["text", "xml", "binary"])
@pytest.mark.parametrize("level", [1, 9, 19])
def test_block_parallel_multi_block_frames(kind, level):
    """C5-shaped frames (1 MiB, 8 blocks: Treeless literals, Repeat tables,
    repeat offsets and matches across blocks) through K4J, forced."""
    bp, fs = _flags()
    n = (2 << 20) if level < 19 else (1 << 20)
    src = {"text": gen.text, "xml": gen.xml, "binary": gen.binary}[kind](n, seed=40 + level)
    data = gen.frames(src, 1 << 20, level)
    ost, _ = _parity(data, bp, f"K4J {kind} L{level}")
    assert ost == 0
    assert _gpu(data, fs) == (0, src)


def test_block_parallel_small_and_raw_rle_frames(kat):
    """Every frame through K4J: the reference's KAT frames, tiny frames, raw and
    RLE blocks between compressed ones (C2), checksums, period-1/2 matches."""
    bp, _ = _flags()
    for c in kat["frames"]:
        _parity(bytes(c["data"]), bp, c["src"])
    for n in (1, 3, 17, 1000, 70000):
        src = bytes(random.Random(n).randrange(256) for _ in range(n))
        _parity(libzstd.compress(src, 3), bp, f"tiny {n}")
    _parity(libzstd.compress(b"a" * 300000, 3), bp, "rle")
    _parity(libzstd.compress(b"ab" * 300000, 19), bp, "period-2")
    _parity(gen.c2_raw_rle(4 << 20), bp, "c2 raw/rle")
    src = gen.text(600_000, seed=7)
    _parity(gen.frames(src, 300_000, 3, checksum=True), bp, "checksum")


def test_block_parallel_corrupted_inputs():
    """Corruptions of multi-block frames through K4J: the first failing
    sequence of the frame decides the error, as in the reference's in-order
    decode (the blocks after it ran in parallel and must not change that)."""
    bp, _ = _flags()
    r = random.Random(4321)
    base = gen.frames(gen.text(3 << 20, seed=13), 1 << 20, 9) + gen.frames(gen.binary(1 << 20, seed=14), 1 << 20, 19)
    stats = {"ok": 0, "err": 0}
    for it in range(150):
        d = bytearray(base)
        for _ in range(r.randrange(1, 4)):
            d[r.randrange(len(d))] = r.randrange(256)
        if r.random() < 0.15:
            d = d[: r.randrange(len(d))]
        ost, gst = _parity(bytes(d), bp, f"K4J corrupt #{it}")
        stats["ok" if ost == 0 else "err"] += 1
    assert stats["ok"] and stats["err"], stats


def test_single_frame_enwik8_shape():
    """`zstd -3` of a 100,000,000-byte enwik-style text: one frame, 763
    blocks, windowLog 21 (BASELINE.json configs[2] as a single file)."""
    from zstd_decompressor.batch import frames_index
    src = gen.text(100_000_000, seed=8)
    data = libzstd.compress(src, 3)
    frames, blocks, st, _ = frames_index(data)
    assert st == 0 and len(frames) == 1 and len(blocks) > 700
    assert oracle.decompress(data) == src
    gst, gout = _gpu(data)                            # automatic: K4J
    assert gst == 0 and gout == src


def test_single_frame_over_128MiB():
    """A single libzstd frame of 160 MiB (windowLog 21): decoded by K4J
    (automatic) and by the streaming executor (forced; int32 positions reach
    2 GiB), both bit-exact against the source and the oracle."""
    _, fs = _flags()
    src = gen.text(160 << 20, seed=9)
    data = libzstd.compress(src, 3)
    assert oracle.decompress(data) == src
    assert _gpu(data) == (0, src)
    assert _gpu(data, fs) == (0, src)


def test_single_frame_over_2GiB():
    """A single libzstd frame of 2.25 GiB (18,432 blocks): K4J's state words
    are distances, so frame positions past 2^31 decode (the streaming
    executor's int32 positions do not reach: forced onto it, the frame is out
    of the GPU path's domain).  The source is a 256 KiB text tile repeated
    with a counter stamped into each copy, so every tile copies the one
    before it: pointer chains as long as the frame has tiles, resolved by the
    rounds' doubling.  Checked against the source bytes (the oracle would
    take minutes at this size; the round trip is the property)."""
    import numpy as np
    _, fs = _flags()
    tile = np.frombuffer(gen.text(256 << 10, seed=10), dtype=np.uint8)
    n = 9 * (1 << 30) // (4 * len(tile))             # 2.25 GiB
    arr = np.tile(tile, n).reshape(n, len(tile))
    arr[:, :4] = np.arange(n, dtype="<u4").view(np.uint8).reshape(n, 4)
    src = arr.tobytes()
    del arr
    assert len(src) == (1 << 31) + (1 << 28)
    data = libzstd.compress(src, 1)
    from zstd_decompressor.batch import frames_index
    frames, blocks, st, _ = frames_index(data)
    assert st == 0 and len(frames) == 1 and len(blocks) >= len(src) // (128 << 10)
    gst, gout = _gpu(data)                            # automatic: K4J (past the streaming K4's positions)
    assert gst == 0 and len(gout) == len(src)
    assert gout == src
    del gout
    assert _gpu(data, fs)[0] == OUT_OF_DOMAIN


_UNCONVERGED = r"""
import sys
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/zstd-decompressor_amd"]
from corpus import gen, libzstd
from zstd_decompressor import _lib
from zstd_decompressor.batch import Plan, run_plan
tile = gen.text(4096, seed=15)
src = b"".join(bytes([i & 255]) + tile for i in range(1200))      # every tile copies the one before
for s in (src, gen.text(3_000_000, seed=16)):
    data = libzstd.compress(s, 3)
    p = Plan(data, False, _lib.F_BLOCK_PARALLEL | _lib.F_J_ONE_ROUND)
    pp, n, keep = _lib.buf(data)
    st, out = run_plan(p, pp, n)
    print(st, int(out == s), p.refresh_info().replans, flush=True)
    p.close()
"""


def test_block_parallel_unconverged_replans(tmp_path):
    """K4J with its pointer jumping cut to one round of one hop (the plan's
    test switch ZD_F_J_ONE_ROUND: the rounds' last sweep finds pending
    pieces): the frame keys LS_JROUNDS and zd_plan_decompress plans it again
    on the streaming executor -- same bytes, one re-plan.  In a child
    process."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "unconverged.py"
    script.write_text(_UNCONVERGED)
    env = dict(os.environ)
    r = subprocess.run([sys.executable, str(script), root], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l.split() for l in r.stdout.strip().splitlines()]
    assert len(lines) == 2, r.stdout
    for st, same, replans in lines:
        assert st == "0" and same == "1", r.stdout
    assert any(int(x[2]) >= 1 for x in lines), r.stdout   # the deep chains did not converge in one hop
