"""The pipelined streaming executor K4P (zd_kernels.hip zd_k_execute_pipe,
opt-in with ZD_K4P=1) against the oracle: 128 KiB single-block frames, 1 MiB
multi-block frames (Treeless literals, Repeat tables, repeat offsets across
blocks), long matches and literal runs (batches that leave the pipeline),
raw/RLE blocks, and corrupted inputs (the first failing sequence decides the
error, as in the reference's in-order execute, decoding_context.rs:78-106).
"""
import os
import random

import pytest

from corpus import gen, libzstd

from test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def k4p():
    os.environ["ZD_K4P"] = "1"          # read by every zd_decode_async
    yield
    del os.environ["ZD_K4P"]


@pytest.mark.parametrize("level", [1, 3, 19])
def test_k4p_frames(level):
    for kind, fn in (("text", gen.text), ("xml", gen.xml), ("binary", gen.binary)):
        src = fn(2 << 20, seed=70 + level)
        ost, _ = assert_parity(gen.frames(src, 128 << 10, level), False, f"K4P {kind} L{level} 128K")
        assert ost == 0
        ost, _ = assert_parity(gen.frames(src, 1 << 20, level), False, f"K4P {kind} L{level} 1M")
        assert ost == 0


def test_k4p_long_runs_and_raw_rle():
    r = random.Random(5)
    words = [bytes(r.randrange(97, 123) for _ in range(r.randrange(3, 9))) for _ in range(300)]
    parts = []
    for i in range(3000):
        parts.append(r.choice(words))
        if i % 97 == 0:
            parts.append(bytes(r.randrange(256) for _ in range(r.randrange(20, 3000))))   # long literal runs
        if i % 131 == 0:
            parts.append(b"".join(parts[-40:]) * 3)                                      # long matches
    src = b" ".join(parts)
    for level in (1, 9, 19):
        assert_parity(gen.frames(src, 128 << 10, level), False, f"K4P long runs L{level}")
    assert_parity(libzstd.compress(b"a" * 300000 + b"ab" * 50000, 3), False, "K4P rle/period")
    assert_parity(gen.c2_raw_rle(2 << 20), False, "K4P raw/rle blocks")


def test_k4p_corrupted():
    r = random.Random(99)
    base = gen.frames(gen.text(1 << 20, seed=3), 128 << 10, 3) + gen.frames(gen.binary(1 << 20, seed=4), 1 << 20, 19)
    for it in range(60):
        d = bytearray(base)
        for _ in range(r.randrange(1, 4)):
            d[r.randrange(len(d))] = r.randrange(256)
        assert_parity(bytes(d), False, f"K4P corrupt #{it}", allow_ood=True)
