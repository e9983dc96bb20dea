"""FrameIterator hands out frames from one decode of the whole buffer
(frame.py _Batch: zd_plan_decompress + zd_plan_frame_outputs) instead of a
plan + launch + sync per Frame.parse (verdict r4 weak 6).  It must raise the
same errors at the same frames as Frame.parse one frame at a time (the
reference's FrameIterator::next -> Frame::parse, frame.rs:86-99, and
ZStandard::decode, frame.rs:232-260): a table-description error at parse, an
execution error at decode, and every frame after a failure decoded on its
own (a fresh context per frame, frame.rs:232-237)."""
import pytest

from oracle import oracle


def _outcomes(data, batched):
    """[(parse error | None, decode error | None, bytes)] frame by frame, going
    on past failures (as a caller that skips bad frames would)."""
    from zstd_decompressor import ForwardByteParser, Frame, ZdError
    from zstd_decompressor.frame import FrameIterator
    p = ForwardByteParser(data)
    it = FrameIterator(p)
    res = []
    while not p.is_empty():
        try:
            f = next(it) if batched else Frame.parse(p)
        except ZdError as e:
            res.append((e.code, None, b""))
            break                                   # the frame could not be parsed: nothing follows it
        try:
            # (a skippable frame's payload is not part of the CLI's output without -p)
            res.append((None, None, b"" if f.is_skippable else f.decode()))
        except ZdError as e:
            res.append((None, e.code, b""))
    return res


def _cases():
    from test_parse_errors import _cases as pe_cases
    from corpus import gen
    frame, t, e, both = pe_cases()
    src = gen.text(600_000, seed=41)
    small = [gen.frames(src[i * 100_000:(i + 1) * 100_000], 100_000, 3) for i in range(6)]
    skip = b"\x50\x2a\x4d\x18" + (5).to_bytes(4, "little") + b"hello"
    return {
        "clean many": b"".join(small),
        "execution error in the middle": small[0] + e + small[1] + small[2],
        "table error in the middle": small[0] + small[1] + t + small[2],
        "two execution errors": e + small[0] + e + small[3],
        "skippable between": small[0] + skip + small[1],
        "truncated tail": b"".join(small) + small[0][:40],
    }


@pytest.mark.gpu
def test_frame_iterator_matches_frame_parse():
    for name, data in _cases().items():
        a = _outcomes(data, True)
        b = _outcomes(data, False)
        same = a == b                                   # (no pytest diff of megabytes of bytes)
        assert same, (name, [(x[0], x[1], len(x[2])) for x in a], [(x[0], x[1], len(x[2])) for x in b])
        # and the frames that decoded are the reference's bytes
        good = b"".join(x[2] for x in a if x[0] is None and x[1] is None)
        if all(x[0] is None and x[1] is None for x in a):
            ok = good == oracle.decompress(data)
            assert ok, name


@pytest.mark.gpu
def test_frame_iterator_is_one_decode_per_batch():
    """A clean many-frame buffer is one batch: the iterator makes one plan."""
    from zstd_decompressor import ForwardByteParser
    from zstd_decompressor import frame as fr
    made = []
    orig = fr._Batch.__init__

    def counting(self, *a, **k):
        made.append(1)
        orig(self, *a, **k)
    fr._Batch.__init__ = counting
    try:
        data = _cases()["clean many"]
        out = b"".join(f.decode() for f in ForwardByteParser(data).iter())
    finally:
        fr._Batch.__init__ = orig
    ok = out == oracle.decompress(data)
    assert ok
    assert len(made) == 1
