"""Which call fails (verdict r3 item 7): the reference's ZStandard::parse builds
every block's Huffman and FSE tables before any block decodes
(frame.rs:198-230, literals.rs:88-133, sequences.rs:91-143), so a corrupt
table description in block 3 is reported by Frame::parse even when block 1
would fail to execute, and an execution error alone by Frame::decode.  The
GPU path orders its per-frame error keys the same way (parse phase first,
zd_common.h make_key), and the crate mirror's Frame.parse raises the
parse-phase ones."""
import functools

import pytest

from oracle import oracle

TABLE_ERRORS = (-12, -13)          # LargeAccuracyLog, CorruptedTable (decoders/mod.rs:10-23)


@functools.lru_cache(maxsize=1)
def _cases():
    """(clean frame, block-3 table corruption, block-1 execution corruption,
    both) of one eight-block 1 MiB frame at level 9."""
    from corpus import gen
    from zstd_decompressor.batch import frames_index
    src = gen.text(1 << 20, seed=31)
    frame = gen.frames(src, 1 << 20, 9)
    frames, blocks, st, _ = frames_index(frame)
    assert st == 0 and len(frames) == 1 and len(blocks) >= 4
    def flip(data, at, x):
        b = bytearray(data)
        b[at] ^= x
        return bytes(b)
    b3 = blocks[3]
    table = None
    for k in range(0, 64):                 # the block's first bytes: literal header, tree description
        for x in (0xFF, 0x80, 0x0F, 0x10):
            cand = flip(frame, b3["src_offset"] + k, x)
            if oracle.decompress_status(cand, False)[0] in TABLE_ERRORS:
                table = (b3["src_offset"] + k, x)
                break
        if table:
            break
    b1 = blocks[1]
    end1 = b1["src_offset"] + b1["block_size"]
    execution = None
    for k in range(2, 400):                # the tail of block 1: its sequence bitstream
        cand = flip(frame, end1 - k, 0x5A)
        st1 = oracle.decompress_status(cand, False)[0]
        if st1 != 0 and st1 not in TABLE_ERRORS:
            execution = (end1 - k, 0x5A)
            break
    assert table and execution, (table, execution)
    t = flip(frame, *table)
    e = flip(frame, *execution)
    return frame, t, e, flip(t, *execution)


def test_reference_reports_the_table_error_first():
    """The oracle (the reference's order): block 3's table error wins over
    block 1's execution error."""
    frame, t, e, both = _cases()
    st_t = oracle.decompress_status(t, False)[0]
    st_e = oracle.decompress_status(e, False)[0]
    st_b = oracle.decompress_status(both, False)[0]
    assert st_t in TABLE_ERRORS and st_e not in TABLE_ERRORS and st_e != 0
    assert st_b == st_t


@pytest.mark.gpu
def test_gpu_and_frame_parse_fail_where_the_reference_does():
    from zstd_decompressor import ForwardByteParser, Frame, ZdError
    from test_gpu_parity import assert_parity
    frame, t, e, both = _cases()
    for name, data in (("clean", frame), ("table", t), ("execution", e), ("both", both)):
        assert_parity(data, False, name)
    # Frame::parse fails on a table description in any block ...
    for data in (t, both):
        with pytest.raises(ZdError) as ex:
            Frame.parse(ForwardByteParser(data))
        assert ex.value.code == oracle.decompress_status(data, False)[0]
    # ... and an execution error alone is Frame::decode's
    f = Frame.parse(ForwardByteParser(e))
    with pytest.raises(ZdError) as ex:
        f.decode()
    assert ex.value.code == oracle.decompress_status(e, False)[0]
    assert Frame.parse(ForwardByteParser(frame)).decode() == oracle.decompress(frame)
