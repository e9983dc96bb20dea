"""CPU-side checks of the C ABI: the library loads, exports every entry point
declared in include/zd.h, and the host index (no GPU needed) agrees with the
oracle's frame structure."""
import os
import re

import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "zd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zd_[a-z_0-9]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    from zstd_decompressor import _lib
    L = _lib.lib()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_lib.SIGNATURES), "ctypes signatures out of sync with zd.h"


def test_status_names():
    from zstd_decompressor import _lib
    assert _lib.status_name(0) == "Ok"
    assert _lib.status_name(_lib.NOT_ENOUGH_BYTES) == "NotEnoughBytes"
    assert _lib.status_name(_lib.REF_PANIC) == "ReferencePanic"
    assert _lib.lib().zd_abi_version() == 8


def test_index_resources(resources):
    from zstd_decompressor.batch import frames_index
    for name, data in resources.items():
        frames, blocks, st, cons = frames_index(data)
        assert st == 0 and cons == len(data), name
        off = 0
        for f in frames:
            c, _, sk = oracle.frame_decode(data[off:])
            assert f["src_offset"] == off and f["src_size"] == c and bool(f["kind"]) == sk, name
            off += c


def test_index_kat_frames(kat):
    from zstd_decompressor.batch import frames_index
    for c in kat["frames"]:
        data = bytes(c["data"])
        frames, blocks, st, cons = frames_index(data)
        ost, _ = oracle.decompress_status(data, True)
        if ost in (-1, -6, -50, -60, -61, -64, -66):   # structural errors are host-detected
            assert st == ost, c["src"]
        else:
            assert st == 0, c["src"]


def test_index_block_kats():
    # tests/block.rs:12-79 through the Python Block.parse mirror
    from zstd_decompressor import ForwardByteParser, Block, ZdError
    p = ForwardByteParser(bytes([0x21, 0x0, 0x0, 0x10, 0x20, 0x30, 0x40, 0x50]))
    b, last = Block.parse(p)
    assert last and b.kind == 0 and b.raw[3:] == bytes([0x10, 0x20, 0x30, 0x40]) and p.len() == 1
    p = ForwardByteParser(bytes([0x22, 0x0, 0x18, 0x42, 0x50]))
    b, last = Block.parse(p)
    assert not last and b.kind == 1 and b.byte == 0x42 and b.repeat == 196612 and p.len() == 1
    with pytest.raises(ZdError) as e:
        Block.parse(ForwardByteParser(bytes([0x27, 0x0, 0x0, 0x10, 0x20, 0x30, 0x40, 0x50])))
    assert e.value.name == "ReservedBlockType"
    with pytest.raises(ZdError) as e:
        Block.parse(ForwardByteParser(bytes([0x21, 0x0, 0x0, 0x10, 0x20, 0x30])))
    assert e.value.name == "NotEnoughBytes"


def test_frames_index_headers(kat):
    """The host index (zd_frames_index, the header pass of Frame::parse) on
    the reference's header KATs (tests/frame.rs:155-257), no GPU."""
    from zstd_decompressor.batch import frames_index
    none = (1 << 64) - 1
    for c in kat["header_parse"]:
        if "error" in c:
            continue
        data = bytes([0x28, 0xB5, 0x2F, 0xFD] + c["data"] + [0x03, 0x00, 0x00, 0x00])
        frames, _, st, _ = frames_index(data)
        f = frames[0]
        got = (f["window_size"], None if f["content_size"] == none else f["content_size"],
               None if f["dict_id"] == none else f["dict_id"])
        assert st == 0 and got == (c["window"], c["fcs"], c["dict"]), c["src"]


@pytest.mark.gpu
def test_frame_parse_headers(kat):
    """Frame.parse (the crate mirror): the header pass, then the GPU pass that
    builds the frame's tables (ZStandard::parse)."""
    from zstd_decompressor import ForwardByteParser, Frame
    for c in kat["header_parse"]:
        if "error" in c:
            continue
        data = bytes([0x28, 0xB5, 0x2F, 0xFD] + c["data"] + [0x01, 0x00, 0x00])  # + empty raw... last RLE block
        # last RLE block of 0 bytes: header 0b011 -> last, RLE, size 0, byte 0
        data = bytes([0x28, 0xB5, 0x2F, 0xFD] + c["data"] + [0x03, 0x00, 0x00, 0x00])
        f = Frame.parse(ForwardByteParser(data))
        h = f.inner.header()
        assert (h.window_size, h.content_size, h.dictionnary_id) == (c["window"], c["fcs"], c["dict"]), c["src"]


def test_buf_from_points_into_the_bytes():
    """_lib.buf_from (Frame.parse's remaining bytes, no slice copy): the
    pointer is the bytes' own buffer at the offset."""
    import ctypes as C
    from zstd_decompressor import _lib
    data = bytes(range(256)) * 17
    for off in (0, 1, 255, len(data) - 1, len(data)):
        p, n, keep = _lib.buf_from(data, off)
        assert n == max(len(data) - off, 0)
        if n:
            assert C.string_at(p, n) == data[off:]
            base, _, _ = _lib.buf(data)
            assert p.value == base.value + off

