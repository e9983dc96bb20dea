"""Block (block.rs:27-99): Block.parse reads the 3-byte header and slices the
content (block.rs:43-72); Block.decode(ctx) runs the HIP pipeline on that
block against a GPU-resident DecodingContext (zd_block_decode)."""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import ZdError

RAW, RLE, COMPRESSED = 0, 1, 2


class Block:
    def __init__(self, kind: int, raw: bytes, last: bool, size: int, byte: int = 0):
        self.kind = kind          # RawBlock / RLEBlock / CompressedBlock
        self.raw = raw            # header + content bytes
        self.last = last
        self.size = size          # Block_Size
        self.byte = byte          # RLEBlock::byte

    def __repr__(self):
        names = {RAW: "RawBlock", RLE: "RLEBlock", COMPRESSED: "CompressedBlock"}
        return f"{names[self.kind]}(size={self.size}{', byte=%#x' % self.byte if self.kind == RLE else ''})"

    @property
    def repeat(self) -> int:
        return self.size

    @staticmethod
    def _from_desc(frame_raw: bytes, d, frame_off: int) -> "Block":
        start = d.src_offset - frame_off - 3
        end = d.src_offset - frame_off + (1 if d.type == RLE else d.block_size)
        return Block(d.type, frame_raw[start:end], bool(d.last), d.block_size, d.rle_byte)

    @staticmethod
    def parse(parser):
        """-> (Block, last).  block.rs:43-72."""
        h = parser.slice(3)
        x = h[0] | (h[1] << 8) | (h[2] << 16)
        last, kind, size = bool(x & 1), (x >> 1) & 3, x >> 3
        if kind == RAW:
            body = parser.slice(size)
            return Block(RAW, bytes(h) + body, last, size), last
        if kind == RLE:
            b = parser.u8()
            return Block(RLE, bytes(h) + bytes([b]), last, size, b), last
        if kind == COMPRESSED:
            body = parser.slice(size)
            return Block(COMPRESSED, bytes(h) + body, last, size), last
        raise ZdError(_lib.RESERVED_BLOCK_TYPE, "Block::parse")

    def decode(self, context) -> None:
        """Block::decode (block.rs:74-99) on the GPU, appending to context.decoded."""
        L = _lib.lib()
        p, n, keep = _lib.buf(self.raw)
        cons, last = C.c_size_t(), C.c_int()
        _lib.check(L.zd_block_decode(context._h, p, n, C.byref(cons), C.byref(last)), "Block::decode")
