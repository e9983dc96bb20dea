"""Frame layer (frame.rs): Frame, ZStandard, Skippable, Header, FrameIterator.

Frame.parse runs the host index (zd_frames_index: FrameIterator/Frame::parse/
Header::parse/Block::parse structure, frame.rs:61-230) and then the HIP
pipeline on the frame: ZStandard::parse builds every block's Huffman and FSE
tables and fails there (frame.rs:198-230, literals.rs:88-133,
sequences.rs:91-143), and the GPU builds those tables in its first kernel, so
an error in a table description (error key phase 0, parse) is raised by
Frame.parse as in the reference, whatever block it is in; the frame's output
or its execution error (phase 1) is kept for decode() (ZStandard::decode,
frame.rs:232-260).  Host-only callers that want the index without a GPU
pass use zd_frames_index (batch.frames_index).

FrameIterator (frame.rs:86-99, the loop of src/main.rs:43-53) does not pay a
plan + launch + sync per frame: it decodes the parser's remaining bytes in
ONE zd_plan_decompress and hands out each frame's status and bytes from it
(zd_plan_frame_outputs), with the same per-frame parse / decode errors as
Frame.parse.  Frames after the batch's first failing frame were not decoded
(ZD_E_NOT_DECODED): an iterator that goes on past a failure decodes the rest
in a new batch from there.
"""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import ZdError, FrameDesc, BlockDesc

MAGIC_ZSTD = 0xFD2FB528           # frame.rs:41
MAGIC_SKIP = 0x184D2A50           # frame.rs:42
MAX_WIN_SIZE = 8 << 20            # frame.rs:44
_NONE = (1 << 64) - 1


class Header:                     # frame.rs:103-108
    def __init__(self, d: FrameDesc):
        self.content_checksum_flag = bool(d.has_checksum)
        self.window_size = d.window_size
        self.dictionnary_id = None if d.dict_id == _NONE else d.dict_id
        self.content_size = None if d.content_size == _NONE else d.content_size

    def __repr__(self):
        return (f"Header(content_checksum_flag={self.content_checksum_flag}, window_size={self.window_size}, "
                f"dictionnary_id={self.dictionnary_id}, content_size={self.content_size})")


class Skippable:                  # frame.rs:55-58
    def __init__(self, magic: int, data: bytes):
        self.magic, self.data = magic, data

    def decode(self) -> bytes:
        return bytes(self.data)


class ZStandard:                  # frame.rs:189-272
    def __init__(self, raw: bytes, d: FrameDesc, blocks, decoded=None):
        self._raw, self._d, self._blocks = raw, d, blocks
        self._header = Header(d)
        self._decoded = decoded       # (status, output) of the GPU pass Frame.parse ran

    def header(self) -> Header:
        return self._header

    def checksum(self):
        return self._d.checksum if self._d.has_checksum else None

    def blocks(self):
        return self._blocks

    def decode(self) -> bytes:
        if self._decoded is None:
            from .batch import decompress
            return decompress(self._raw)
        st, out = self._decoded
        _lib.check(st, "ZStandard::decode")
        return out


class Frame:
    """Frame::ZStandardFrame / Frame::SkippableFrame (frame.rs:48-84)."""

    def __init__(self, inner):
        self.inner = inner

    @property
    def is_skippable(self) -> bool:
        return isinstance(self.inner, Skippable)

    @staticmethod
    def parse(parser) -> "Frame":
        L = _lib.lib()
        base = parser._pos
        p, n, keep = _lib.buf_from(parser._data, base)    # the remaining bytes, not copied
        fa = (FrameDesc * 1)()
        nf, nb, cons = C.c_size_t(), C.c_size_t(), C.c_size_t()
        # first pass: block count of the first frame
        st = L.zd_frames_index(p, n, fa, 1, C.byref(nf), None, 0, C.byref(nb), C.byref(cons))
        if st != 0 and nf.value == 0:
            raise ZdError(st, "Frame::parse")
        ba = (BlockDesc * max(nb.value, 1))()
        L.zd_frames_index(p, n, fa, 1, C.byref(nf), ba, nb.value, C.byref(nb), C.byref(cons))
        d = fa[0]
        raw = parser._data[base + d.src_offset:base + d.src_offset + d.src_size]
        parser.advance(d.src_offset + d.src_size)
        if d.kind == 1:
            return Frame(Skippable(d.magic, raw[8:]))
        from .block import Block
        from .batch import decode_keyed, KEY_NONE, PH_PARSE
        blocks = [Block._from_desc(raw, ba[i], d.src_offset) for i in range(nb.value)]
        fst, out, key = decode_keyed(raw)
        if fst != 0 and key != KEY_NONE and (key >> 62) == PH_PARSE:
            raise ZdError(fst, "Frame::parse")        # a Huffman / FSE table description (ZStandard::parse)
        return Frame(ZStandard(raw, d, blocks, (fst, out)))

    def decode(self) -> bytes:
        return self.inner.decode()


class _Batch:
    """One GPU decode of a parser's remaining bytes, frame by frame: the host
    index of the frames (zd_frames_index), one zd_plan_decompress, and each
    frame's (status, offset, length) in the output (zd_plan_frame_outputs)."""

    def __init__(self, data: bytes, start: int):
        from .batch import Plan, KEY_NONE, run_plan
        L = _lib.lib()
        self.start, self.data = start, data
        p, n, keep = _lib.buf(data)
        nf, nb, cons = C.c_size_t(), C.c_size_t(), C.c_size_t()
        L.zd_frames_index(p, n, None, 0, C.byref(nf), None, 0, C.byref(nb), C.byref(cons))
        self.fa = (FrameDesc * max(nf.value, 1))()
        self.ba = (BlockDesc * max(nb.value, 1))()
        L.zd_frames_index(p, n, self.fa, nf.value, C.byref(nf), self.ba, nb.value, C.byref(nb), C.byref(cons))
        self.nf = nf.value
        self.key = KEY_NONE
        self.first = -1                      # the batch's first failing frame (its key is the plan's)
        self.status = [0] * self.nf
        self.off = [0] * self.nf
        self.len = [0] * self.nf
        self.out = b""
        self.next = 0                        # the next frame to hand out
        if self.nf == 0:
            return
        plan = Plan(data)
        try:
            st, self.out = run_plan(plan, p, n)
            self.key = plan.refresh_info().error_key
            fs = (C.c_int32 * self.nf)()
            fo = (C.c_uint64 * self.nf)()
            fl = (C.c_uint64 * self.nf)()
            m = C.c_size_t()
            _lib.check(L.zd_plan_frame_outputs(plan._h, fs, fo, fl, self.nf, C.byref(m)), "zd_plan_frame_outputs")
            k = min(m.value, self.nf)
            self.status[:k], self.off[:k], self.len[:k] = list(fs)[:k], list(fo)[:k], list(fl)[:k]
            for f in range(k, self.nf):
                self.status[f] = _lib.NOT_DECODED
            self.first = next((f for f in range(self.nf) if self.status[f] != 0), -1)
        finally:
            plan.close()

    def frame(self, parser):
        """Frame.parse for the parser's next frame from this batch, or None
        when the batch does not hold it (past a failure, or not indexed)."""
        f = self.next
        if parser._pos != self.start + (self.fa[f].src_offset if f < self.nf else -1) or f >= self.nf:
            return None
        st = self.status[f]
        if st == _lib.NOT_DECODED:
            return None
        from .batch import PH_PARSE, KEY_NONE
        d = self.fa[f]
        raw = self.data[d.src_offset:d.src_offset + d.src_size]
        self.next += 1
        parser.advance(d.src_size)
        if d.kind == 1:
            return Frame(Skippable(d.magic, raw[8:]))
        from .block import Block
        blocks = [Block._from_desc(raw, self.ba[d.first_block + i], d.src_offset) for i in range(d.num_blocks)]
        if st != 0 and f == self.first and self.key != KEY_NONE and (self.key >> 62) == PH_PARSE:
            raise ZdError(st, "Frame::parse")        # a Huffman / FSE table description (ZStandard::parse)
        out = self.out[self.off[f]:self.off[f] + self.len[f]] if st == 0 else b""
        return Frame(ZStandard(raw, d, blocks, (st, out)))


class FrameIterator:              # frame.rs:86-99
    def __init__(self, parser):
        self.parser = parser
        self._batch = None

    def __iter__(self):
        return self

    def __next__(self) -> Frame:
        if self.parser.is_empty():
            raise StopIteration
        fr = self._batch.frame(self.parser) if self._batch is not None else None
        if fr is None:
            # a new batch from here (the first call, or past the last batch's failure)
            self._batch = _Batch(self.parser.remaining(), self.parser._pos)
            fr = self._batch.frame(self.parser)
        if fr is None:                          # a frame the host index rejects: Frame.parse raises its error
            return Frame.parse(self.parser)
        return fr
