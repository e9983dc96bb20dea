"""ForwardByteParser (parsing.rs:9-112): a zero-copy cursor over the input."""
from __future__ import annotations

from . import _lib
from ._lib import ZdError


class ForwardByteParser:
    def __init__(self, data):
        self._data = bytes(data) if not isinstance(data, bytes) else data
        self._pos = 0

    def iter(self):                                     # parsing.rs:34-36
        from .frame import FrameIterator
        return FrameIterator(self)

    def __len__(self):                                  # parsing.rs:53-55
        return len(self._data) - self._pos

    def len(self) -> int:
        return len(self)

    def is_empty(self) -> bool:                         # parsing.rs:58-60
        return len(self) == 0

    def remaining(self) -> bytes:
        return self._data[self._pos:]

    def advance(self, n: int):
        self._pos += n

    def u8(self) -> int:                                # parsing.rs:39-50
        if not len(self):
            raise ZdError(_lib.NOT_ENOUGH_BYTES, "u8")
        v = self._data[self._pos]
        self._pos += 1
        return v

    def slice(self, n: int) -> bytes:                   # parsing.rs:63-79
        if n == 0:
            raise ZdError(_lib.EMPTY_SLICE, "slice")
        if len(self) < n:
            raise ZdError(_lib.NOT_ENOUGH_BYTES, f"slice({n}) of {len(self)}")
        s = self._data[self._pos:self._pos + n]
        self._pos += n
        return s

    def le_u32(self) -> int:                            # parsing.rs:82-95
        if len(self) < 4:
            raise ZdError(_lib.NOT_ENOUGH_BYTES, "le_u32")
        return int.from_bytes(self.slice(4), "little")

    def le_u16(self) -> int:                            # parsing.rs:98-111
        if len(self) < 2:
            raise ZdError(_lib.NOT_ENOUGH_BYTES, "le_u16")
        return int.from_bytes(self.slice(2), "little")
