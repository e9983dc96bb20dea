"""DecodingContext (decoding_context.rs:17-106), GPU-resident: the decoded
window lives in HBM; repeat offsets and the previous Huffman/FSE tables
persist across Block.decode calls."""
from __future__ import annotations

import ctypes as C

from . import _lib


class DecodingContext:
    def __init__(self, window_size: int):
        h = C.c_void_p()
        _lib.check(_lib.lib().zd_context_new(window_size, C.byref(h)), "DecodingContext::new")
        self._h = h
        self.window_size = window_size

    @property
    def decoded(self) -> bytes:
        L = _lib.lib()
        n = C.c_size_t()
        L.zd_context_decoded(self._h, None, 0, C.byref(n))
        out = (C.c_uint8 * max(n.value, 1))()
        _lib.check(L.zd_context_decoded(self._h, out, n.value, C.byref(n)), "decoded")
        return _lib.take(out, n.value)

    @property
    def offsets(self):
        o = (C.c_uint64 * 3)()
        _lib.check(_lib.lib().zd_context_offsets(self._h, o))
        return [o[0], o[1], o[2]]

    def execute_sequences(self, sequences, literals: bytes) -> None:
        """sequences: iterable of (literals_length, offset_value, match_length)."""
        seqs = list(sequences)
        n = len(seqs)
        ll = (C.c_uint32 * max(n, 1))(*[s[0] for s in seqs])
        of = (C.c_uint32 * max(n, 1))(*[s[1] for s in seqs])
        ml = (C.c_uint32 * max(n, 1))(*[s[2] for s in seqs])
        p, nl, keep = _lib.buf(bytes(literals))
        _lib.check(_lib.lib().zd_execute_sequences(self._h, ll, of, ml, n, p, nl), "execute_sequences")

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().zd_context_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
