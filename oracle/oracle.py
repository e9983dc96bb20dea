"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/build/libzd_oracle.so, the plain-C restatement of the
reference Rust decoder (AchilleBailly/zstd-decompressor).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this, as the
checker or the timed CPU baseline — never as a decode path of the product.

Parity pinning: tests/golden/kat.json (the reference's own known-answer tests,
transcribed) and libzstd goldens on in-domain frames (tests/golden/).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libzd_oracle.so")
_lib = None
_lock = threading.Lock()


class OracleError(Exception):
    def __init__(self, code: int, a: int = 0, b: int = 0, partial: bytes = b""):
        super().__init__(f"oracle status {code} ({a}, {b})")
        self.code, self.a, self.b, self.partial = code, a, b, partial


class _Err(C.Structure):
    _fields_ = [("code", C.c_int), ("a", C.c_int64), ("b", C.c_int64)]


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc only)."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)
    return _LIB_PATH


def lib():
    global _lib
    with _lock:
        if _lib is None:
            build()
            L = C.CDLL(_LIB_PATH)
            u8p, sz, szp = C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_size_t)
            L.zdo_decompress.argtypes = [u8p, sz, C.c_int, C.POINTER(u8p), szp, szp, C.POINTER(_Err)]
            L.zdo_frame_decode.argtypes = [u8p, sz, szp, C.POINTER(u8p), szp, C.POINTER(C.c_int), C.POINTER(_Err)]
            L.zdo_free.argtypes = [C.c_void_p]
            L.zdo_forward_bits.argtypes = [u8p, sz, C.POINTER(C.c_uint32), sz, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(_Err)]
            L.zdo_backward_bits.argtypes = [u8p, sz, C.POINTER(C.c_uint32), sz, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(_Err)]
            L.zdo_parse_fse_table.argtypes = [u8p, sz, u8p, C.POINTER(C.c_int16), szp, C.POINTER(C.c_uint64), C.POINTER(_Err)]
            L.zdo_fse_from_distribution.argtypes = [C.c_uint8, C.POINTER(C.c_int16), sz, C.POINTER(C.c_uint16), C.POINTER(_Err)]
            L.zdo_fse_decode.argtypes = [C.POINTER(C.c_uint16), C.c_uint8, u8p, sz, sz, C.POINTER(C.c_uint16), C.POINTER(_Err)]
            L.zdo_alternating_decode.argtypes = L.zdo_fse_decode.argtypes
            L.zdo_huffman_weights_decode.argtypes = [u8p, sz, u8p, sz, u8p, sz, szp, C.POINTER(_Err)]
            L.zdo_huffman_parse_decode.argtypes = [u8p, sz, szp, u8p, sz, u8p, sz, szp, C.POINTER(_Err)]
            L.zdo_huffman_widths.argtypes = [u8p, sz, u8p, szp, szp, C.POINTER(_Err)]
            L.zdo_execute_sequences.argtypes = [C.POINTER(C.c_uint64), sz, u8p, sz, u8p, sz, szp, C.POINTER(_Err)]
            L.zdo_header_parse.argtypes = [u8p, sz, C.POINTER(C.c_uint64), szp, C.POINTER(_Err)]
            L.zdo_block_stages.argtypes = [u8p, sz, sz, C.POINTER(C.POINTER(C.c_uint64)), szp, C.POINTER(u8p), szp, C.POINTER(_Err)]
            _lib = L
    return _lib


def _buf(data: bytes):
    n = len(data)
    return (C.c_uint8 * max(n, 1)).from_buffer_copy(data if n else b"\0"), n


def _check(r: int, e: _Err, partial: bytes = b""):
    if r != 0:
        raise OracleError(r, e.a, e.b, partial)


def decompress(data: bytes, print_skippable: bool = False) -> bytes:
    """CLI semantics (src/main.rs:43-58). Raises OracleError on failure."""
    L = lib()
    b, n = _buf(data)
    out = C.POINTER(C.c_uint8)()
    ol, nf, e = C.c_size_t(), C.c_size_t(), _Err()
    r = L.zdo_decompress(b, n, int(print_skippable), C.byref(out), C.byref(ol), C.byref(nf), C.byref(e))
    res = C.string_at(out, ol.value) if out else b""
    L.zdo_free(out)
    _check(r, e, res)
    return res


def decompress_status(data: bytes, print_skippable: bool = False):
    """(status, output) — output holds what the reference would have produced
    before failing (the CLI itself prints nothing on failure)."""
    try:
        return 0, decompress(data, print_skippable)
    except OracleError as ex:
        return ex.code, ex.partial


def frame_decode(data: bytes):
    """Frame::parse + Frame::decode of the frame at data[0:]; returns
    (consumed, output, is_skippable)."""
    L = lib()
    b, n = _buf(data)
    out = C.POINTER(C.c_uint8)()
    ol, cons, sk, e = C.c_size_t(), C.c_size_t(), C.c_int(), _Err()
    r = L.zdo_frame_decode(b, n, C.byref(cons), C.byref(out), C.byref(ol), C.byref(sk), C.byref(e))
    res = C.string_at(out, ol.value) if out else b""
    L.zdo_free(out)
    _check(r, e)
    return cons.value, res, bool(sk.value)


def forward_bits(data: bytes, takes):
    L = lib(); b, n = _buf(data)
    t = (C.c_uint32 * max(len(takes), 1))(*takes)
    v = (C.c_uint64 * max(len(takes), 1))()
    la, e = C.c_uint64(), _Err()
    r = L.zdo_forward_bits(b if n else None, n, t, len(takes), v, C.byref(la), C.byref(e))
    return r, (e.a, e.b), list(v)[: len(takes)], la.value


def backward_bits(data: bytes, takes):
    L = lib(); b, n = _buf(data)
    t = (C.c_uint32 * max(len(takes), 1))(*takes)
    v = (C.c_uint64 * max(len(takes), 1))()
    lb, la, e = C.c_uint64(), C.c_uint64(), _Err()
    r = L.zdo_backward_bits(b if n else None, n, t, len(takes), v, C.byref(lb), C.byref(la), C.byref(e))
    return r, (e.a, e.b), list(v)[: len(takes)], lb.value, la.value


def parse_fse_table(data: bytes):
    L = lib(); b, n = _buf(data)
    al = C.c_uint8(); dist = (C.c_int16 * 256)(); ns = C.c_size_t(); bl = C.c_uint64(); e = _Err()
    r = L.zdo_parse_fse_table(b, n, C.byref(al), dist, C.byref(ns), C.byref(bl), C.byref(e))
    _check(r, e)
    return al.value, list(dist)[: ns.value], bl.value


def fse_from_distribution(al: int, dist):
    L = lib()
    d = (C.c_int16 * max(len(dist), 1))(*dist)
    out = (C.c_uint16 * (3 << min(al, 9)))()
    e = _Err()
    r = L.zdo_fse_from_distribution(al, d, len(dist), out, C.byref(e))
    _check(r, e)
    o = list(out)
    return [(o[3 * i], o[3 * i + 1], o[3 * i + 2]) for i in range(1 << al)]


def _table(states):
    flat = [x for s in states for x in s]
    return (C.c_uint16 * len(flat))(*flat)


def fse_decode(states, al, stream: bytes, nsym):
    L = lib(); b, n = _buf(stream)
    out = (C.c_uint16 * max(nsym, 1))(); e = _Err()
    r = L.zdo_fse_decode(_table(states), al, b, n, nsym, out, C.byref(e))
    _check(r, e)
    return list(out)[:nsym]


def alternating_decode(states, al, stream: bytes, nsym):
    L = lib(); b, n = _buf(stream)
    out = (C.c_uint16 * max(nsym, 1))(); e = _Err()
    r = L.zdo_alternating_decode(_table(states), al, b, n, nsym, out, C.byref(e))
    _check(r, e)
    return list(out)[:nsym]


def huffman_weights_decode(weights, stream: bytes, cap=1 << 20) -> bytes:
    L = lib(); w, nw = _buf(bytes(weights)); s, n = _buf(stream)
    out = (C.c_uint8 * cap)(); no = C.c_size_t(); e = _Err()
    r = L.zdo_huffman_weights_decode(w, nw, s, n, out, cap, C.byref(no), C.byref(e))
    _check(r, e)
    return bytes(out[: no.value])


def huffman_parse_decode(desc: bytes, stream: bytes, cap=1 << 20):
    L = lib(); d, dn = _buf(desc); s, n = _buf(stream)
    out = (C.c_uint8 * cap)(); no = C.c_size_t(); cons = C.c_size_t(); e = _Err()
    r = L.zdo_huffman_parse_decode(d, dn, C.byref(cons), s, n, out, cap, C.byref(no), C.byref(e))
    _check(r, e)
    return cons.value, bytes(out[: no.value])


def huffman_widths(desc: bytes):
    L = lib(); d, dn = _buf(desc)
    w = (C.c_uint8 * (1 << 18))(); nw = C.c_size_t(); cons = C.c_size_t(); e = _Err()   # (>= the weights a 127-byte stream can give)
    r = L.zdo_huffman_widths(d, dn, w, C.byref(nw), C.byref(cons), C.byref(e))
    _check(r, e)
    return cons.value, list(w)[: nw.value]


def execute_sequences(seqs, literals: bytes, cap=1 << 24) -> bytes:
    L = lib()
    flat = [x for s in seqs for x in s]
    sq = (C.c_uint64 * max(len(flat), 1))(*flat)
    lb, ln = _buf(literals)
    out = (C.c_uint8 * cap)(); no = C.c_size_t(); e = _Err()
    r = L.zdo_execute_sequences(sq, len(seqs), lb, ln, out, cap, C.byref(no), C.byref(e))
    _check(r, e)
    return bytes(out[: no.value])


def header_parse(data: bytes):
    L = lib(); b, n = _buf(data)
    out = (C.c_uint64 * 4)(); cons = C.c_size_t(); e = _Err()
    r = L.zdo_header_parse(b, n, out, C.byref(cons), C.byref(e))
    _check(r, e)
    none = (1 << 64) - 1
    return dict(content_checksum_flag=bool(out[0]), window_size=out[1],
                dictionnary_id=None if out[2] == none else out[2],
                content_size=None if out[3] == none else out[3]), cons.value


def block_stages(frame: bytes, block_index: int):
    """(sequences[(ll, offset_value, ml)], literals) of a compressed block."""
    L = lib(); b, n = _buf(frame)
    sq = C.POINTER(C.c_uint64)(); ns = C.c_size_t(); lt = C.POINTER(C.c_uint8)(); nl = C.c_size_t(); e = _Err()
    r = L.zdo_block_stages(b, n, block_index, C.byref(sq), C.byref(ns), C.byref(lt), C.byref(nl), C.byref(e))
    try:
        _check(r, e)
        seqs = [(sq[3 * i], sq[3 * i + 1], sq[3 * i + 2]) for i in range(ns.value)]
        lits = C.string_at(lt, nl.value) if nl.value else b""
    finally:
        L.zdo_free(sq); L.zdo_free(lt)
    return seqs, lits
