"""ctypes binding of the system libzstd (1.4.8 in this image).

Used only as the *compressor* that makes synthetic .zst corpora and as an
independent RFC 8878 decoder for golden outputs on in-domain frames
(SURVEY.md §8c).  Never on the product's decode path.
"""
from __future__ import annotations

import ctypes as C
import ctypes.util

_lib = None

# ZSTD_cParameter values (zstd.h, stable since 1.4.0)
ZSTD_c_compressionLevel = 100
ZSTD_c_windowLog = 101
ZSTD_c_checksumFlag = 201
ZSTD_c_contentSizeFlag = 200


def lib():
    global _lib
    if _lib is None:
        path = None
        for cand in ("libzstd.so.1", ctypes.util.find_library("zstd")):
            if not cand:
                continue
            try:
                _lib = C.CDLL(cand)
                path = cand
                break
            except OSError:
                continue
        if _lib is None:
            raise OSError("libzstd not found")
        L = _lib
        L.ZSTD_compressBound.restype = C.c_size_t
        L.ZSTD_compressBound.argtypes = [C.c_size_t]
        L.ZSTD_compress.restype = C.c_size_t
        L.ZSTD_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
        L.ZSTD_decompress.restype = C.c_size_t
        L.ZSTD_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.ZSTD_isError.restype = C.c_uint
        L.ZSTD_isError.argtypes = [C.c_size_t]
        L.ZSTD_getErrorName.restype = C.c_char_p
        L.ZSTD_getErrorName.argtypes = [C.c_size_t]
        L.ZSTD_createCCtx.restype = C.c_void_p
        L.ZSTD_freeCCtx.argtypes = [C.c_void_p]
        L.ZSTD_CCtx_setParameter.restype = C.c_size_t
        L.ZSTD_CCtx_setParameter.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.ZSTD_compress2.restype = C.c_size_t
        L.ZSTD_compress2.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.ZSTD_getFrameContentSize.restype = C.c_ulonglong
        L.ZSTD_getFrameContentSize.argtypes = [C.c_void_p, C.c_size_t]
        L.ZSTD_versionNumber.restype = C.c_uint
        L.ZSTD_findFrameCompressedSize.restype = C.c_size_t
        L.ZSTD_findFrameCompressedSize.argtypes = [C.c_void_p, C.c_size_t]
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except OSError:
        return False


def version() -> int:
    return lib().ZSTD_versionNumber()


def _chk(r):
    L = lib()
    if L.ZSTD_isError(r):
        raise RuntimeError(L.ZSTD_getErrorName(r).decode())
    return r


def compress(data: bytes, level: int = 3, checksum: bool = False, window_log: int = 0,
             content_size: bool = True) -> bytes:
    """One frame (content_size False: no Frame_Content_Size field, as a
    streaming compressor writes).  ctypes drops the GIL, so threads compress
    in parallel."""
    L = lib()
    cap = L.ZSTD_compressBound(len(data))
    dst = C.create_string_buffer(cap)
    cctx = L.ZSTD_createCCtx()
    try:
        _chk(L.ZSTD_CCtx_setParameter(cctx, ZSTD_c_compressionLevel, level))
        _chk(L.ZSTD_CCtx_setParameter(cctx, ZSTD_c_checksumFlag, int(checksum)))
        if window_log:
            _chk(L.ZSTD_CCtx_setParameter(cctx, ZSTD_c_windowLog, window_log))
        if not content_size:
            _chk(L.ZSTD_CCtx_setParameter(cctx, ZSTD_c_contentSizeFlag, 0))
        n = _chk(L.ZSTD_compress2(cctx, dst, cap, data, len(data)))
    finally:
        L.ZSTD_freeCCtx(cctx)
    return dst.raw[:n]


def decompress_frame(frame: bytes, size: int) -> bytes:
    L = lib()
    dst = C.create_string_buffer(max(size, 1))
    n = _chk(L.ZSTD_decompress(dst, size, frame, len(frame)))
    return dst.raw[:n]


def frame_content_size(frame: bytes) -> int:
    return lib().ZSTD_getFrameContentSize(frame, len(frame))
