"""ctypes binding of lib/libzd.so (C ABI in include/zd.h).

The decode path is the HIP library only: if it is missing this module raises
at import time — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("ZD_LIB_PATH") or os.path.join(_PKG, "lib", "libzd.so")

# status codes (include/zd.h)
OK = 0
STATUS_NAMES = {}


class ZdError(Exception):
    """A non-zero zd status.  `name` is the reference's error variant
    (parsing::Error, literals::Error, frame::Error, ...)."""

    def __init__(self, code: int, where: str = ""):
        self.code = code
        self.name = status_name(code)
        super().__init__(f"{self.name} ({code}){' in ' + where if where else ''}")


class FrameDesc(C.Structure):
    _fields_ = [("src_offset", C.c_uint64), ("src_size", C.c_uint64), ("content_size", C.c_uint64),
                ("window_size", C.c_uint64), ("dict_id", C.c_uint64), ("magic", C.c_uint32),
                ("kind", C.c_uint32), ("first_block", C.c_uint32), ("num_blocks", C.c_uint32),
                ("has_checksum", C.c_uint32), ("checksum", C.c_uint32)]


class BlockDesc(C.Structure):
    _fields_ = [("src_offset", C.c_uint64), ("block_size", C.c_uint32), ("type", C.c_uint8),
                ("last", C.c_uint8), ("rle_byte", C.c_uint8), ("_pad", C.c_uint8)]


class PlanInfo(C.Structure):
    _fields_ = [("nframes", C.c_uint64), ("nblocks", C.c_uint64), ("ncompressed", C.c_uint64),
                ("src_bytes", C.c_uint64), ("out_bytes", C.c_uint64), ("out_exact", C.c_uint64),
                ("workspace_bytes", C.c_uint64), ("nsequences", C.c_uint64), ("nliterals", C.c_uint64),
                ("index_status", C.c_int32), ("executors", C.c_uint32), ("host_ns", C.c_uint64),
                ("device_ns", C.c_uint64), ("walk_serial_bytes", C.c_uint64),
                ("io_h2d_ns", C.c_uint64), ("io_decode_ns", C.c_uint64), ("io_d2h_ns", C.c_uint64),
                ("error_key", C.c_uint64), ("replans", C.c_uint64),
                ("fused_redo_frames", C.c_uint64), ("device_descriptors", C.c_uint64)]


class GatherResult(C.Structure):
    _fields_ = [("total_len", C.c_uint64), ("status", C.c_int32), ("failed_rank", C.c_int32),
                ("first_error_frame", C.c_int64)]


COMM_ID_BYTES = 128

# every entry point declared in include/zd.h: name -> (restype, argtypes)
_u8p, _sz, _szp, _vp = C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_size_t), C.c_void_p
SIGNATURES = {
    "zd_status_name": (C.c_char_p, [C.c_int]),
    "zd_route": (C.c_int, [C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, C.c_uint32,
                           C.POINTER(C.c_uint32)]),
    "zd_abi_version": (C.c_int, []),
    "zd_trim_cache": (None, []),
    "zd_frames_index": (C.c_int, [_vp, _sz, C.POINTER(FrameDesc), _sz, _szp, C.POINTER(BlockDesc), _sz, _szp, _szp]),
    "zd_plan_create": (C.c_int, [_vp, _sz, C.c_uint32, C.POINTER(_vp)]),
    "zd_plan_create_device": (C.c_int, [_vp, _sz, C.c_uint32, _vp, C.POINTER(_vp)]),
    "zd_plan_info_get": (C.c_int, [_vp, C.POINTER(PlanInfo)]),
    "zd_plan_destroy": (None, [_vp]),
    "zd_decode_async": (C.c_int, [_vp, _vp, _vp, _sz, _vp]),
    "zd_plan_results": (C.c_int, [_vp, _vp, _vp, C.POINTER(C.c_int32), C.POINTER(C.c_uint64),
                                  C.POINTER(C.c_uint64), C.POINTER(C.c_int32)]),
    "zd_plan_checksums": (C.c_int, [_vp, _vp, _vp, C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]),
    "zd_plan_set_profiling": (C.c_int, [_vp, C.c_int]),
    "zd_plan_kernel_times": (C.c_int, [_vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_int)]),
    "zd_decompress": (C.c_int, [_vp, _sz, _vp, _sz, _szp, C.c_uint32]),
    "zd_plan_decompress": (C.c_int, [_vp, _vp, _sz, _vp, _sz, _szp]),
    "zd_context_new": (C.c_int, [C.c_uint64, C.POINTER(_vp)]),
    "zd_context_free": (None, [_vp]),
    "zd_block_decode": (C.c_int, [_vp, _vp, _sz, _szp, C.POINTER(C.c_int)]),
    "zd_execute_sequences": (C.c_int, [_vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                       _sz, _vp, _sz]),
    "zd_context_decoded": (C.c_int, [_vp, _vp, _sz, _szp]),
    "zd_context_offsets": (C.c_int, [_vp, C.POINTER(C.c_uint64)]),
    "zd_shard_partition": (C.c_int, [C.POINTER(C.c_uint64), _sz, C.c_int, _szp]),
    "zd_shard_range": (C.c_int, [_vp, _sz, C.c_int, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                 C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "zd_plan_frame_outputs": (C.c_int, [_vp, C.POINTER(C.c_int32), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                        C.c_size_t, C.POINTER(C.c_size_t)]),
    "zd_comm_unique_id": (C.c_int, [_vp]),
    "zd_comm_create": (C.c_int, [_vp, C.c_int, C.c_int, C.POINTER(_vp)]),
    "zd_comm_destroy": (None, [_vp]),
    "zd_comm_buffers": (C.c_int, [_vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "zd_gather_layout": (C.c_int, [C.POINTER(C.c_int64), C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                   C.POINTER(GatherResult)]),
    "zd_comm_gather": (C.c_int, [_vp, _vp, C.c_uint64, C.c_int32, C.c_int64, _vp, C.c_uint64,
                                 C.POINTER(GatherResult), _vp]),
    "zd_decode_sharded": (C.c_int, [_vp, _vp, _sz, C.c_uint32, _vp, C.c_uint64, C.POINTER(GatherResult), _vp]),
    "zd_decode_sharded_at": (C.c_int, [_vp, _vp, _sz, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_uint32, _vp,
                                       C.c_uint64, C.POINTER(GatherResult), _vp]),
    "zd_shard_cuts": (C.c_int, [_vp, _sz, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "zd_shard_range_at": (C.c_int, [_vp, _sz, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_int, C.c_int,
                                    C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_uint64)]),
}

_lib = None


def _one_hip_runtime():
    """One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64
    (soname libamdhip64.so.7, loaded as torch/lib/libamdhip64.so), and libzd's
    dependency on libamdhip64.so.7 binds to whichever copy is loaded first;
    loading libzd before torch would leave torch a second runtime that finds
    no GPU.  So torch's copy goes in first -- by path, without importing torch
    (which costs seconds): a later `import torch` then maps the same file and
    shares it.  With no torch installed, libzd takes ROCm's own runtime."""
    import sys
    if "torch" in sys.modules:
        return
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        rt = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(rt):
            C.CDLL(rt, mode=C.RTLD_GLOBAL)
            return


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C zstd-decompressor_amd` "
                              "(or __graft_entry__.build()); there is no CPU fallback")
        _one_hip_runtime()
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def status_name(code: int) -> str:
    return lib().zd_status_name(code).decode()


def check(code: int, where: str = ""):
    if code != OK:
        raise ZdError(code, where)
    return code


def buf(data):
    """(pointer, length) for a bytes-like object without copying when possible."""
    if isinstance(data, (bytes, bytearray, memoryview)):
        mv = memoryview(data).cast("B")
        n = mv.nbytes
        if n == 0:
            return None, 0, None
        if isinstance(data, bytes):
            keep = C.c_char_p(data)
            return C.cast(keep, C.c_void_p), n, keep
        arr = (C.c_uint8 * n).from_buffer(mv if not mv.readonly else bytearray(mv))
        return C.cast(arr, C.c_void_p), n, arr
    raise TypeError("bytes-like object required")

def buf_from(data: bytes, off: int):
    """(pointer, length, keep) for data[off:] of a bytes object, without the
    copy a slice makes (Frame.parse on a parser's remaining bytes: a 100 MB
    input cost ~10 ms a frame in slicing alone)."""
    n = len(data) - off
    if n <= 0:
        return None, 0, None
    keep = C.c_char_p(data)
    return C.c_void_p(C.cast(keep, C.c_void_p).value + off), n, keep


def take(arr, n: int) -> bytes:
    """The first n bytes of a ctypes byte array, one memcpy (a buffer view:
    C.string_at's size is a C int, and a ctypes slice goes element by element)."""
    return bytes(memoryview(arr).cast("B")[:n])


# status codes mirrored from include/zd.h
NOT_ENOUGH_BYTES, NOT_ENOUGH_BITS, MAX_READABLE_BITS_EXCEEDED = -1, -2, -3
EMPTY_INPUT_DATA, NULL_BYTE, EMPTY_SLICE = -4, -5, -6
LARGE_ACCURACY_LOG, CORRUPTED_TABLE, SEQUENCE_CODE_MAX_EXCEEDED = -12, -13, -14
HUFFMAN_DECODER_MISSING, CORRUPTED_STREAMS_SIZE = -20, -21
SEQ_RESERVED_SET, NO_PREVIOUS_DECODER = -30, -31
CTX_WINDOW_SIZE_TOO_BIG, NULL_OFFSET, IMPOSSIBLE_VALUE = -40, -41, -42
RESERVED_BLOCK_TYPE = -50
UNRECOGNIZED_MAGIC, FRAME_RESERVED_SET, MISSING_CHECKSUM, WINDOW_SIZE_TOO_BIG = -60, -61, -64, -66
REF_PANIC, OUT_OF_DOMAIN, DST_TOO_SMALL, INVALID_ARG, HIP, NO_MEMORY, NOT_DECODED = -90, -91, -92, -93, -94, -95, -96
F_SKIPPABLE = 1
F_BLOCK_PARALLEL = 2   # every frame with a compressed block -> K4J (block-parallel execute)
F_FRAME_SERIAL = 4     # no frame -> K4J
F_SEQ_ONE_LANE = 8     # K3 one lane per block instead of four (K3Q)
F_NO_FUSE = 32         # K3 then K4 as two launches in few-frame plans (no zd_k_fused)
F_K1_LANES = 64        # K1's sequence half on serial lanes in plans of <= 16,384 tables
F_J_ONE_ROUND = 128    # test switch: K4J pointer jumping cut to one round of one hop
F_SEQ_NO_LATENCY = 256 # K3Q instead of the one-block-per-wave K3L in plans of few blocks
EXEC_FUSED, EXEC_K4F, EXEC_K4J = 1, 2, 4   # zd_plan_info.executors bits (include/zd.h ZD_EXEC_*)
