"""Batch decode over the C ABI — the hot path.

`decompress` mirrors the CLI loop (src/main.rs:43-58) on host buffers;
`Plan` keeps input/output in HBM (torch tensors or raw device pointers) and is
what bench.py times.
"""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import ZdError, FrameDesc, BlockDesc, PlanInfo


def frames_index(data: bytes, max_frames: int = 0):
    """zd_frames_index: ([frame dicts], [block dicts], status, consumed)."""
    L = _lib.lib()
    p, n, keep = _lib.buf(data)
    nf, nb, cons = C.c_size_t(), C.c_size_t(), C.c_size_t()
    L.zd_frames_index(p, n, None, 0, C.byref(nf), None, 0, C.byref(nb), C.byref(cons))
    fa = (FrameDesc * max(nf.value, 1))()
    ba = (BlockDesc * max(nb.value, 1))()
    st = L.zd_frames_index(p, n, fa, nf.value, C.byref(nf), ba, nb.value, C.byref(nb), C.byref(cons))
    frames = [{k: getattr(fa[i], k) for k, _ in FrameDesc._fields_} for i in range(nf.value)]
    blocks = [{k: getattr(ba[i], k) for k, _ in BlockDesc._fields_ if k != "_pad"} for i in range(nb.value)]
    return frames, blocks, st, cons.value


def run_plan(plan, p, n):
    """(status, output): zd_plan_decompress into a buffer sized from the plan;
    again with the size it reports when the output came out larger (a frame
    that decodes past its declared size is re-planned inside the call).  The
    output is read back with one memcpy (_lib.take), not an element-wise
    ctypes slice (seconds per 100 MB)."""
    L = _lib.lib()
    cap = max(plan.info.out_bytes, 1)
    for _ in range(2):
        out = (C.c_uint8 * cap)()
        ol = C.c_size_t()
        st = L.zd_plan_decompress(plan._h, p, n, out, cap, C.byref(ol))
        if st in (_lib.HIP, _lib.INVALID_ARG, _lib.NO_MEMORY):
            _lib.check(st, "zd_plan_decompress")
        if ol.value <= cap:
            break
        cap = ol.value
    return st, _lib.take(out, min(ol.value, cap))


def _decompress(data: bytes, flags: int):
    """One plan (the host walk once) and zd_plan_decompress — what
    zd_decompress does, with the plan's output size read first."""
    p, n, keep = _lib.buf(data)
    plan = Plan(data, bool(flags & _lib.F_SKIPPABLE), flags & ~_lib.F_SKIPPABLE)
    try:
        return run_plan(plan, p, n)
    finally:
        plan.close()


def decompress(data: bytes, print_skippable: bool = False) -> bytes:
    """Decode every frame of `data` on the GPU (host in, host out)."""
    st, out = _decompress(data, _lib.F_SKIPPABLE if print_skippable else 0)
    _lib.check(st, "zd_decompress")
    return out


KEY_NONE = (1 << 64) - 1
PH_PARSE = 0


def decode_keyed(data: bytes, flags: int = 0):
    """(status, output of the frames before the first failure, error key):
    one plan and zd_plan_decompress; the key's phase (key >> 62: 0 parse, 1
    decode, 3 a limit) tells a table-description error, which the reference
    raises in Frame::parse, from an execution error it raises in decode."""
    plan = Plan(data, bool(flags & _lib.F_SKIPPABLE), flags & ~_lib.F_SKIPPABLE)
    try:
        p, n, keep = _lib.buf(data)
        st, out = run_plan(plan, p, n)
        return st, out, plan.refresh_info().error_key
    finally:
        plan.close()


def decompress_status(data: bytes, print_skippable: bool = False, flags: int = 0):
    """(status, output of the frames before the first failure).  flags: extra
    zd_plan flags (_lib.F_BLOCK_PARALLEL / F_FRAME_SERIAL pick the executor)."""
    return _decompress(data, (_lib.F_SKIPPABLE if print_skippable else 0) | flags)


class Plan:
    """zd_plan: host index + device workspace for one byte range of frames."""

    def __init__(self, data: bytes, print_skippable: bool = False, flags: int = 0):
        L = _lib.lib()
        self._data = data
        p, n, self._keep = _lib.buf(data)
        h = C.c_void_p()
        _lib.check(L.zd_plan_create(p, n, (_lib.F_SKIPPABLE if print_skippable else 0) | flags, C.byref(h)),
                   "zd_plan_create")
        self._h = h
        self.info = PlanInfo()
        _lib.check(L.zd_plan_info_get(h, C.byref(self.info)), "zd_plan_info_get")

    @classmethod
    def from_device(cls, d_src: int, n: int, print_skippable: bool = False, flags: int = 0, stream: int = 0):
        """zd_plan_create_device: the same plan for n bytes resident in HBM at d_src
        (readable for n + 16 bytes); the frame/block header walk runs on the GPU."""
        self = cls.__new__(cls)
        L = _lib.lib()
        self._data, self._keep = None, None
        h = C.c_void_p()
        _lib.check(L.zd_plan_create_device(C.c_void_p(d_src), n, (_lib.F_SKIPPABLE if print_skippable else 0) | flags,
                                           C.c_void_p(stream), C.byref(h)), "zd_plan_create_device")
        self._h = h
        self.info = PlanInfo()
        _lib.check(L.zd_plan_info_get(h, C.byref(self.info)), "zd_plan_info_get")
        return self

    def set_profiling(self, on=True):
        """zd_plan_set_profiling: True / 1 every kernel timed one after another,
        2 the pipeline as it runs with events around its dominant launch, 0 off."""
        _lib.check(_lib.lib().zd_plan_set_profiling(self._h, int(on)))

    def refresh_info(self):
        """zd_plan_info again (the fields of the last decode / results)."""
        _lib.check(_lib.lib().zd_plan_info_get(self._h, C.byref(self.info)), "zd_plan_info_get")
        return self.info

    def decode_async(self, d_src: int, d_dst: int, dst_cap: int, stream: int = 0):
        """Launch the pipeline; pointers/stream are integers (e.g. tensor.data_ptr(),
        torch.cuda.current_stream().cuda_stream)."""
        _lib.check(_lib.lib().zd_decode_async(self._h, C.c_void_p(d_src), C.c_void_p(d_dst), dst_cap,
                                              C.c_void_p(stream)), "zd_decode_async")

    def results(self, d_dst: int, stream: int = 0):
        """(status, total_len, per-frame statuses, per-frame lengths, first error frame)."""
        nf = self.info.nframes
        st_arr = (C.c_int32 * max(nf, 1))()
        ln_arr = (C.c_uint64 * max(nf, 1))()
        total, first = C.c_uint64(), C.c_int32()
        st = _lib.lib().zd_plan_results(self._h, C.c_void_p(d_dst), C.c_void_p(stream), st_arr, ln_arr,
                                        C.byref(total), C.byref(first))
        if st in (_lib.HIP, _lib.INVALID_ARG):
            _lib.check(st, "zd_plan_results")
        return st, total.value, list(st_arr)[:nf], list(ln_arr)[:nf], first.value

    def checksums(self, d_dst: int, stream: int = 0):
        """After results(): (ok per frame: 1 match / 0 mismatch / -1 none, XXH64 digests),
        computed on the GPU (zd_plan_checksums; an extra, the reference never enforces it)."""
        nf = self.info.nframes
        ok = (C.c_int32 * max(nf, 1))()
        h = (C.c_uint64 * max(nf, 1))()
        _lib.check(_lib.lib().zd_plan_checksums(self._h, C.c_void_p(d_dst), C.c_void_p(stream), ok, h),
                   "zd_plan_checksums")
        return list(ok)[:nf], list(h)[:nf]

    def kernel_times(self):
        names = (C.c_char_p * 8)()
        ms = (C.c_float * 8)()
        n = C.c_int()
        _lib.check(_lib.lib().zd_plan_kernel_times(self._h, names, ms, 8, C.byref(n)))
        return {names[i].decode(): ms[i] for i in range(n.value)}

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().zd_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
