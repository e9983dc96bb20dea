"""The executor routing (zd_route, zd_host.cpp route_plan) is a pure function
of the plan's shape and the device's CU count: every bound scales with the
CU count (measured on the 256-CU MI355X).  Host only."""
import ctypes as C

import pytest

from zstd_decompressor import _lib

FUSED, K4F, SEQW, FORK, K1FORK = 1, 2, 4, 8, 16


def route(cus, nframes, n_tables=None, n_seq=None, n_huf=None, single=True, flags=0):
    n_tables = 2 * nframes if n_tables is None else n_tables
    n_seq = nframes if n_seq is None else n_seq
    n_huf = nframes if n_huf is None else n_huf
    r = C.c_uint32()
    assert _lib.lib().zd_route(cus, nframes, n_tables, n_seq, n_huf, int(single), flags, C.byref(r)) == 0
    return r.value


@pytest.mark.parametrize("cus", [80, 256, 304])
def test_routing_scales_with_the_cu_count(cus):
    # the measured MI355X shapes, scaled: C3 (763 frames on 256 CUs: ~3 per CU)
    c3 = round(763 * cus / 256)
    assert route(cus, c3) & FUSED
    assert not route(cus, c3) & K4F                       # fused plans take no K4F
    assert route(cus, c3, flags=_lib.F_NO_FUSE) & K4F     # 1-3 frames per CU: K4F when not fused
    assert not route(cus, c3, single=False) & FUSED       # multi-block frames never fuse
    # fused from one to four frames per CU
    assert route(cus, cus) & FUSED and route(cus, 4 * cus) & FUSED
    assert not route(cus, cus - 1) & FUSED and not route(cus, 4 * cus + 1) & FUSED
    # K4F from one to three frames per CU
    assert route(cus, 3 * cus, flags=_lib.F_NO_FUSE) & K4F and not route(cus, 3 * cus + 1, flags=_lib.F_NO_FUSE) & K4F
    # wave-per-block sequence tables while the tables fit 64 per CU
    assert route(cus, 32 * cus, n_tables=64 * cus) & SEQW
    assert not route(cus, 32 * cus, n_tables=64 * cus + 1) & SEQW
    assert not route(cus, 10, flags=_lib.F_K1_LANES) & SEQW
    # the K2 | K3 fork: K3's last round of 64 chains per CU filled 0 < f <= 0.65
    slots = 64 * cus
    full_c4 = 320 * cus                                   # 81,920 blocks on 256 CUs: whole rounds
    assert not route(cus, full_c4) & FORK and route(cus, full_c4) & K1FORK
    share8 = 40 * cus                                     # 10,240 on 256: f 0.625
    assert route(cus, share8) & FORK and not route(cus, share8) & K1FORK
    assert not route(cus, slots + int(0.75 * slots)) & FORK   # f 0.75
    assert not route(cus, cus - 1) & FORK                 # fewer blocks than CUs


def test_routing_rejects_bad_arguments():
    r = C.c_uint32()
    assert _lib.lib().zd_route(0, 1, 1, 1, 1, 1, 0, C.byref(r)) == _lib.INVALID_ARG
