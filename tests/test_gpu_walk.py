"""The device header walk (zd_plan_create_device, zd_kernels.hip zd_k_walk):
the frame / block header walk and the section-header parse on the GPU for an
input resident in HBM (frame.rs:61-230, block.rs:43-72,
literals.rs:88-206, sequences.rs:52-143).  Its plan must equal the host
walk's (zd_plan_create) descriptor for descriptor (ZD_PLAN_DUMP) on every
input: the reference's resources, libzstd frames of every shape, magic numbers
planted inside compressed data, frames longer than a walk range, skippable
frames, corruptions and truncations (tests/test_host_walk.py's inputs); and a
decode through it must give the host plan's output and status.
"""
import os

import pytest

from corpus import gen, libzstd

pytestmark = pytest.mark.gpu


def _dump(path, make):
    os.environ["ZD_PLAN_DUMP"] = path
    try:
        plan = make()
    finally:
        del os.environ["ZD_PLAN_DUMP"]
    return plan, open(path, "rb").read()


def _decode(plan, d_src, dev):
    import torch
    n = plan.info.out_bytes
    d_dst = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), n, s)
    st, total, fst, flen, first = plan.results(d_dst.data_ptr(), s)
    return st, bytes(d_dst[:total].cpu().numpy().tobytes()), fst, flen, first


def _inputs(resources):
    for name, data in resources.items():
        yield name, data
    yield "empty", b""
    yield "three bytes", b"\x28\xb5\x2f"
    yield "one frame", libzstd.compress(gen.text(200 << 10, seed=91), 3)
    yield "multi-block frames", gen.frames(gen.text(3 << 20, seed=92), 1 << 20, 9)
    yield "raw/rle", libzstd.compress(gen.binary(300 << 10, seed=93), 1) + libzstd.compress(bytes(500 << 10), 3)
    import test_host_walk
    yield from test_host_walk._inputs()


def test_device_walk_plan_equals_host_walk(resources, tmp_path):
    import torch
    from zstd_decompressor.batch import Plan
    dev = torch.device("cuda", 0)
    for name, data in _inputs(resources):
        for skip in (False, True):
            d_src = torch.zeros(len(data) + 64, dtype=torch.uint8, device=dev)
            if data:
                d_src[: len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
            torch.cuda.synchronize(dev)
            hp, hd = _dump(str(tmp_path / "h.bin"), lambda: Plan(data, skip))
            dp, dd = _dump(str(tmp_path / "d.bin"),
                           lambda: Plan.from_device(d_src.data_ptr(), len(data), skip,
                                                    stream=torch.cuda.current_stream(dev).cuda_stream))
            assert dd == hd, f"{name} (-p {skip}): device-walk plan differs from the host walk's"
            assert dp.info.index_status == hp.info.index_status, name
            if not skip and len(data) < (8 << 20):
                assert _decode(dp, d_src, dev) == _decode(hp, d_src, dev), name
            hp.close()
            dp.close()


def test_device_walk_false_frame_costs_one_range():
    """A planted magic number that parses as a whole frame, first in device
    range 4 (256 KiB ranges): the stitch walks on the device one range at a
    time until the chain meets a later range's (it used to walk the rest of
    the input as one serial range); the plan still equals the host walk's."""
    import torch
    import test_host_walk
    from zstd_decompressor.batch import Plan
    dev = torch.device("cuda", 0)
    data, rsize, at = test_host_walk.false_frame_input(cut=4 << 18)
    d_src = torch.zeros(len(data) + 64, dtype=torch.uint8, device=dev)
    d_src[: len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    torch.cuda.synchronize(dev)
    hp = Plan(data)
    dp = Plan.from_device(d_src.data_ptr(), len(data), stream=torch.cuda.current_stream(dev).cuda_stream)
    assert 0 < dp.info.walk_serial_bytes <= 2 * (256 << 10), dp.info.walk_serial_bytes
    assert dp.info.nframes == hp.info.nframes and dp.info.index_status == hp.info.index_status == 0
    assert _decode(dp, d_src, dev) == _decode(hp, d_src, dev)
    hp.close()
    dp.close()


def test_device_descriptors(tmp_path):
    """SURVEY §8f1's rest: when the device walk's chains meet (no stitch) and no
    frame goes to K4J, zd_plan_create_device builds the descriptors on the GPU
    (zd_k_plan_count / zd_k_plan_fill: the host planner's own per-frame pass,
    zd_plan.h) and reads back only the totals and the frames' output offsets
    and capacities (info.device_descriptors).  The plan equals the host
    planner's descriptor for descriptor, with and without -p, and decodes the
    same; a C4-shaped plan of 2,048 single-block frames, the host-walk inputs
    with skippable frames or a failing frame, and plans with K4J frames (a
    single frame of many blocks, few multi-block frames, 16-block frames in a
    larger plan) take that path."""
    import torch
    import test_host_walk
    from zstd_decompressor.batch import Plan
    dev = torch.device("cuda", 0)
    inputs = dict(test_host_walk._inputs())
    c4 = gen.frames(gen.text(64 << 20, seed=94), 128 << 10, 3)          # 512 frames
    cases = [("c4 x4", c4 * 4, True), ("intact", inputs["intact"], True), ("skippable", inputs["skippable"], True)]
    for i in range(6):
        cases.append((f"corrupt {i}", inputs[f"corrupt {i}"], False))
    # plans with K4J frames (round 5: their descriptors are built on the GPU
    # too): a c3s-shaped single frame of many blocks, a plan of <= 64 frames
    # of 2+ blocks each, and 16-block frames in a larger plan
    from corpus import libzstd
    big = gen.text(24 << 20, seed=95)
    few = b"".join(gen.frames(big[i << 20:(i + 1) << 20], 1 << 20, 9) for i in range(6))
    many = gen.frames(gen.text(80 << 20, seed=96), 2 << 20, 3) + c4[: len(c4) // 4]
    cases += [("c3s-shaped single frame", libzstd.compress(big, 3), True), ("few multi-block frames", few, True),
              ("16-block frames among single-block ones", many, True)]
    took = 0
    for name, data, must in cases:
        for skip in (False, True):
            d_src = torch.zeros(len(data) + 64, dtype=torch.uint8, device=dev)
            d_src[: len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
            torch.cuda.synchronize(dev)
            hp, hd = _dump(str(tmp_path / "h.bin"), lambda: Plan(data, skip))
            dp, dd = _dump(str(tmp_path / "d.bin"),
                           lambda: Plan.from_device(d_src.data_ptr(), len(data), skip,
                                                    stream=torch.cuda.current_stream(dev).cuda_stream))
            assert hp.info.device_descriptors == 0
            assert not must or dp.info.device_descriptors == 1, f"{name}: the device build was not taken"
            took += dp.info.device_descriptors
            assert dd == hd, f"{name} (-p {skip}): device descriptors differ from the host planner's"
            if not skip:
                assert _decode(dp, d_src, dev) == _decode(hp, d_src, dev), name
            hp.close()
            dp.close()
    assert took >= 12
