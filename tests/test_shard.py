"""Frame sharding across ranks: partition balance, and the
gather of decoded ranges to rank 0 over torch.distributed — gloo on CPU with
world_size 2 and 3 here; the GPU leg (RCCL) runs the same code on device
tensors.  No decode happens in the CPU tests (that needs the HIP path); the
ranks gather the oracle-free source slices their frames cover, which is
exactly what decode_sharded hands to gather_to_root."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from zstd_decompressor import shard


def test_partition_covers_and_balances():
    sizes = [5, 1, 1, 1, 9, 2, 2, 2, 2, 8, 3, 3]
    for world in range(1, 8):
        rs = shard.partition(sizes, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(sizes)
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        assert all(e - b >= 1 for b, e in rs)           # every rank gets a frame
    # equal sizes split evenly
    assert shard.partition([1] * 80, 8) == [(10 * k, 10 * k + 10) for k in range(8)]
    # more ranks than items: empty tail ranges, still a cover
    rs = shard.partition([3, 4], 4)
    assert rs[0][0] == 0 and rs[-1][1] == 2 and sum(e - b for b, e in rs) == 2


def test_native_partition_matches():
    """zd_shard_partition (the C ABI a host binding calls) cuts exactly where
    shard.partition does; zd_shard_range gives shard_of's byte ranges."""
    import random
    import ctypes as C
    from zstd_decompressor import _lib
    r = random.Random(3)
    for trial in range(300):
        n = r.randrange(0, 40)
        sizes = [r.choice([1, 2, 3, 100, 5000, 1 << 20, 1 << 33]) for _ in range(n)]
        for world in (1, 2, 3, 4, 7, 8):
            assert shard.partition_native(sizes, world) == shard.partition(sizes, world), (sizes, world)
    from corpus import gen
    from zstd_decompressor.batch import frames_index
    data = gen.frames(gen.text(3 << 20, seed=2), 100_000, 1)
    frames = frames_index(data)[0]
    p, n, keep = _lib.buf(data)
    for world in (1, 3, 8):
        for rank in range(world):
            v = [C.c_uint64() for _ in range(4)]
            _lib.check(_lib.lib().zd_shard_range(p, n, rank, world, *[C.byref(x) for x in v]))
            assert tuple(x.value for x in v) == shard.shard_of(frames, rank, world)
    # a frame that fails to index: it and the rest of the input go to the last rank
    bad = data[: frames[20]["src_offset"]] + b"\x00\x01\x02\x03" + data[frames[20]["src_offset"]:]
    v = [C.c_uint64() for _ in range(4)]
    _lib.check(_lib.lib().zd_shard_range(*_lib.buf(bad)[:2], 2, 3, *[C.byref(x) for x in v]))
    assert v[1].value == len(bad) and v[3].value == 20


def test_shard_of_real_frames():
    from corpus import gen
    from zstd_decompressor.batch import frames_index
    src = gen.text(1 << 20, seed=11)
    data = gen.frames(src, 128 << 10, 3)
    frames, _, st, _ = frames_index(data)
    assert st == 0 and len(frames) == 8
    spans = [shard.shard_of(frames, r, 3) for r in range(3)]
    assert spans[0][0] == 0 and spans[-1][1] == len(data)
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, payloads, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = payloads[rank]
        local = torch.frombuffer(bytearray(mine + b"\xAA" * 7), dtype=torch.uint8)  # slack past the length
        out = shard.gather_to_root(local, len(mine), rank, world)
        if rank == 0:
            q.put(bytes(out.numpy().tobytes()))
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_to_root_gloo(world):
    from corpus import gen
    from zstd_decompressor.batch import frames_index
    src = gen.text(1 << 20, seed=5)
    data = gen.frames(src, 128 << 10, 3)
    frames, _, _, _ = frames_index(data)
    # each rank's decoded range = the source bytes of its frames (FCS layout)
    payloads = []
    for r in range(world):
        _, _, fb, fe = shard.shard_of(frames, r, world)
        a = sum(f["content_size"] for f in frames[:fb])
        b = a + sum(f["content_size"] for f in frames[fb:fe])
        payloads.append(src[a:b])
    payloads[-1] = payloads[-1] if world < 3 else b""      # an empty rank too
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, payloads, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == b"".join(payloads)


def _worker_fail(rank, world, port, payloads, statuses, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = payloads[rank]
        st, first = statuses[rank]
        local = torch.frombuffer(bytearray(mine + b"\x55" * 5), dtype=torch.uint8)
        gst, gfirst, n, out = shard.collect(local, len(mine), st, first, rank, world)
        q.put((rank, gst, gfirst, n, None if out is None else bytes(out.numpy().tobytes())))
    finally:
        dist.destroy_process_group()


def test_collect_stops_at_first_failing_rank():
    """A failure on a middle rank: every rank reports that rank's status and
    frame, rank 0 gets the frames before it (the failing rank's partial
    output) and nothing of the ranks after it (src/main.rs:43-53)."""
    world = 3
    payloads = [b"frames of rank 0|", b"rank 1 before its failure|", b"rank 2 frames, after the failure"]
    statuses = [(0, -1), (-42, 17), (0, -1)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_fail, args=(r, world, port, payloads, statuses, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    for _ in range(world):
        r, gst, gfirst, n, out = q.get(timeout=120)
        got[r] = (gst, gfirst, n, out)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert got[r][:2] == (-42, 17)
    assert got[2][2] == 0
    assert got[0][3] == payloads[0] + payloads[1]


@pytest.mark.gpu
def test_decode_sharded_single_rank_gpu():
    from corpus import gen
    src = gen.text(2 << 20, seed=3)
    data = gen.frames(src, 128 << 10, 3)
    st, local, n, gathered = shard.decode_sharded(data, 0, 1, torch.device("cuda", 0))
    assert st == 0 and n == len(src)
    assert bytes(gathered.cpu().numpy().tobytes()) == src


def test_bench_strong_shards_cover_the_corpus():
    """bench.py's strong-scaling split (one corpus, contiguous frame ranges of
    the replicated frame set): the ranks' compressed bytes and expected
    outputs concatenate to the whole corpus and its source."""
    import bench
    from corpus import gen
    from zstd_decompressor.batch import frames_index
    src = gen.text(1 << 20, seed=17)
    frame_set = gen.frames(src, 100_000, 3)
    frames = frames_index(frame_set)[0]
    reps = 3
    n = len(frames) * reps
    for world in (1, 2, 5, 8):
        ranges = shard.partition([frames[k % len(frames)]["src_size"] for k in range(n)], world)
        parts = [bench.shard_bytes(frame_set, frames, src, reps, b, e) for b, e in ranges]
        assert b"".join(p[0] for p in parts) == frame_set * reps
        assert b"".join(p[1] for p in parts) == src * reps
    assert bench.host_cores()[0] >= 1


def _comm_world1_worker(port, q):
    import torch.distributed as dist
    from oracle import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        import ctypes as C
        from zstd_decompressor import _lib
        comm = shard.Comm(0, 1, dev)
        payload = torch.arange(0, 1 << 20, dtype=torch.int64, device=dev).to(torch.uint8)
        root = torch.zeros((1 << 20) + 64, dtype=torch.uint8, device=dev)
        st, res = comm.gather(payload.data_ptr(), 1 << 20, 0, -1, root.data_ptr(), root.numel(),
                              torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        ok1 = st == 0 and res.status == 0 and res.total_len == 1 << 20 and bool(torch.equal(root[:1 << 20], payload))
        # the whole sharded decode through the C ABI, on the reference's sample
        data = open(os.path.join(os.path.dirname(__file__), "golden", "resources", "moby-dick.txt.zst"), "rb").read()
        expect = oracle.decompress(data)
        out = torch.zeros(len(expect) + 64, dtype=torch.uint8, device=dev)
        res2 = _lib.GatherResult()
        p, n, keep = _lib.buf(data)
        st2 = _lib.lib().zd_decode_sharded(comm._h, p, n, 0, C.c_void_p(out.data_ptr()), out.numel(), C.byref(res2),
                                           C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        ok2 = st2 == 0 and res2.status == 0 and res2.total_len == len(expect) and \
            bytes(out[:len(expect)].cpu().numpy().tobytes()) == expect
        # the same through given cuts (zd_decode_sharded_at), and cuts that
        # are not the input's: the collective completes, res.status says so
        sc, fc = shard.cuts(data, 1)
        csc, cfc = (C.c_uint64 * 2)(*sc), (C.c_uint64 * 2)(*fc)
        out.zero_()
        res2 = _lib.GatherResult()
        st2 = _lib.lib().zd_decode_sharded_at(comm._h, p, n, csc, cfc, 0, C.c_void_p(out.data_ptr()), out.numel(),
                                              C.byref(res2), C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        ok2 = ok2 and st2 == 0 and res2.status == 0 and res2.total_len == len(expect) and \
            bytes(out[:len(expect)].cpu().numpy().tobytes()) == expect
        cfc[1] += 1
        st2 = _lib.lib().zd_decode_sharded_at(comm._h, p, n, csc, cfc, 0, C.c_void_p(out.data_ptr()), out.numel(),
                                              C.byref(res2), C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        ok2 = ok2 and st2 == 0 and res2.status == _lib.INVALID_ARG and res2.total_len == 0
        # inputs that take zd_plan_decompress's re-plan, a > 12-bit Huffman
        # tree and a corrupt middle frame, each against the oracle (status,
        # first failing frame, output of the frames before it)
        bad = []
        for name, data in _sharded_cases():
            ost, oout = oracle.decompress_status(data, False)
            cap = max(len(oout), 1) + 64
            for root_cap in (cap, 16):          # in place at the root / through the comm's buffer
                out = torch.zeros(cap, dtype=torch.uint8, device=dev)
                res3 = _lib.GatherResult()
                p, n, keep = _lib.buf(data)
                st3 = _lib.lib().zd_decode_sharded(comm._h, p, n, 0, C.c_void_p(out.data_ptr()), root_cap,
                                                   C.byref(res3), C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
                torch.cuda.synchronize(dev)
                if root_cap < len(oout):
                    if not (st3 == _lib.DST_TOO_SMALL or res3.status == _lib.DST_TOO_SMALL or len(oout) == 0):
                        bad.append((name, "small root", st3, res3.status))
                    continue
                got = bytes(out[:res3.total_len].cpu().numpy().tobytes())
                if st3 != 0 or res3.status != ost or got != oout:
                    bad.append((name, st3, res3.status, ost, res3.total_len, len(oout)))
        comm.close()
        # a rank-0 re-plan that outgrows the lent root buffer: the comm's own
        # output buffer is sized from what the re-plan needs, not from root_cap
        # (a fresh comm, so no earlier buffer is reused)
        from zstd_decompressor.batch import Plan
        data, need = _late_overrun_case()
        ost, oout = oracle.decompress_status(data, False)
        pl = Plan(data)
        root_cap = int(pl.info.out_bytes) + 64
        pl.close()
        assert need > root_cap and len(oout) <= need
        comm = shard.Comm(0, 1, dev)
        out = torch.zeros(len(oout) + 64, dtype=torch.uint8, device=dev)
        res4 = _lib.GatherResult()
        p, n, keep = _lib.buf(data)
        st4 = _lib.lib().zd_decode_sharded(comm._h, p, n, 0, C.c_void_p(out.data_ptr()), root_cap, C.byref(res4),
                                           C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        torch.cuda.synchronize(dev)
        sb, ob = C.c_uint64(), C.c_uint64()
        _lib.check(_lib.lib().zd_comm_buffers(comm._h, C.byref(sb), C.byref(ob)), "zd_comm_buffers")
        # the output itself comes back through the gather into `out`: root_cap
        # is short of it, so the call reports DST_TOO_SMALL or decodes in full
        if not (st4 == _lib.DST_TOO_SMALL or res4.status == _lib.DST_TOO_SMALL or
                (st4 == 0 and bytes(out[:res4.total_len].cpu().numpy().tobytes()) == oout)):
            bad.append(("late overrun", st4, res4.status))
        if not (need <= ob.value < root_cap + root_cap // 2):
            bad.append(("late overrun buffer", ob.value, need, root_cap))
        comm.close()
        q.put((ok1, ok2, bad))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_comm_gather_and_sharded_decode_world1_gpu():
    """libzd's RCCL communicator (zd_comm_create / zd_comm_gather) and the
    one-call zd_decode_sharded, on one GPU (world 1: the RCCL calls run, the
    sends are to self).  The N>1 legs run in the driver's multi-GPU bench."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_comm_world1_worker, args=(_free_port(), q))
    p.start()
    got = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert got == (True, True, [])


def _lower_fcs(frame: bytes, fcs: int) -> bytes:
    """A libzstd frame whose Frame_Content_Size field claims `fcs` bytes (the
    reference checks no FCS, decoding_context.rs:29-47: it decodes the whole
    frame; the GPU plan reserves fcs bytes and must re-plan)."""
    fhd = frame[4]
    single = (fhd >> 5) & 1
    flen = {0: 1 if single else 0, 1: 2, 2: 4, 3: 8}[fhd >> 6]
    at = 5 + (0 if single else 1) + {0: 0, 1: 1, 2: 2, 3: 4}[fhd & 3]
    assert flen >= 4, "a frame with a 4- or 8-byte FCS field"
    return frame[:at] + fcs.to_bytes(flen, "little") + frame[at + flen:]


def _sharded_cases():
    """Inputs for zd_decode_sharded against the oracle: an FCS-overrun frame
    in the middle (re-planned, twice over), a > 12-bit Huffman tree frame (K2's
    interval decode), a corrupt middle frame (the output stops before it)."""
    import random
    from corpus import gen
    from test_gpu_parity import _deep_tree_frame
    src = gen.text(1 << 20, seed=23)
    fr = [gen.frames(src[i * 100_000:(i + 1) * 100_000], 100_000, 3) for i in range(8)]
    r = random.Random(5)
    deep = next(f for f in (_deep_tree_frame(r, r.randrange(20, 200), list(range(13, 0, -1))) for _ in range(200))
                if oracle_status(f) == 0)
    corrupt = None
    for at in range(len(fr[3]) // 2, len(fr[3]) - 4):    # the first flip the reference rejects
        c = bytearray(fr[3])
        c[at] ^= 0x5A
        if oracle_status(bytes(c)) != 0:
            corrupt = c
            break
    return [
        ("fcs overrun", b"".join(fr[:3]) + _lower_fcs(fr[3], 3000) + b"".join(fr[4:])),
        ("fcs overrun x2", fr[0] + _lower_fcs(fr[1], 100) + _lower_fcs(fr[2], 70_000) + fr[3]),
        ("deep tree", fr[0] + deep + fr[1] + deep + fr[2]),
        ("corrupt middle", b"".join(fr[:3]) + bytes(corrupt) + b"".join(fr[4:])),
    ]


def _late_overrun_case():
    """40 frames of 100,000 bytes, frame 38 claiming an FCS of 3000: the plan
    reserves 3,903,000 bytes, the re-plan from frame 38 on needs the 3,800,000
    before it plus 3000 + 1 MiB for it (zd_host.cpp decode_resident) plus
    frame 39's 100,000.  Returns (input, bytes the re-plan needs)."""
    from corpus import gen
    src = gen.text(4_000_000, seed=29)
    fr = [gen.frames(src[i * 100_000:(i + 1) * 100_000], 100_000, 3) for i in range(40)]
    need = 38 * 100_000 + 3000 + (1 << 20) + 100_000
    return b"".join(fr[:38]) + _lower_fcs(fr[38], 3000) + fr[39], need


def oracle_status(data: bytes) -> int:
    from oracle import oracle
    return oracle.decompress_status(data, False)[0]


def test_sharded_cases_are_what_they_claim():
    """Host: the oracle decodes the FCS-overrun inputs fully (past their FCS),
    and the corrupt-middle input fails at its fourth frame."""
    from oracle import oracle
    cases = dict(_sharded_cases())
    for k in ("fcs overrun", "fcs overrun x2", "deep tree"):
        st, out = oracle.decompress_status(cases[k], False)
        assert st == 0 and len(out) > 0, k
    st, out = oracle.decompress_status(cases["corrupt middle"], False)
    assert st != 0 and len(out) == 300_000


def _layout_py(meta, world):
    """shard.collect's rule on all-gathered outcomes: (status, first frame,
    failing rank, kept lengths)."""
    failed = next((r for r in range(world) if meta[r][0] != 0), world)
    lens = [meta[r][2] if r <= failed else 0 for r in range(world)]
    st = meta[failed][0] if failed < world else 0
    first = meta[failed][1] if failed < world else -1
    return st, first, failed, lens


def _layout_c(meta, world):
    import ctypes as C
    from zstd_decompressor import _lib
    flat = (C.c_int64 * (4 * world))(*[v for row in meta for v in row])
    off = (C.c_uint64 * world)()
    ln = (C.c_uint64 * world)()
    res = _lib.GatherResult()
    st = _lib.lib().zd_gather_layout(flat, world, off, ln, C.byref(res))
    return st, res, list(off), list(ln)


def test_gather_layout_host_only():
    """zd_gather_layout (the merge every rank of zd_comm_gather runs on the
    all-gathered outcomes; host only, so it runs here) against shard.collect's
    rule at world 1/2/3/8: clean, a failing middle rank, a failing rank 0 and
    last rank, empty ranks, and rank 0's capacity limit."""
    import random
    from zstd_decompressor import _lib
    r = random.Random(8)
    for world in (1, 2, 3, 8):
        for trial in range(200):
            lens = [r.choice([0, 1, 17, 4096, 1 << 20]) for _ in range(world)]
            sts = [0] * world
            fail = r.choice([None] + list(range(world)))
            if fail is not None:
                sts[fail] = r.choice([_lib.IMPOSSIBLE_VALUE, _lib.NOT_ENOUGH_BYTES, _lib.OUT_OF_DOMAIN])
                if r.random() < 0.5 and fail + 1 < world:
                    sts[r.randrange(fail + 1, world)] = _lib.NULL_OFFSET     # a later failure does not count
            firsts = [r.randrange(0, 1000) if s else -1 for s in sts]
            need = sum(lens[: (fail if fail is not None else world - 1) + 1])
            cap = r.choice([need, need + 5, max(need - 1, 0), 1 << 40])
            meta = [[sts[k], firsts[k], lens[k], cap if k == 0 else 0] for k in range(world)]
            st, first, failed, klens = _layout_py(meta, world)
            cst, res, off, ln = _layout_c(meta, world)
            assert (res.status, res.first_error_frame, res.failed_rank) == (st, first, failed)
            if sum(klens) > cap:
                assert cst == _lib.DST_TOO_SMALL and res.total_len == 0
            else:
                assert cst == 0 and res.total_len == sum(klens)
                assert ln == klens and off == [sum(klens[:k]) for k in range(world)]


def _worker_layout(rank, world, port, payloads, statuses, cap, q):
    """Every rank: shard.collect over gloo (the Python gather) and the C-ABI
    merge on the same all-gathered outcomes; both must agree on every rank."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = payloads[rank]
        st, first = statuses[rank]
        meta = torch.tensor([st, first if st else -1, len(mine), cap if rank == 0 else 0], dtype=torch.int64)
        alls = [torch.zeros(4, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(alls, meta)
        cst, res, off, ln = _layout_c([t.tolist() for t in alls], world)
        local = torch.frombuffer(bytearray(mine + b"\x55" * 3), dtype=torch.uint8)
        gst, gfirst, n, out = shard.collect(local, len(mine), st, first, rank, world)
        q.put((rank, cst, res.status, res.first_error_frame, res.total_len, off, ln, gst, gfirst, n,
               None if out is None else bytes(out.numpy().tobytes())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fail,short", [(2, None, False), (3, 1, False), (8, 5, False), (8, None, True)])
def test_gather_layout_multi_rank_gloo(world, fail, short):
    """zd_comm_gather's merge at world 2/3/8 on CPU ranks (gloo), beside
    shard.collect: the same status / first failing frame on every rank, each
    rank's kept length, rank 0's offsets tile the gathered bytes, and a short
    root capacity refuses on every rank (nothing would be sent)."""
    from zstd_decompressor import _lib
    payloads = [bytes([65 + r]) * (100 + 37 * r) for r in range(world)]
    statuses = [(0, -1)] * world
    if fail is not None:
        statuses[fail] = (_lib.IMPOSSIBLE_VALUE, 1000 + fail)
    upto = (fail if fail is not None else world - 1) + 1
    need = sum(len(p) for p in payloads[:upto])
    cap = need - 1 if short else need
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_layout, args=(r, world, port, payloads, statuses, cap, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    for _ in range(world):
        v = q.get(timeout=180)
        got[v[0]] = v[1:]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        cst, rst, rfirst, total, off, ln, gst, gfirst, n, out = got[r]
        assert (rst, rfirst) == (gst, gfirst)
        assert ln[r] == n                                   # the kept length matches collect's cut
        if short:
            assert cst == _lib.DST_TOO_SMALL and total == 0
        else:
            assert cst == 0 and total == need
    if not short:
        out = got[0][-1]
        _, _, _, _, off, ln, *_ = got[0]
        assert out == b"".join(payloads[:upto])
        assert all(out[off[k]: off[k] + ln[k]] == payloads[k][: ln[k]] for k in range(world))


def _cut_input():
    from corpus import gen
    return gen.frames(gen.text(3 << 20, seed=2), 100_000, 1)


def test_shard_cuts_and_range_at_host():
    """zd_shard_cuts gives every rank zd_shard_range's range from one walk;
    zd_shard_range_at takes those cuts and walks only the rank's own frames:
    it still gives the same range with every byte outside the range zeroed
    (so it reads nothing there), and rejects cuts that are not the input's."""
    import ctypes as C
    from zstd_decompressor import _lib
    data = _cut_input()
    p, n, keep = _lib.buf(data)
    for world in (1, 2, 3, 8, 41):
        sc, fc = shard.cuts(data, world)
        assert len(sc) == len(fc) == world + 1 and sc[0] == 0 and sc[-1] == len(data)
        for rank in range(world):
            v = [C.c_uint64() for _ in range(4)]
            _lib.check(_lib.lib().zd_shard_range(p, n, rank, world, *[C.byref(x) for x in v]))
            want = tuple(x.value for x in v)
            assert (sc[rank], sc[rank + 1], fc[rank], fc[rank + 1]) == want
            assert shard.range_at(data, sc, fc, rank, world) == want
            b, e = sc[rank], sc[rank + 1]
            blind = bytes(b) + data[b:e] + bytes(len(data) - e)
            assert shard.range_at(blind, sc, fc, rank, world) == want
    sc, fc = shard.cuts(data, 4)
    for bad_sc, bad_fc in (([sc[0], sc[1] + 1] + sc[2:], fc),           # a cut inside a frame
                           (sc, [fc[0], fc[1] + 1] + fc[2:]),           # a wrong frame count
                           (sc[:-1] + [len(data) + 1], fc)):            # past the input
        with pytest.raises(Exception):
            for rank in range(4):
                shard.range_at(data, bad_sc, bad_fc, rank, 4)
    # a frame that fails to index: it and the rest go to the last rank, whose
    # range_at accepts a range that ends in it
    from zstd_decompressor.batch import frames_index
    frames = frames_index(data)[0]
    bad = data[: frames[20]["src_offset"]] + b"\x00\x01\x02\x03" + data[frames[20]["src_offset"]:]
    sc, fc = shard.cuts(bad, 3)
    assert sc[-1] == len(bad) and fc[-1] == 20
    for rank in range(3):
        v = [C.c_uint64() for _ in range(4)]
        _lib.check(_lib.lib().zd_shard_range(*_lib.buf(bad)[:2], rank, 3, *[C.byref(x) for x in v]))
        assert shard.range_at(bad, sc, fc, rank, 3) == tuple(x.value for x in v)


def _worker_cuts(rank, world, port, q):
    """Rank 0 walks the input once (zd_shard_cuts) and broadcasts the cuts;
    every rank then takes its range with zd_shard_range_at, walking only its
    own frames, and compares it with today's whole-input zd_shard_range."""
    import ctypes as C
    import torch.distributed as dist
    from zstd_decompressor import _lib
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = _cut_input()
        t = torch.zeros(2 * (world + 1), dtype=torch.int64)
        if rank == 0:
            sc, fc = shard.cuts(data, world)
            t = torch.tensor(sc + fc, dtype=torch.int64)
        dist.broadcast(t, 0)
        sc, fc = t[: world + 1].tolist(), t[world + 1:].tolist()
        got = shard.range_at(data, sc, fc, rank, world)
        v = [C.c_uint64() for _ in range(4)]
        p, n, keep = _lib.buf(data)
        _lib.check(_lib.lib().zd_shard_range(p, n, rank, world, *[C.byref(x) for x in v]))
        q.put((rank, got, tuple(x.value for x in v)))
    finally:
        dist.destroy_process_group()


def test_shard_range_at_gloo_world8():
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_cuts, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    for _ in range(world):
        r, a, b = q.get(timeout=180)
        got[r] = (a, b)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert got[r][0] == got[r][1]
    assert got[0][0][0] == 0 and all(got[r][0][1] == got[r + 1][0][0] for r in range(world - 1))
