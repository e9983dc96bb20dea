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


@pytest.mark.gpu
def test_decode_sharded_single_rank_gpu():
    from corpus import gen
    src = gen.text(2 << 20, seed=3)
    data = gen.frames(src, 128 << 10, 3)
    st, local, n, gathered = shard.decode_sharded(data, 0, 1, torch.device("cuda", 0))
    assert st == 0 and n == len(src)
    assert bytes(gathered.cpu().numpy().tobytes()) == src
