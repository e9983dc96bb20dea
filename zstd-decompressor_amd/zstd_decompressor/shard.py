"""Frame-sharded multi-GPU decode.

Frames are independent: each gets a fresh DecodingContext (frame.rs:232-237)
and the CLI only concatenates frame outputs (src/main.rs:43-53).  So ranks
take contiguous frame ranges balanced by compressed bytes, each rank decodes
its range into its own HBM with the batch plan (no collective on the data
path), and the decoded ranges are gathered to rank 0 with point-to-point
sends — RCCL over xGMI for device tensors (backend "nccl"), gloo on CPU.

One process per GPU; torch.distributed must already be initialised by the
caller (torchrun / init_process_group) when world > 1.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch


def partition(sizes: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous [begin, end) item ranges, one per rank, cut where the
    running sum of `sizes` crosses k/world of the total (every range is
    non-empty while there are at least `world` items)."""
    import bisect
    n = len(sizes)
    if world <= 0:
        raise ValueError("world must be positive")
    prefix = [0]
    for s in sizes:
        prefix.append(prefix[-1] + s)
    total = prefix[-1]
    cuts = [0]
    for k in range(1, world):
        # first item boundary whose prefix reaches k/world of the bytes
        c = bisect.bisect_left(prefix, -(-total * k // world))
        if n >= world:                       # leave one item for each remaining rank
            c = max(c, cuts[-1] + 1)
            c = min(c, n - (world - k))
        cuts.append(min(max(c, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


def partition_native(sizes: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """The same cut through the C ABI (zd_shard_partition), which a host
    binding (e.g. the reference's Rust CLI) calls."""
    import ctypes as C
    from . import _lib
    arr = (C.c_uint64 * max(len(sizes), 1))(*sizes)
    cuts = (C.c_size_t * (world + 1))()
    _lib.check(_lib.lib().zd_shard_partition(arr, len(sizes), world, cuts), "zd_shard_partition")
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


def cuts(data: bytes, world: int) -> Tuple[List[int], List[int]]:
    """(src_cuts, frame_cuts), world + 1 entries each: every rank's byte and
    frame range from one walk of the input (zd_shard_cuts).  Made on one rank
    and broadcast, so the others walk only their own frames (range_at)."""
    import ctypes as C
    from . import _lib
    p, n, keep = _lib.buf(data)
    sc, fc = (C.c_uint64 * (world + 1))(), (C.c_uint64 * (world + 1))()
    _lib.check(_lib.lib().zd_shard_cuts(p, n, world, sc, fc), "zd_shard_cuts")
    return list(sc), list(fc)


def range_at(data: bytes, src_cuts: Sequence[int], frame_cuts: Sequence[int], rank: int,
             world: int) -> Tuple[int, int, int, int]:
    """shard_of's (src_begin, src_end, frame_begin, frame_end) from given cuts,
    walking only this rank's frames (zd_shard_range_at); raises if the cuts
    are not this input's."""
    import ctypes as C
    from . import _lib
    p, n, keep = _lib.buf(data)
    sc = (C.c_uint64 * (world + 1))(*src_cuts)
    fc = (C.c_uint64 * (world + 1))(*frame_cuts)
    v = [C.c_uint64() for _ in range(4)]
    _lib.check(_lib.lib().zd_shard_range_at(p, n, sc, fc, rank, world, *[C.byref(x) for x in v]),
               "zd_shard_range_at")
    return tuple(x.value for x in v)


class Comm:
    """zd_comm: libzd's own RCCL communicator (one GPU per rank).  The id is
    made on rank 0 and broadcast over an initialised torch.distributed group."""

    def __init__(self, rank: int, world: int, device, group=None):
        import ctypes as C
        import torch.distributed as dist
        from . import _lib
        L = _lib.lib()
        idb = (C.c_uint8 * _lib.COMM_ID_BYTES)()
        if rank == 0:
            _lib.check(L.zd_comm_unique_id(idb), "zd_comm_unique_id")
        t = torch.tensor(list(idb), dtype=torch.uint8, device=device)
        dist.broadcast(t, 0, group=group)
        idb = (C.c_uint8 * _lib.COMM_ID_BYTES)(*t.cpu().tolist())
        h = C.c_void_p()
        _lib.check(L.zd_comm_create(idb, world, rank, C.byref(h)), "zd_comm_create")
        self._h, self.rank, self.world = h, rank, world

    def gather(self, d_local: int, length: int, status: int, first_error_frame: int, d_root: int,
               root_cap: int, stream: int = 0):
        """zd_comm_gather -> (call status, GatherResult)."""
        import ctypes as C
        from . import _lib
        res = _lib.GatherResult()
        st = _lib.lib().zd_comm_gather(self._h, C.c_void_p(d_local), length, status, first_error_frame,
                                       C.c_void_p(d_root), root_cap, C.byref(res), C.c_void_p(stream))
        return st, res

    def close(self):
        if getattr(self, "_h", None):
            from . import _lib
            _lib.lib().zd_comm_destroy(self._h)
            self._h = None


def shard_of(frames: Sequence[dict], rank: int, world: int) -> Tuple[int, int, int, int]:
    """(src_begin, src_end, frame_begin, frame_end) of this rank's frames, as
    given by zstd_decompressor.batch.frames_index."""
    ranges = partition([f["src_size"] for f in frames], world)
    b, e = ranges[rank]
    if b == e:
        off = frames[b]["src_offset"] if b < len(frames) else (
            frames[-1]["src_offset"] + frames[-1]["src_size"] if frames else 0)
        return off, off, b, e
    return frames[b]["src_offset"], frames[e - 1]["src_offset"] + frames[e - 1]["src_size"], b, e


def gather_to_root(local: torch.Tensor, length: int, rank: int, world: int, group=None) -> Optional[torch.Tensor]:
    """Concatenate every rank's first `length` bytes of `local` (uint8, 1-D) on
    rank 0, in rank order.  Lengths are exchanged first (all_gather), then
    each peer sends its range to rank 0 (point-to-point; over RCCL each send
    rides the peer's own xGMI link to GPU 0).  Returns the concatenation on
    rank 0 and None elsewhere."""
    import torch.distributed as dist
    if world == 1:
        return local[:length]
    dev = local.device
    lens = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(lens, torch.tensor([length], dtype=torch.int64, device=dev), group=group)
    lens = [int(t.item()) for t in lens]
    if rank == 0:
        out = torch.empty(sum(lens), dtype=torch.uint8, device=dev)
        out[: lens[0]].copy_(local[: lens[0]])
        off = lens[0]
        reqs = []
        for r in range(1, world):
            if lens[r]:
                reqs.append(dist.irecv(out[off: off + lens[r]], src=r, group=group))
            off += lens[r]
        for q in reqs:
            q.wait()
        return out
    if length:
        dist.send(local[:length].contiguous(), dst=0, group=group)
    return None


def global_status(status: int, first_frame: int, rank: int, world: int, device, group=None):
    """The whole input's outcome from every rank's own one, on every rank.

    The reference's CLI stops at the first frame that fails and keeps the
    frames before it (src/main.rs:43-53, FrameIterator frame.rs:94-99); ranks
    hold contiguous frame ranges in order, so that frame is the first failing
    one of the lowest failing rank.  Returns (status, first_error_frame or -1,
    failing rank or world): ranks after the failing one contribute nothing."""
    if world == 1:
        return status, first_frame if status else -1, 0 if status else world
    import torch.distributed as dist
    mine = torch.tensor([status, first_frame], dtype=torch.int64, device=device)
    alls = [torch.zeros(2, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(alls, mine, group=group)
    for r, t in enumerate(alls):
        st, ff = (int(x) for x in t.tolist())
        if st != 0:
            return st, ff, r
    return 0, -1, world


def decode_sharded(data: bytes, rank: int, world: int, device: torch.device, group=None,
                   gather: bool = True):
    """Decode this rank's share of the frames of `data` on `device` (one GPU
    per rank) and optionally gather the whole output on rank 0.

    Returns (status, local_output_tensor, local_length, gathered_or_None).
    status is the whole input's (global_status): a failure on any rank fails
    every rank, and the gathered output stops at the first failing frame,
    keeping the frames before it, like the reference CLI."""
    from .batch import Plan, frames_index
    frames, _, st, _ = frames_index(data)
    if st != 0:
        raise ValueError(f"frame index failed with status {st}")
    sb, se, fb, _ = shard_of(frames, rank, world)
    part = data[sb:se]
    length = 0
    status, first = 0, -1
    local = torch.empty(1, dtype=torch.uint8, device=device)
    if part:
        plan = Plan(part)
        cap = max(int(plan.info.out_bytes), 1)
        d_src = torch.zeros(len(part) + 64, dtype=torch.uint8, device=device)
        d_src[: len(part)].copy_(torch.frombuffer(bytearray(part), dtype=torch.uint8))
        local = torch.empty(cap + 64, dtype=torch.uint8, device=device)
        s = torch.cuda.current_stream(device).cuda_stream
        plan.decode_async(d_src.data_ptr(), local.data_ptr(), cap, s)
        torch.cuda.synchronize(device)
        status, length, _, _, first = plan.results(local.data_ptr(), s)
        plan.close()
    gst, _, length, gathered = collect(local, length, status, fb + first if status else -1, rank, world,
                                       group, gather)
    return gst, local, length, gathered


def collect(local: torch.Tensor, length: int, status: int, first_frame: int, rank: int, world: int,
            group=None, gather: bool = True):
    """Every rank's decode outcome -> (global status, first error frame,
    this rank's output length after the cut, gathered output on rank 0 or
    None).  A rank after the first failing one outputs nothing; the failing
    rank keeps the frames before its failure (its zd_plan_results length)."""
    gst, gfirst, frank = global_status(status, first_frame, rank, world, local.device, group)
    if rank > frank:
        length = 0
    gathered = gather_to_root(local, length, rank, world, group) if gather else None
    return gst, gfirst, length, gathered
