"""Benchmark: decompressed MB/s of the MI355X ZSTD block-decode path.

Workload (default `c4`, BASELINE.json configs[3]): enwik-style synthetic
text, 128 KiB independent frames at zstd level 3, a 1 GiB unique frame set
replicated to one 10 GiB corpus (SURVEY.md §8d allows replication).  One
step = one zd_decode_async over the whole resident share (K1 tables -> K2
Huffman -> K3 FSE -> K4 execute).  Inputs are resident in HBM before timing;
output is verified bit-exact against the source bytes after timing.

Multi-GPU (torchrun, one process per GPU): by default the one 10 GiB corpus
is split into contiguous frame ranges balanced by compressed bytes
(shard.partition, zd_shard_partition), each rank planning and decoding only
its range — no data-path collective ("scaling": "strong", value = all
ranks' bytes / the slowest rank's time).  The gather of every rank's output
to rank 0 over RCCL (libzd's zd_comm_gather) is timed after that and
reported apart.  `--scaling weak` gives every rank its own 10 GiB corpus.

Other workloads: c2 (one 64 MiB raw/RLE frame), c3 (enwik8 shape in 763
frames), c3s (the same 100,000,000 bytes as ONE frame, `zstd -3 enwik8`:
block-parallel executor K4J), c5 (1 MiB eight-block frames, --level 1/9/19).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "zstd-decompressor_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_corpus(workload: str, unique_bytes: int, seed: int, level: int = 9, c2_mib: int = 64):
    from corpus import gen, libzstd
    t0 = time.time()
    if workload == "c2":
        data, src = gen.c2_raw_rle(c2_mib << 20, with_content=True)
        return data, src, 1, {"frames": 1, "frame_bytes": c2_mib << 20}, time.time() - t0
    if workload == "c3":
        # C3 (BASELINE.json configs[2]): enwik8-style, 100,000,000 bytes in
        # 763 independent 128 KiB frames at level 3; few frames, so it
        # measures the latency-bound regime (not replicated)
        src = gen.text(100_000_000, seed=seed)[:100_000_000]
        data = gen.frames(src, 128 << 10, 3)
        return data, src, 1, {"frame_bytes": 128 << 10, "level": 3}, time.time() - t0
    if workload == "c3s":
        # the same 100,000,000 bytes as the stock CLI writes them: ONE frame
        # (763 blocks, windowLog 21), executed block-parallel (K4J)
        src = gen.text(100_000_000, seed=seed)[:100_000_000]
        data = libzstd.compress(src, 3)
        return data, src, 1, {"frames": 1, "level": 3}, time.time() - t0
    if workload == "c5":
        # Silesia-style mix (BASELINE.json configs[4]): xml, dickens-like
        # prose and mozilla-like binary, a third each, 1 MiB frames
        third = (unique_bytes // 3) >> 20 << 20
        src = gen.xml(third, seed=seed) + gen.text(third, seed=seed + 1) + gen.binary(unique_bytes - 2 * third, seed=seed + 2)
        data = gen.frames(src, 1 << 20, level)
        return data, src, None, {"frame_bytes": 1 << 20, "level": level}, time.time() - t0
    src = gen.text(unique_bytes, seed=seed)
    data = gen.frames(src, 128 << 10, 3)
    return data, src, None, {"frame_bytes": 128 << 10, "level": 3}, time.time() - t0


def host_cores():
    """(threads for the CPU baseline, note).  BASELINE.md §3 asks for every host
    core; a container's share can be smaller than os.cpu_count() (the GPU box
    shows the whole machine there), so the cores this process may run on
    (affinity, then a cgroup v2 CPU quota) bound it."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    note = f"os.cpu_count()={os.cpu_count()}, affinity={n}"
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
            note += f", cgroup cpu.max quota={quota}"
            n = min(n, quota)
    except (OSError, ValueError):
        pass
    return max(1, n), note


def shard_bytes(frame_set: bytes, frames, src, reps: int, begin: int, end: int):
    """The compressed bytes and the source bytes of global frames [begin, end)
    of `frame_set` replicated `reps` times (frame k = frame k % F of the set)."""
    F = len(frames)
    coff = [0]
    for f in frames:
        coff.append(coff[-1] + f["content_size"])
    data, ref = [], []
    k = begin
    while k < end:
        i = k % F
        run = min(end - k, F - i)                      # contiguous inside one replica
        a, b = frames[i]["src_offset"], frames[i + run - 1]["src_offset"] + frames[i + run - 1]["src_size"]
        data.append(frame_set[a:b])
        if src is not None:
            ref.append(src[coff[i]:coff[i + run]])
        k += run
    return b"".join(data), (b"".join(ref) if src is not None else None)


def cpu_baseline(frame_set: bytes, threads: int, budget_s: float = 20.0):
    """The oracle (C restatement of the reference decoder, kind "port") over a
    bounded sample of the same frames, frames spread over `threads` threads."""
    from oracle import oracle
    from zstd_decompressor.batch import frames_index
    frames, _, st, _ = frames_index(frame_set)
    spans = [(f["src_offset"], f["src_size"]) for f in frames]
    # calibrate on a few frames, then size the sample to ~budget_s of CPU work
    t0 = time.time()
    out0 = 0
    for o, s in spans[:8]:
        out0 += len(oracle.frame_decode(frame_set[o:o + s])[1])
    per_byte = (time.time() - t0) / max(out0, 1)
    want = int(budget_s * threads / max(per_byte, 1e-12))
    sizes = [f["content_size"] if f["content_size"] is not None and f["content_size"] >= 0 else 128 << 10
             for f in frames]
    sample, acc = [], 0
    i = 0
    while acc < want and i < len(spans) * 4:
        o, s = spans[i % len(spans)]
        sample.append((o, s))
        acc += sizes[i % len(spans)]
        i += 1

    def work(chunk):
        n = 0
        for o, s in chunk:
            n += len(oracle.frame_decode(frame_set[o:o + s])[1])
        return n

    parts = [sample[k::threads] for k in range(threads)]
    t0 = time.time()
    with cf.ThreadPoolExecutor(threads) as ex:
        total_out = sum(ex.map(work, parts))
    dt = time.time() - t0
    # one host thread as well (SURVEY.md §8d i), on the head of the sample (~3 s)
    t1, out1, k1 = time.time(), 0, 0
    while k1 < len(sample) and time.time() - t1 < 3.0:
        out1 += work(sample[k1:k1 + 16])
        k1 += 16
    dt1 = time.time() - t1
    res = {"value": round(total_out / dt / 1e6, 2), "unit": "MB/s", "cores": threads, "kind": "port",
           "value_1thread": round(out1 / dt1 / 1e6, 2),
           "sample": f"{len(sample)} frames ({total_out / 2**20:.0f} MiB decoded) of the same corpus, "
                     f"oracle/zd_oracle.c on {threads} host threads, {dt:.1f} s; value_1thread: "
                     f"{min(k1, len(sample))} frames on one thread, {dt1:.1f} s"}
    return res, (sample, [sizes[k % len(spans)] for k in range(len(sample))])


def cpu_libzstd(frame_set: bytes, sample, threads: int):
    """Context only (not the contract's cpu_baseline): the system libzstd,
    an optimised RFC decoder (SURVEY.md §8d ii), on the same frame sample."""
    import ctypes as C
    from corpus import libzstd
    L = libzstd.lib()
    spans, sizes = sample
    buf = C.create_string_buffer(frame_set, len(frame_set))
    base = C.addressof(buf)

    def work(idx):
        n = 0
        for k in idx:
            (o, s), cap = spans[k], sizes[k]
            out = C.create_string_buffer(cap)
            r = L.ZSTD_decompress(out, cap, base + o, s)
            if L.ZSTD_isError(r):
                raise RuntimeError(L.ZSTD_getErrorName(r))
            n += r
        return n
    parts = [list(range(k, len(spans), threads)) for k in range(threads)]
    t0 = time.time()
    with cf.ThreadPoolExecutor(threads) as ex:
        total = sum(ex.map(work, parts))
    dt = time.time() - t0
    return {"value": round(total / dt / 1e6, 2), "unit": "MB/s", "cores": threads,
            "sample": f"the cpu_baseline sample ({total / 2**20:.0f} MiB), libzstd "
                      f"{L.ZSTD_versionNumber()} ZSTD_decompress on {threads} host threads, {dt:.2f} s"}


plan_io_scratch = []


def host_io_leg(plan, data: bytes, info, src, reps: int):
    """zd_plan_decompress (host in, host out; the INTEGRATION.md decompress())
    on the bench plan: two warm calls, then the best of two timed, phase
    times from zd_plan_info io_*_ns; the output checked against the source.
    Plus the same on the reference's moby-dick sample (one small frame:
    latency, not bandwidth).  Reported apart from value (PCIe-inclusive)."""
    import ctypes as C
    from zstd_decompressor import _lib
    L = _lib.lib()
    cap = int(info.out_bytes)
    out = np.empty(cap + 64, dtype=np.uint8)
    plan_io_scratch.append(out)
    p, n, keep = _lib.buf(data)
    ol = C.c_size_t()
    best = None
    for it in range(4):
        t0 = time.time()
        st = L.zd_plan_decompress(plan._h, p, n, C.c_void_p(out.ctypes.data), cap, C.byref(ol))
        dt = time.time() - t0
        pi = _lib.PlanInfo()
        L.zd_plan_info_get(plan._h, C.byref(pi))
        if st != 0 or ol.value != cap:
            return {"error": f"zd_plan_decompress status {st}, {ol.value} of {cap} bytes"}
        if it >= 2 and (best is None or dt < best[0]):
            best = (dt, pi.io_h2d_ns / 1e6, pi.io_decode_ns / 1e6, pi.io_d2h_ns / 1e6)
    ok = None
    if src is not None:
        u = len(src)
        mv = memoryview(out)
        ok = all(mv[r * u:(r + 1) * u] == src for r in range(reps))
    dt, h2d, dec, d2h = best
    res = {"MBps": round(cap / dt / 1e6, 1), "wall_ms": round(dt * 1e3, 2), "h2d_ms": round(h2d, 2),
           "h2d_GBps": round(n / (h2d / 1e3) / 1e9, 1), "decode_ms": round(dec, 2), "d2h_ms": round(d2h, 2),
           "d2h_GBps": round(cap / (d2h / 1e3) / 1e9, 1), "verified_bit_exact": ok,
           "via": "zd_plan_decompress: pinned 32 MiB chunks, host copies on the worker pool, plan-owned device buffers"}
    # the reference's own sample, host in / host out
    from zstd_decompressor.batch import Plan
    md = open(os.path.join(ROOT, "tests", "golden", "resources", "moby-dick.txt.zst"), "rb").read()
    mp = Plan(md)
    mcap = int(mp.info.out_bytes)
    mout = np.empty(mcap + 64, dtype=np.uint8)
    mpp, mn, mkeep = _lib.buf(md)
    times = []
    for it in range(12):
        t0 = time.time()
        st = L.zd_plan_decompress(mp._h, mpp, mn, C.c_void_p(mout.ctypes.data), mcap, C.byref(ol))
        times.append(time.time() - t0)
    mp.close()
    tm = float(np.median(times[2:]))
    res["moby_dick"] = {"MBps": round(mcap / tm / 1e6, 1), "wall_ms": round(tm * 1e3, 3), "status": int(st),
                        "bytes": mcap}
    return res


def traffic_of(kernel: str, args, world: int):
    """HBM bytes per launch of `kernel` (FETCH_SIZE + WRITE_SIZE, rocprofv3
    --pmc passes of scripts/full_run.sh on the default 1-GPU workload, kept
    with the commit they measured in profiles/traffic.json); None for other
    workloads or when absent."""
    if (args.workload, args.unique_mib, args.replicas, world) != ("c4", 1024, 10, 1):
        return None
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        k = json.load(open(path))["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None
    return None if not k else round(k["traffic"] / 1e9, 3)


def traffic_commit():
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "traffic.json"))).get("commit")
    except (OSError, ValueError):
        return None


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(argv, n: int, port: int):
    """The command and environment that run this bench as `n` ranks, one
    process per GPU (torch.distributed.run on 127.0.0.1), with the same
    arguments.  The children see WORLD_SIZE and take the rank path."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # RCCL needs dmabuf IPC on these hosts
    env.setdefault("OMP_NUM_THREADS", "1")
    return cmd, env


def maybe_launch(argv) -> int | None:
    """`--gpus N` (N > 1) without a launcher: start the N ranks as ONE child
    process group (torchrun) before anything touches the GPU, forward their
    output (rank 0 prints the JSON line) and return their exit code.  Under
    a launcher (WORLD_SIZE set) return None and check WORLD_SIZE == N."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dry-run-launch", action="store_true")
    a, _ = ap.parse_known_args(argv)
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        assert int(world) == a.gpus or a.gpus == 1 and "--gpus" not in " ".join(argv), \
            f"WORLD_SIZE={world} but --gpus {a.gpus}"
        return None
    if a.gpus <= 1:
        return None
    fwd = [x for x in argv if x != "--dry-run-launch"]
    cmd, env = launch_command(fwd, a.gpus, free_port())
    if a.dry_run_launch:
        print(json.dumps({"cmd": cmd, "env": {k: env[k] for k in ("HSA_ENABLE_IPC_MODE_LEGACY", "OMP_NUM_THREADS")}}))
        return 0
    import subprocess
    log(f"[launch] {a.gpus} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


def main():
    rc = maybe_launch(sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    ap = argparse.ArgumentParser()
    ap.add_argument("--dry-run-launch", action="store_true", help="N>1: print the rank launch command and exit")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c4", choices=["c4", "c2", "c3", "c3s", "c5"])
    ap.add_argument("--level", type=int, default=9, help="c5: zstd level (1 / 9 / 19)")
    ap.add_argument("--unique-mib", type=int, default=1024, help="unique decompressed MiB before replication")
    ap.add_argument("--replicas", type=int, default=10)
    ap.add_argument("--c2-mib", type=int, default=64,
                    help="c2: frame size in MiB (BASELINE configs[1]: 64, inside the 256 MiB Infinity Cache; "
                         "1024 makes its roofline an HBM figure)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="N>1: one corpus split across the ranks (strong) or one corpus per rank (weak)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--graph", action="store_true", help="time a captured HIP graph of the decode, not its launches")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every core this process may use")
    ap.add_argument("--corpus-cache", default=os.environ.get("ZD_CORPUS_CACHE"),
                    help="directory to keep the generated corpus in between runs (experiments)")
    ap.add_argument("--gather", choices=["auto", "on", "off"], default="auto",
                    help="N>1: time gathering every rank's output to rank 0 over RCCL, reported apart "
                         "(auto: on for strong scaling)")
    ap.add_argument("--no-host-io", action="store_true",
                    help="skip the host-in / host-out leg (profiling runs of the device path)")
    ap.add_argument("--share", default=None, metavar="R/N",
                    help="one GPU, one process: decode only rank R's frame range of the N-way strong partition "
                         "(the share one rank of an N-GPU run decodes, measured alone; no gather)")
    ap.add_argument("--overlap-streams", type=int, default=0, metavar="N",
                    help="also time the corpus as N contiguous frame chunks, each its own plan on its own stream "
                         "(K1/K2 of one chunk beside K3/K4 of another; reported apart, never value)")
    ap.add_argument("--experiment", action="store_true",
                    help="timing-only variants: do not stop on decode errors")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import zstd_decompressor as zd  # noqa: F401
    from zstd_decompressor import shard
    from zstd_decompressor.batch import Plan, frames_index

    # ---- corpus (host) ----
    # --share R/N: this process plays rank R of an N-way strong split
    prank, pworld = (int(args.share.split("/")[0]), int(args.share.split("/")[1])) if args.share else (rank, world)
    assert world == 1 or not args.share, "--share is a one-process option"
    strong = pworld > 1 and args.scaling == "strong" and args.workload != "c3s"
    seed = 0x5EED + (0 if (strong or world == 1) else 7919 * rank)
    cache = None
    if args.corpus_cache:
        os.makedirs(args.corpus_cache, exist_ok=True)
        lv = f"_L{args.level}" if args.workload == "c5" else (f"_{args.c2_mib}" if args.workload == "c2" else "")
        cache = os.path.join(args.corpus_cache, f"{args.workload}{lv}_{args.unique_mib}_{seed}")
    if cache and os.path.exists(cache + ".zst"):
        frame_set = open(cache + ".zst", "rb").read()
        src = open(cache + ".src", "rb").read() if os.path.exists(cache + ".src") else None
        reps_override, tgen = (1 if args.workload in ("c2", "c3", "c3s") else None), 0.0
    else:
        frame_set, src, reps_override, meta, tgen = make_corpus(args.workload, args.unique_mib << 20, seed, args.level,
                                                                    args.c2_mib)
        if cache:
            open(cache + ".zst", "wb").write(frame_set)
            if src is not None:
                open(cache + ".src", "wb").write(src)
    reps = reps_override or args.replicas
    set_frames = frames_index(frame_set)[0]
    n_global = len(set_frames) * reps
    if strong:
        # one corpus, contiguous frame ranges balanced by compressed bytes
        ranges = shard.partition([set_frames[k % len(set_frames)]["src_size"] for k in range(n_global)], pworld)
        fb, fe = ranges[prank]
        data, ref_bytes = shard_bytes(frame_set, set_frames, src, reps, fb, fe)
    else:
        fb, fe = 0, n_global
        data, ref_bytes = frame_set * reps, None
    log(f"[rank {rank}] corpus: {len(frame_set) / 2**20:.1f} MiB compressed x{reps}, gen {tgen:.1f}s; "
        f"this rank: frames [{fb}, {fe}) of {n_global}, {len(data) / 2**20:.1f} MiB")

    # the host plan (frame/block header walk, descriptors, workspace
    # allocation and upload) is built once per input, outside the timed
    # region; its wall time is reported beside value as host_plan_ms
    # (a plan over the first frame first: HIP runtime / code-object set-up is
    # a one-time process cost, not part of planning an input)
    f0 = set_frames[0]
    Plan(frame_set[f0["src_offset"]:f0["src_offset"] + f0["src_size"]]).close()
    t0 = time.time()
    plan = Plan(data)
    host_plan_first_s = time.time() - t0
    # steady state: the plan of a next input of this shape (the destroyed
    # plan's device workspace is reused from libzd's cache, zd_trim_cache)
    plan.close()
    t0 = time.time()
    plan = Plan(data)
    host_plan_s = time.time() - t0
    info = plan.info
    log(f"[rank {rank}] plan: {info.nframes} frames, {info.ncompressed} compressed blocks, "
        f"{info.nsequences} sequences, out {info.out_bytes / 2**30:.2f} GiB, ws {info.workspace_bytes / 2**30:.2f} GiB, "
        f"{time.time() - t0:.2f}s")
    assert info.out_exact and info.index_status == 0

    d_src = torch.empty(len(data) + 64, dtype=torch.uint8, device=dev)
    d_src[: len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    d_dst = torch.empty(info.out_bytes + 64, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    # the same plan with the frame/block header walk on the GPU
    # (zd_plan_create_device: the input is resident in HBM), warm
    dev_plan_ms = None
    if not args.experiment:
        torch.cuda.synchronize(dev)
        for _ in range(2):
            t0 = time.time()
            dplan = Plan.from_device(d_src.data_ptr(), len(data), stream=sptr)
            dev_plan_ms = (time.time() - t0) * 1e3
            dinfo = dplan.info
            dplan.close()
            assert (dinfo.nframes, dinfo.nblocks, dinfo.nsequences, dinfo.out_bytes) == \
                (info.nframes, info.nblocks, info.nsequences, info.out_bytes)

    def step():
        plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), info.out_bytes, sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    st, total, _, _, first = plan.results(d_dst.data_ptr(), sptr)
    assert args.experiment or (st == 0 and total == info.out_bytes), (st, total, first)

    # --graph: the timed steps replay one decode captured in a HIP graph
    # (zd_decode_async is graph-safe: no allocation, no host memory read, its
    # fork stream made at plan time; tests/test_gpu_parity.py
    # test_hip_graph_capture_replay).  Not the default: in the captured graph
    # the forked K2 ran before zd_k_fused instead of beside it (C3 2.07 ms a
    # step against 1.42) and a short step paid the graph launch (C2 64 MiB
    # 27 us against 19); profiles/r6_graph_replay_ab.txt.
    timed_step = step
    if args.graph:
        cap = torch.cuda.Stream(dev)
        graph = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(dev)
        with torch.cuda.graph(graph, stream=cap):
            plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), info.out_bytes, cap.cuda_stream)
        torch.cuda.synchronize(dev)
        timed_step = graph.replay
        for _ in range(args.warmup):
            timed_step()
        torch.cuda.synchronize(dev)

    # ---- timed region ----
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_wall = time.time()
    ev0.record(stream)
    for _ in range(args.steps):
        timed_step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    t_wall = time.time() - t_wall
    if dist:
        dist.barrier()
    ms_total = ev0.elapsed_time(ev1)
    elapsed = torch.tensor([ms_total], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    ms_per_step = float(elapsed.item()) / args.steps

    # ---- verify (outside timing): d_dst as the last timed step left it ----
    # (the timed configuration itself: fused kernel, K2 | K3 fork and all;
    # the profiled passes below run after this check)
    verified = None
    st, total, _, _, _ = plan.results(d_dst.data_ptr(), sptr)
    redo_frames = int(plan.refresh_info().fused_redo_frames)
    if not args.no_verify and src is not None:
        ok = st == 0 and total == info.out_bytes
        if strong:
            ref = torch.frombuffer(bytearray(ref_bytes), dtype=torch.uint8).to(dev)
            ok = ok and total == ref.numel() and bool(torch.equal(d_dst[:total], ref))
        else:
            ref = torch.frombuffer(bytearray(src), dtype=torch.uint8).to(dev)
            u = len(src)
            ok = ok and total == u * reps
            for r in range(reps):
                ok = ok and bool(torch.equal(d_dst[r * u:(r + 1) * u], ref))
        verified = bool(ok)
        del ref
        if dist:
            v = torch.tensor([1 if verified else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(v, op=dist.ReduceOp.MIN)
            verified = bool(v.item())
        assert args.experiment or verified, "GPU output differs from the source bytes"

    # ---- the dominant launch of the timed pipeline, as it runs: events on the
    # plan's stream around every launch group that carries work (K0, the
    # fused kernel, K4, K4F, the K4J kernels; fork and fusion kept), the
    # longest one is the roofline's kernel ----
    nprof = max(2, min(args.steps, 3))
    plan.set_profiling(2)
    dts = []
    for _ in range(nprof):
        step()
        dts.append(plan.kernel_times())
    plan.set_profiling(0)
    dom_all = {k: float(np.mean([d[k] for d in dts])) for k in dts[0]}
    dom = max(dom_all, key=dom_all.get)
    dom_ms = dom_all[dom]

    # ---- per-kernel breakdown (events between launches on the same stream:
    # the launches one after another, no fork, no fused kernel) ----
    plan.set_profiling(True)
    kt = {}
    for _ in range(nprof):
        step()
        for k, v in plan.kernel_times().items():
            kt.setdefault(k, []).append(v)
    plan.set_profiling(False)
    kt = {k: float(np.mean(v)) for k, v in kt.items()}

    # ---- chunks on parallel streams (an experiment: reported apart) ----
    overlap = None
    if args.overlap_streams > 1 and world == 1:
        N = args.overlap_streams
        fr = frames_index(data)[0]
        cut = [len(fr) * k // N for k in range(N + 1)]
        subs, ob = [], 0
        for k in range(N):
            a = fr[cut[k]]["src_offset"]
            b = fr[cut[k + 1] - 1]["src_offset"] + fr[cut[k + 1] - 1]["src_size"]
            sp = Plan(data[a:b])
            subs.append((sp, a, ob, torch.cuda.Stream(dev)))
            ob += int(sp.info.out_bytes)
        assert ob == info.out_bytes

        def ostep():
            ev = torch.cuda.Event()
            ev.record(stream)
            for sp, a, o, st_ in subs:
                st_.wait_event(ev)
                sp.decode_async(d_src.data_ptr() + a, d_dst.data_ptr() + o, int(sp.info.out_bytes), st_.cuda_stream)
            for sp, a, o, st_ in subs:
                e2 = torch.cuda.Event()
                e2.record(st_)
                stream.wait_event(e2)
        for _ in range(2):
            ostep()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):
            ostep()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        oms = e0.elapsed_time(e1) / args.steps
        ook = None
        if src is not None and not args.no_verify:
            ook = all(sp.results(d_dst.data_ptr() + o, st_.cuda_stream)[0] == 0 for sp, a, o, st_ in subs)
            ref = torch.frombuffer(bytearray(src), dtype=torch.uint8).to(dev)
            u = len(src)
            ook = ook and all(bool(torch.equal(d_dst[r * u:(r + 1) * u], ref)) for r in range(reps))
            del ref
        overlap = {"chunks": N, "ms_per_step": round(oms, 3), "MBps": round(info.out_bytes / (oms / 1e3) / 1e6, 1),
                   "vs_one_plan_ms": round(ms_per_step, 3), "verified_bit_exact": ook}
        for sp, a, o, st_ in subs:
            sp.close()

    # ---- gather of the decoded ranges to rank 0 over RCCL (never part of value) ----
    out_bytes = info.out_bytes
    comp_bytes = len(data)
    total_out = torch.tensor([float(out_bytes)], dtype=torch.float64, device=dev)
    total_alg = torch.tensor([float(out_bytes + comp_bytes)], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(total_out)
        dist.all_reduce(total_alg)
    gather = None
    if dist and (args.gather == "on" or (args.gather == "auto" and strong)):
        comm = shard.Comm(rank, world, dev)
        all_out = int(total_out.item())
        root = torch.empty(all_out + 64 if rank == 0 else 1, dtype=torch.uint8, device=dev)
        gst = None
        tg = []
        for it in range(3):                           # one warm-up, two timed
            dist.barrier()
            torch.cuda.synchronize(dev)
            t1 = time.time()
            cst, res = comm.gather(d_dst.data_ptr(), out_bytes, 0, -1, root.data_ptr(), all_out if rank == 0 else 0,
                                   sptr)
            torch.cuda.synchronize(dev)
            dt = torch.tensor([time.time() - t1], dtype=torch.float64, device=dev)
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            if it:
                tg.append(dt.item())
            gst = (cst, res.status, res.total_len)
        gms = min(tg) * 1e3
        gok = None
        if rank == 0 and not args.no_verify and src is not None:
            ref = torch.frombuffer(bytearray(src), dtype=torch.uint8).to(dev)
            u = len(src)
            gok = gst[0] == 0 and gst[1] == 0 and gst[2] == u * reps and all(
                bool(torch.equal(root[r * u:(r + 1) * u], ref)) for r in range(reps))
            del ref
        gather = {"gather_ms": round(gms, 3), "gathered_bytes": int(gst[2]),
                  "gather_GBps": round(gst[2] / (gms / 1e3) / 1e9, 1),
                  "decode_plus_gather_MBps": round(all_out / (ms_per_step / 1e3 + gms / 1e3) / 1e6, 1),
                  "via": "libzd zd_comm_gather (RCCL point-to-point to rank 0 over xGMI)",
                  "verified_bit_exact": gok}
        del root
        comm.close()

    # ---- the drop-in's host-in / host-out path (never part of value) ----
    # zd_plan_decompress on the same plan: input host -> HBM and output HBM ->
    # host through pinned chunks, plan-owned device buffers (rank 0 only, the
    # other ranks wait: one PCIe link measured alone)
    host_io = None
    if rank == 0 and not args.experiment and not args.no_host_io:
        host_io = host_io_leg(plan, data, info, src if not strong else ref_bytes, reps if not strong else 1)
        del plan_io_scratch[:]
    if dist:
        dist.barrier()

    value = total_out.item() / (ms_per_step / 1e3) / 1e6
    alg_per_launch = out_bytes + comp_bytes          # C + D, this rank's launch
    achieved = alg_per_launch / (dom_ms / 1e3) / 1e9
    # a fraction above 1 would mean the timed launch is not the one doing the
    # work (the algorithmic bytes cannot move faster than the HBM peak)
    assert args.experiment or achieved <= HBM_PEAK_GBS, (dom, dom_ms, achieved)

    cpu = cpu_zstd = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and src is not None:
        threads, note = host_cores()
        if args.cpu_threads:
            threads = args.cpu_threads
        cpu, sample = cpu_baseline(frame_set, threads)
        cpu["cores_note"] = note
        try:
            cpu_zstd = cpu_libzstd(frame_set, sample, threads)
        except Exception as ex:                     # context only: never fails the bench
            cpu_zstd = {"error": str(ex)[:200]}

    if rank == 0:
        wl = {"c4": "C4: enwik-style text, 128 KiB frames, zstd -3, 1 GiB unique x10 = one 10 GiB corpus",
              "c2": f"C2: single {args.c2_mib} MiB frame, {args.c2_mib * 8} alternating raw/RLE 128 KiB blocks",
              "c3": "C3: enwik8-style 100,000,000 B, 763 x 128 KiB frames, zstd -3",
              "c3s": "C3 single frame: enwik8-style 100,000,000 B as ONE zstd -3 frame (763 blocks)",
              "c5": f"C5: Silesia-style mix (xml / prose / binary thirds), 1 MiB multi-block frames, zstd -{args.level}, "
                    f"{args.unique_mib} MiB unique x{reps}"}[args.workload]
        if world > 1:
            wl += (f", frame-sharded across {world} GPUs" if strong else f", one such corpus per GPU ({world})")
        if args.share:
            wl += f", rank {prank}'s share of a {pworld}-way frame split, decoded alone on one GPU"
        res = {
            "metric": "decompressed MB/s (bit-exact vs ref) + % HBM roofline",
            "value": round(value, 1),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            # the one corpus split over the ranks (one rank: all of it), so the
            # N = 1 line and the N > 1 lines are the same strong-scaling series
            "scaling": "strong" if args.scaling == "strong" and args.workload != "c3s" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": wl,
                "frames_total": int(n_global) if strong else int(info.nframes) * world,
                "frames_rank0": int(info.nframes),
                "decompressed_bytes_total": int(total_out.item()),
                "decompressed_bytes_rank0": int(out_bytes),
                "compressed_bytes_rank0": int(comp_bytes),
                "sequences_rank0": int(info.nsequences),
                "compression_ratio": round(out_bytes / max(comp_bytes, 1), 3),
                "fidelity_note": "synthetic corpus (no enwik/Silesia offline): it compresses at compression_ratio, "
                                 "real enwik text at ~3.5-4x at these levels (SURVEY.md Appendix A), so each output "
                                 "byte here carries more sequences and literals than enwik9's would; value and "
                                 "roofline.frac are not directly comparable to a real-enwik run",
                "parallelism": (f"share {prank}/{pworld} alone" if args.share else
                                f"frame-sharded x{world}" if strong else f"replicas x{world}"),
                "step": "zd_decode_async over every resident frame" +
                        (", replayed from a captured HIP graph" if args.graph else ", launched per step"),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "kernel_ms": round(dom_ms, 3),
                "launch_groups_ms": {k: round(v, 3) for k, v in dom_all.items()},
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic_of(dom, args, world),
                "traffic_unit": "GB per launch (rocprofv3 2 x FETCH_SIZE + WRITE_SIZE, the x2 calibrated on K4's own "
                                "access patterns: profiles/r3_fetch_calibration.txt; profiles/traffic.json)",
                "traffic_commit": traffic_commit(),
                "alg_bytes_per_launch": int(alg_per_launch),
                "pipeline_achieved": round(alg_per_launch / (ms_per_step / 1e3) / 1e9, 1),
                "pipeline_frac": round(alg_per_launch / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            },
            "kernel_ms": {k: round(v, 3) for k, v in kt.items()},
            "kernel_ms_note": "kernel_ms: a profiled pass with the launches one after another (no K2 | K3 fork, "
                              "no fused kernel); roofline.kernel_ms: the dominant launch of the timed pipeline "
                              "as it runs (HIP events on its stream around it)",
            "fused_redo_frames": redo_frames,
            "host_plan_ms": round(host_plan_s * 1e3, 1),
            "host_plan_first_ms": round(host_plan_first_s * 1e3, 1),
            "device_walk_plan_ms": None if dev_plan_ms is None else round(dev_plan_ms, 1),
            "host_plan_split_ms": {"headers_and_descriptors": round(info.host_ns / 1e6, 1),
                                   "workspace_alloc_and_upload": round(info.device_ns / 1e6, 1)},
            "value_incl_host_plan": round(total_out.item() / (ms_per_step / 1e3 + host_plan_s) / 1e6, 1),
            # the same with the plan built on the GPU from the HBM-resident input
            # (zd_plan_create_device: header walk + descriptors), one plan per step
            "value_incl_device_plan": None if dev_plan_ms is None else
            round(total_out.item() / (ms_per_step / 1e3 + dev_plan_ms / 1e3) / 1e6, 1),
            "h2d_ms": None if not host_io else host_io["h2d_ms"],
            "d2h_ms": None if not host_io else host_io["d2h_ms"],
            "host_io": host_io,
            "cpu_baseline": cpu,
            "cpu_libzstd": cpu_zstd,
            "verified_bit_exact": verified,
        }
        if gather:
            res["gather_to_rank0"] = gather
        if overlap:
            res["overlap_streams"] = overlap
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
