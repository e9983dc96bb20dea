"""Corrupt-input hardening of the C ABI, after the reference's libFuzzer
target (zstd-decompressor/fuzz/fuzz_targets/fuzz_target_1.rs: iterate the
frames of arbitrary bytes, decode each, never crash).  Seeded structure-aware
mutations of valid frames (header fields, block headers, literal/sequence
section headers, splices, truncations, random tails) go through the GPU path;
every input must come back with the oracle's status and bytes, and the process
must survive all of them.  ZD_E_OUT_OF_DOMAIN (a limit of the GPU path,
DESIGN.md) fails a campaign; ZD_FUZZ_DUMP=DIR keeps such inputs."""
import os
import random

import pytest

from corpus import gen, libzstd
from oracle import oracle

pytestmark = pytest.mark.gpu
OUT_OF_DOMAIN = -91


def _seeds():
    src = gen.text(120_000, seed=5)
    return [gen.frames(src, 40_000, 1), gen.frames(src, 60_000, 9, checksum=True),
            gen.frames(gen.xml(50_000, seed=2), 50_000, 19), libzstd.compress(bytes(4000), 3),
            gen.frames(gen.binary(30_000, seed=3), 30_000, 3)]


def _mutate(r: random.Random, seeds):
    d = bytearray(r.choice(seeds))
    kind = r.randrange(6)
    if kind == 0:                       # header region bit flips (frame header, first block header)
        for _ in range(r.randrange(1, 4)):
            i = r.randrange(min(len(d), 24))
            d[i] ^= 1 << r.randrange(8)
    elif kind == 1:                     # literal / sequence section headers of the first block
        for _ in range(r.randrange(1, 3)):
            i = r.randrange(6, min(len(d), 64))
            d[i] = r.randrange(256)
    elif kind == 2:                     # random bytes anywhere
        for _ in range(r.randrange(1, 8)):
            d[r.randrange(len(d))] = r.randrange(256)
    elif kind == 3:                     # splice two seeds at random points
        e = r.choice(seeds)
        d = d[: r.randrange(len(d))] + e[r.randrange(len(e)):]
    elif kind == 4:                     # truncation
        d = d[: r.randrange(len(d))]
    else:                               # valid magic, random body
        d = bytearray(b"\x28\xb5\x2f\xfd" + bytes(r.randrange(256) for _ in range(r.randrange(1, 300))))
    return bytes(d)


def _dump_ood(data, p, tag):
    """ZD_FUZZ_DUMP=DIR keeps every input that left the GPU path's domain."""
    d = os.environ.get("ZD_FUZZ_DUMP")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"{tag}_p{int(p)}.zst"), "wb") as f:
            f.write(data)


def test_fuzz_structure_aware():
    """ZD_FUZZ_ITERS / ZD_FUZZ_SEED run longer campaigns (default: 600 inputs).
    A quarter of the inputs build their tables on K1's lanes (ZD_F_K1_LANES),
    the rest on the wave-per-block build of small plans; a third decode their
    sequences on K3Q (ZD_F_SEQ_NO_LATENCY), the rest on K3L, small plans'
    default chain."""
    from zstd_decompressor import _lib
    from zstd_decompressor.batch import decompress_status
    iters = int(os.environ.get("ZD_FUZZ_ITERS", "600"))
    r = random.Random(int(os.environ.get("ZD_FUZZ_SEED", str(0xF022)), 0))
    seeds = _seeds()
    seen = {"ok": 0, "err": 0, "ood": 0}
    for it in range(iters):
        data = _mutate(r, seeds)
        p = r.random() < 0.3
        flags = _lib.F_K1_LANES if r.random() < 0.25 else 0
        flags |= _lib.F_SEQ_NO_LATENCY if r.random() < 0.33 else 0
        ost, oout = oracle.decompress_status(data, p)
        gst, gout = decompress_status(data, p, flags)
        if gst == OUT_OF_DOMAIN:
            seen["ood"] += 1
            _dump_ood(data, p, f"s{it}")
            continue
        assert gst == ost, f"#{it}: oracle {ost}, gpu {gst}"
        assert gout == oout, f"#{it}: output differs"
        seen["ok" if ost == 0 else "err"] += 1
    print("fuzz outcome counts:", seen)
    assert seen["ood"] == 0, seen


def test_fuzz_forked_plans():
    """The same mutations spliced into the middle of a 300-frame plan.  Plans
    of 256-768 frames take the few-frames path: K1's two halves and K2 | K3
    on two streams, K4F (zd_host.cpp FORK_* / K4F_AUTO_*).  Inputs this size
    also take the threaded header walk.  ZD_FUZZ_PLAN_ITERS runs longer
    campaigns (default: 40 inputs)."""
    from zstd_decompressor.batch import decompress_status, frames_index
    iters = int(os.environ.get("ZD_FUZZ_PLAN_ITERS", "40"))
    r = random.Random(int(os.environ.get("ZD_FUZZ_SEED", str(0xF022)), 0) + 1)
    seeds = _seeds()
    src = gen.text(300 * 4096, seed=8)
    base = gen.frames(src, 4096, 3)
    spans = [(f["src_offset"], f["src_size"]) for f in frames_index(base)[0]]
    assert len(spans) == 300
    seen = {"ok": 0, "err": 0, "ood": 0}
    for it in range(iters):
        o, n = spans[r.randrange(16, 284)]
        data = base[:o] + _mutate(r, seeds) + base[o + n:]
        p = r.random() < 0.3
        ost, oout = oracle.decompress_status(data, p)
        gst, gout = decompress_status(data, p)
        if gst == OUT_OF_DOMAIN:
            seen["ood"] += 1
            _dump_ood(data, p, f"plan{it}")
            continue
        assert gst == ost, f"#{it}: oracle {ost}, gpu {gst}"
        assert gout == oout, f"#{it}: output differs"
        seen["ok" if ost == 0 else "err"] += 1
    print("fuzz outcome counts (plans):", seen)
    assert seen["ood"] == 0, seen


def _seeds_multi_block():
    """Frames of several blocks (the block-parallel executor K4J's inputs)."""
    src = gen.text(700_000, seed=12)
    return [libzstd.compress(src[:450_000], 3), libzstd.compress(gen.xml(300_000, seed=13), 19),
            libzstd.compress(gen.binary(260_000, seed=14), 1), gen.frames(src, 300_000, 9)]


def test_fuzz_block_parallel():
    """The mutations on frames of several blocks, half of them forced onto
    K4J (ZD_F_BLOCK_PARALLEL: scatter checks, pointer-jumping rounds, the
    per-block prefix of repeat offsets), the rest on the automatic routing
    (K4J for frames of >= 2 compressed blocks in plans of <= 64 frames).
    ZD_FUZZ_ITERS / 4 inputs (default 150)."""
    from zstd_decompressor import _lib
    from zstd_decompressor.batch import decompress_status
    iters = int(os.environ.get("ZD_FUZZ_ITERS", "600")) // 4
    r = random.Random(int(os.environ.get("ZD_FUZZ_SEED", str(0xF022)), 0) + 2)
    seeds = _seeds_multi_block()
    seen = {"ok": 0, "err": 0, "ood": 0}
    for it in range(iters):
        data = _mutate(r, seeds)
        p = r.random() < 0.3
        flags = _lib.F_BLOCK_PARALLEL if r.random() < 0.5 else 0
        ost, oout = oracle.decompress_status(data, p)
        gst, gout = decompress_status(data, p, flags)
        if gst == OUT_OF_DOMAIN:
            seen["ood"] += 1
            _dump_ood(data, p, f"bp{it}")
            continue
        assert gst == ost, f"#{it}: oracle {ost}, gpu {gst}"
        same = gout == oout                           # (no pytest diff of large bytes)
        assert same, f"#{it}: output differs ({len(gout)} vs {len(oout)} bytes)"
        seen["ok" if ost == 0 else "err"] += 1
    print("fuzz outcome counts (block-parallel):", seen)
    assert seen["ood"] == 0, seen


# (seed, input index) of campaign inputs that once disagreed with the oracle
REGRESSIONS = [
    (6, 4281),     # runaway Huffman-weight stream before a reserved sequence-mode bit: oracle REF_PANIC
    # (seed 601: inputs that left the GPU path's domain before round 3)
    (601, 1103),   # Huffman tree of maxBits > 12, an absent node reached: REF_PANIC (deep_build)
    (601, 1140),
    (601, 2459),
    (601, 36),     # streams decode 53 literals past Regenerated_Size: re-planned with room
    (601, 1046),
    (601, 1307),   # back-to-back streams end within 16 bytes past R (K2's slack now past them)
    (601, 1531),   # frame decodes past its Frame_Content_Size: re-planned with 4x capacity
    (601, 2835),
    (601, 2183),
]


def test_fuzz_regressions():
    from zstd_decompressor.batch import decompress_status
    seeds = _seeds()
    for seed, idx in REGRESSIONS:
        r = random.Random(seed)
        for _ in range(idx + 1):
            data = _mutate(r, seeds)
            p = r.random() < 0.3
        ost, oout = oracle.decompress_status(data, p)
        gst, gout = decompress_status(data, p)
        assert gst == ost, f"seed {seed} #{idx}: oracle {ost}, gpu {gst}"
        assert gout == oout, f"seed {seed} #{idx}: output differs"
