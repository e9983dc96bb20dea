"""GPU parity: the HIP path (through the C ABI) against the oracle — the CPU
restatement of the reference decoder — on the same inputs.

Bit-exact output is required wherever the oracle succeeds; wherever it fails
the GPU path must fail too, with the same reference error variant.  A frame
past the GPU path's limits would report ZD_E_OUT_OF_DOMAIN: no
input here may.
"""
import random

import numpy as np
import pytest

from corpus import gen, libzstd
from oracle import oracle

pytestmark = pytest.mark.gpu

OUT_OF_DOMAIN = -91


def gpu(data, p=False, flags=0):
    from zstd_decompressor.batch import decompress_status
    return decompress_status(data, p, flags)


def assert_parity(data, p=False, what="", flags=0):
    """Status and output as the oracle's; ZD_E_OUT_OF_DOMAIN (a limit of the
    GPU path) fails the test."""
    ost, oout = oracle.decompress_status(data, p)
    gst, gout = gpu(data, p, flags)
    assert gst != OUT_OF_DOMAIN, f"{what}: out of the GPU path's domain (oracle status {ost})"
    if ost == 0:
        assert gst == 0, f"{what}: oracle ok, gpu status {gst}"
        assert gout == oout, f"{what}: output differs (len {len(gout)} vs {len(oout)})"
    else:
        assert gst == ost, f"{what}: oracle status {ost}, gpu status {gst}"
        assert gout == oout, f"{what}: partial output of the frames before the failure differs"
    return ost, gst


def test_kat_frames(kat):
    for c in kat["frames"]:
        data = bytes(c["data"])
        assert_parity(data, False, c["src"])
        assert_parity(data, True, c["src"])


def test_resources(resources):
    for name, data in resources.items():
        ost, _ = assert_parity(data, False, name)
        assert ost == 0
        assert_parity(data, True, name)


def test_execute_sequences_kat(kat):
    from zstd_decompressor import DecodingContext
    for c in kat["execute_sequences"]:
        ctx = DecodingContext(0x42)
        ctx.execute_sequences([tuple(s) for s in c["seqs"]], bytes(c["literals"]))
        assert ctx.decoded == bytes(c["out"]), c["src"]


def test_execute_sequences_large_values():
    """DecodingContext.execute_sequences with values past the direct records'
    packed fields (literals_length >= 2^17 - 1, match_length >= 2^18 - 1,
    offset_value >= 2^29 - 1): escape records whose exact triple the executor
    reads from a side array.  Long literal runs, long overlapping and
    non-overlapping matches, repeat codes after them, and offsets past the
    output (ImpossibleValue), against the oracle's DecodingContext."""
    import random
    from zstd_decompressor import DecodingContext, ZdError
    r = random.Random(77)
    lits = bytes(r.randrange(256) for _ in range(700_000))
    cases = [
        [(200_000, 4, 300_000)],                                   # a long literal run, then an RLE-like match
        [(131_071, 5000 + 3, 262_143), (0, 1, 7), (9, 2, 300_000), (3, 3, 12)],   # exactly at the field maxima
        [(150_000, 140_000 + 3, 140_000), (1, 1, 270_000), (70_000, 3, 5)],       # long copies, repeat codes
        [(10, (1 << 29) + 10, 4)],                                 # an offset past the output: ImpossibleValue
        [(262_144, 200_000 + 3, 1 << 18), (0, (1 << 31) + 7, 3)],  # a giant offset after a long run
        [(20, 4, 1), (0xFFFFFFF0, 4, 1)],                          # 20 + ll wraps 32 bits: ImpossibleValue
        [(0xFFFFFFFF, 4, 1)],                                      # the largest literals_length
        [(5, 4, 1)] * 63 + [(0xFFFFFFF0, 4, 1)] * 3 + [(1, 4, 1)], # wrapping lanes inside one batch
    ]
    for i, seqs in enumerate(cases):
        try:
            want, werr = oracle.execute_sequences(seqs, lits, cap=4 << 20), None
        except Exception as e:                                     # the oracle's error variant
            want, werr = None, getattr(e, "code", e)
        ctx = DecodingContext(8 << 20)
        try:
            ctx.execute_sequences(seqs, lits)
            got, gerr = ctx.decoded, None
        except ZdError as e:
            got, gerr = None, e.code
        ctx.close()
        assert (werr is None) == (gerr is None), f"case {i}: oracle {werr}, gpu {gerr}"
        if werr is None:
            same = got == want
            assert same, f"case {i}: {len(got)} vs {len(want)} bytes"
        else:
            assert gerr == werr, f"case {i}: oracle {werr}, gpu {gerr}"


def test_context_block_by_block(resources):
    """Block.parse + Block.decode(ctx) over moby-dick's blocks == Frame.decode
    (tests/block.rs usage pattern with DecodingContext::new(MAX_WIN_SIZE))."""
    from zstd_decompressor import ForwardByteParser, Block, DecodingContext, MAX_WIN_SIZE
    data = resources["moby-dick.txt.zst"]
    _, expect, _ = oracle.frame_decode(data)
    p = ForwardByteParser(data)
    p.slice(4)                                     # magic
    fhd = p.u8()                                   # Header::parse (frame.rs:111-177)
    single = bool(fhd & 0x20)
    if not single:
        p.u8()                                     # window descriptor
    fcs_len = {0: 1 if single else 0, 1: 2, 2: 4, 3: 8}[fhd >> 6]
    if fcs_len:
        p.slice(fcs_len)
    ctx = DecodingContext(MAX_WIN_SIZE)
    nblocks = 0
    while True:
        b, last = Block.parse(p)
        b.decode(ctx)
        nblocks += 1
        if last:
            break
    assert nblocks > 1
    assert ctx.decoded == expect


def test_context_window_too_big():
    from zstd_decompressor import DecodingContext, ZdError
    with pytest.raises(ZdError) as e:
        DecodingContext((8 << 20) + 1)
    assert e.value.name.startswith("WindowSizeTooBig")


@pytest.mark.parametrize("kind", ["text", "xml", "binary"])
@pytest.mark.parametrize("level", [1, 3, 9, 19])
def test_synthetic_single_block_frames(kind, level):
    src = {"text": gen.text, "xml": gen.xml, "binary": gen.binary}[kind](1 << 20 if level < 19 else 512 << 10)
    data = gen.frames(src, 128 << 10, level)
    ost, gst = assert_parity(data, False, f"{kind} L{level} 128K")
    assert ost == 0
    from zstd_decompressor import decompress
    assert decompress(data) == src


@pytest.mark.parametrize("kind", ["text", "xml", "binary"])
@pytest.mark.parametrize("level", [1, 9, 19])
def test_synthetic_multi_block_frames(kind, level):
    """C5 shape: 1 MiB frames of 8 blocks -> Treeless literals, Repeat modes,
    repeat offsets across blocks, matches into earlier blocks."""
    n = (2 << 20) if level < 19 else (1 << 20)
    src = {"text": gen.text, "xml": gen.xml, "binary": gen.binary}[kind](n, seed=level)
    data = gen.frames(src, 1 << 20, level)
    ost, gst = assert_parity(data, False, f"{kind} L{level} 1M")
    assert ost == 0


@pytest.mark.parametrize("mib", [8, 64])
def test_c2_raw_rle(mib):
    """C2 (BASELINE configs[1]): one raw/RLE-only frame; 64 MiB is the bench
    size (K0 copies the frame whole)."""
    data = gen.c2_raw_rle(mib << 20)
    ost, gst = assert_parity(data, False, f"c2 {mib} MiB")
    assert ost == 0


def test_checksum_and_no_fcs_frames():
    src = gen.text(300_000, seed=7)
    # checksum flag, and a frame without FCS (streaming API absent: emulate by
    # clearing the FCS flag is not valid; use libzstd output as is + checksum)
    data = gen.frames(src, 100_000, 3, checksum=True)
    assert_parity(data, False, "checksum")


def test_empty_and_tiny_frames():
    for n in (1, 2, 3, 5, 17, 100, 1000):
        src = bytes(random.Random(n).randrange(256) for _ in range(n))
        assert_parity(libzstd.compress(src, 3), False, f"tiny {n}")
    assert_parity(libzstd.compress(b"", 3), False, "empty frame (raw block of size 0)")
    assert_parity(libzstd.compress(b"a" * 100000, 3), False, "rle")
    assert_parity(libzstd.compress(b"ab" * 100000, 19), False, "period-2")


def test_out_of_domain_triggers():
    """SURVEY §2.1 D2/D3 triggers: the reference fails; so must the GPU path."""
    r = random.Random(3)
    letters = bytes(r.choice(b"abcdefghijklmnopqrstuvwxyz") for _ in range(65536))
    assert_parity(libzstd.compress(letters, 1), False, "D2 random letters L1")
    two = bytes(r.choice(b"ab") for _ in range(100000))
    assert_parity(libzstd.compress(two, 3), False, "D3 two symbols")
    ff = bytes(0xFF if r.random() < 0.5 else r.randrange(256) for _ in range(100000))
    assert_parity(libzstd.compress(ff, 3), False, "D3 0xFF heavy")


def test_corrupted_inputs():
    """Byte flips / truncations of valid frames: success/failure and error
    variant parity with the oracle (the reference's fuzz target, fuzz/)."""
    r = random.Random(1234)
    src = gen.text(200_000, seed=11)
    base = gen.frames(src, 64 << 10, 3) + gen.frames(gen.binary(100_000), 50_000, 9)
    stats = {"ok": 0, "err_same": 0}
    for it in range(300):
        d = bytearray(base)
        for _ in range(r.randrange(1, 4)):
            d[r.randrange(len(d))] = r.randrange(256)
        if r.random() < 0.2:
            d = d[: r.randrange(len(d))]
        ost, gst = assert_parity(bytes(d), False, f"corrupt #{it}")
        stats["ok" if ost == 0 else "err_same"] += 1
    assert stats["ok"] and stats["err_same"], stats


def test_corrupted_inputs_forked_plan():
    """Corruptions inside a 300-frame plan: plans of 256-768 frames take the
    few-frames path (K1's Huffman half + K2 on a second stream beside K1's
    sequence half + K3, then K4F; zd_host.cpp FORK_* / K4F_AUTO_*), whose
    error keys come from both streams.  Same first error and partial output
    as the oracle."""
    r = random.Random(77)
    src = gen.text(300 * 4096, seed=12)
    base = gen.frames(src, 4096, 3)
    from zstd_decompressor.batch import frames_index
    spans = [(f["src_offset"], f["src_size"]) for f in frames_index(base)[0]]
    assert len(spans) == 300
    assert_parity(base, False, "forked plan, intact")
    stats = {"ok": 0, "err_same": 0}
    for it in range(60):
        d = bytearray(base)
        o, n = spans[r.randrange(20, 280)]
        for _ in range(r.randrange(1, 4)):
            d[o + r.randrange(n)] = r.randrange(256)
        ost, gst = assert_parity(bytes(d), False, f"forked corrupt #{it}")
        stats["ok" if ost == 0 else "err_same"] += 1
    assert stats["ok"] and stats["err_same"], stats


def test_multi_block_frames_forked_plan():
    """C5-shaped frames (1 MiB, 8 blocks: Treeless literals, Repeat tables,
    repeat offsets across blocks) in a plan of 288 sequence blocks, which takes
    the forked path: K1's Huffman half builds the LUTs a Treeless block reuses
    (K2, second stream), its sequence half the tables a Repeat block reuses
    (K3).  Intact parity, then corruptions inside the plan."""
    parts = [gen.frames(gen.text(20 << 20, seed=21), 1 << 20, 9),
             gen.frames(gen.xml(8 << 20, seed=22), 1 << 20, 9),
             gen.frames(gen.binary(8 << 20, seed=23), 1 << 20, 19)]
    data = b"".join(parts)
    from zstd_decompressor.batch import frames_index
    frames, blocks, st, _ = frames_index(data)
    assert st == 0 and len(frames) == 36 and sum(b["type"] == 2 for b in blocks) >= 256
    ost, _ = assert_parity(data, False, "multi-block forked plan")
    assert ost == 0
    r = random.Random(5)
    for it in range(8):
        d = bytearray(data)
        f = frames[r.randrange(4, 32)]
        for _ in range(r.randrange(1, 3)):
            d[f["src_offset"] + r.randrange(f["src_size"])] = r.randrange(256)
        assert_parity(bytes(d), False, f"multi-block forked corrupt #{it}")


def test_parallel_host_walk():
    """Inputs of >= 4 MiB and >= 512 frames are indexed by threads over frame
    ranges (zd_host.cpp plan_index); the plan must equal the serial walk's:
    same first failing frame and status, same output before it.  Corruptions
    around the range boundaries, in block headers (the header-only pass stops
    there) and in block contents, and truncations."""
    src = gen.text(1024 * (16 << 10), seed=31)
    data = gen.frames(src, 16 << 10, 1)
    from zstd_decompressor.batch import frames_index
    frames = frames_index(data)[0]
    assert len(frames) == 1024 and len(data) >= 4 << 20
    ost, _ = assert_parity(data, False, "parallel walk, intact")
    assert ost == 0
    r = random.Random(9)
    for it in range(24):
        d = bytearray(data)
        k = [63, 64, 127, 128, 255, 256, 511, 512, 700, 1000][it % 10] + r.randrange(-2, 3)
        f = frames[max(0, min(k, 1023))]
        if it % 3 == 0:                            # a block header (after the frame header)
            d[f["src_offset"] + 6 + r.randrange(3)] ^= 1 << r.randrange(8)
        else:
            d[f["src_offset"] + r.randrange(f["src_size"])] = r.randrange(256)
        if it % 8 == 7:
            d = d[: f["src_offset"] + r.randrange(f["src_size"])]
        assert_parity(bytes(d), False, f"parallel walk corrupt #{it} (frame {k})")


def test_many_frame_roundtrip_large():
    """Size-independent property at a larger size: decode(compress(x)) == x,
    and the per-frame statuses are all OK."""
    src = gen.text(64 << 20, seed=99)
    data = gen.frames(src, 128 << 10, 3)
    from zstd_decompressor import decompress
    assert decompress(data) == src


def test_one_lane_k3_chain(resources):
    """K3's three chains (sequences.rs:191-237): K3Q, four lanes per block
    (seq_chainq; ZD_F_SEQ_NO_LATENCY forces it in plans of few blocks); K3L,
    one block per wave (seq_chainl, the default in plans of <= 8 blocks per
    CU); the one-lane chain (ZD_F_SEQ_ONE_LANE, seq_chainfl).  All against
    the oracle: the resources, multi-block frames, L19 binary (long offset
    codes) and corruptions inside a 300-frame plan."""
    from zstd_decompressor import _lib
    r = random.Random(79)
    src = gen.text(300 * 4096, seed=15)
    base = gen.frames(src, 4096, 3)
    multi = gen.frames(gen.text(2 << 20, seed=16), 1 << 20, 9)
    binl19 = gen.frames(gen.binary(1 << 20, seed=17), 128 << 10, 19)
    for flags in (_lib.F_SEQ_ONE_LANE, _lib.F_SEQ_NO_LATENCY, 0):
        assert_parity(binl19, False, f"flags={flags} binary L19", flags=flags)
        for name, data in resources.items():
            assert_parity(data, False, f"flags={flags} {name}", flags=flags)
        assert_parity(multi, False, f"flags={flags} multi-block", flags=flags)
        assert_parity(base, False, f"flags={flags} 300 frames", flags=flags)
        for it in range(10):
            d = bytearray(base)
            for _ in range(r.randrange(1, 4)):
                d[r.randrange(len(d))] = r.randrange(256)
            assert_parity(bytes(d), False, f"flags={flags} corrupt #{it}", flags=flags)


def test_mixed_frame_plans():
    """Plans mixing frame sizes, levels and executors against the oracle: 300
    frames of 2-96 KiB at levels 1/3/9 (K4F), and 1,200 runs of 4 KiB frames
    (streaming K4) with a 1 MiB multi-block frame and a frame of 24 blocks
    (K4J), each clean and with corruptions."""
    r = random.Random(83)
    frames = []
    for i in range(300):
        n = r.choice([2048, 8192, 32768, 96 << 10])
        frames.append(gen.frames(gen.text(n, seed=1000 + i), 1 << 20, r.choice([1, 3, 9])))
    k4f_plan = b"".join(frames)
    parts = [gen.frames(gen.text(6000 + 37 * i, seed=2000 + i), 4096, 3) for i in range(1200)]
    parts.insert(600, gen.frames(gen.text(3 << 20, seed=17), 3 << 20, 3))   # 24 blocks: K4J
    parts.insert(100, gen.frames(gen.text(1 << 20, seed=18), 1 << 20, 9))
    k4_plan = b"".join(parts)
    for name, data in (("k4f plan", k4f_plan), ("k4 plan", k4_plan)):
        assert_parity(data, False, name)
        for it in range(6):
            d = bytearray(data)
            for _ in range(r.randrange(1, 4)):
                d[r.randrange(len(d))] = r.randrange(256)
            assert_parity(bytes(d), False, f"{name} corrupt #{it}")


def test_fused_plans():
    """Plans of 256-1024 single-block frames run K3 and K4 fused per group of
    four frames (zd_k_fused: the K4 waves follow their chains' published
    records; a chain the fast path rejects goes to the redo pass);
    ZD_F_NO_FUSE keeps two launches.  Both against the oracle: 300 frames of
    2-128 KiB at levels 1/3/9/19 (raw, RLE and Huffman literals, repeat
    offsets), a C3-shaped plan of 400 x 128 KiB, and corruptions inside both
    (chains rejected mid-plan, K2 and K1 errors)."""
    from zstd_decompressor import _lib
    r = random.Random(91)
    frames = []
    for i in range(300):
        n = r.choice([2048, 16384, 65536, 128 << 10])
        kind = r.choice([gen.text, gen.text, gen.xml, gen.binary])
        frames.append(gen.frames(kind(n, seed=3000 + i), 1 << 20, r.choice([1, 3, 9, 19])))
    mixed = b"".join(frames)
    c3 = gen.frames(gen.text(400 << 17, seed=23), 128 << 10, 3)
    # the fused plan's layout on the two-launch pipeline too (the profiled
    # path runs it): the host walk's parts must start on aligned slots
    import torch
    from zstd_decompressor.batch import Plan
    plan = Plan(c3)
    plan.set_profiling(True)
    d_src = torch.frombuffer(bytearray(c3 + bytes(64)), dtype=torch.uint8).cuda()
    d_dst = torch.zeros(plan.info.out_bytes + 64, dtype=torch.uint8, device="cuda")
    plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), plan.info.out_bytes)
    torch.cuda.synchronize()
    st, total, _, _, _ = plan.results(d_dst.data_ptr())
    ost, oout = oracle.decompress_status(c3)
    assert (st, bytes(d_dst[:total].cpu().numpy())) == (ost, oout), "fused layout, profiled pipeline"
    plan.close()
    for flags in (_lib.F_NO_FUSE, 0):
        for name, data in (("mixed", mixed), ("c3-shaped", c3)):
            assert_parity(data, False, f"flags={flags} {name}", flags=flags)
            for it in range(8):
                d = bytearray(data)
                for _ in range(r.randrange(1, 4)):
                    d[r.randrange(len(d))] = r.randrange(256)
                assert_parity(bytes(d), False, f"flags={flags} {name} corrupt #{it}", flags=flags)


def _random_probs(r, al, nsym):
    """A random NCount distribution of nsym symbols summing to 1 << al in
    absolute value, with "less than one" (-1) and zero probabilities."""
    T = 1 << al
    probs = [0] * nsym
    rem = T
    for i in r.sample(range(nsym), min(nsym, T)):
        if rem == 0:
            break
        if r.random() < 0.2:
            probs[i] = -1
            rem -= 1
    while rem > 0:
        i = r.randrange(nsym)
        if probs[i] >= 0:
            k = min(rem, r.randint(1, max(1, rem // 4)))
            probs[i] += k
            rem -= k
    while probs and probs[-1] == 0:                   # the description ends at its last nonzero
        probs.pop()
    return probs


def _table_frame(r):
    """One single-block frame whose sequence section exercises the table
    builders: per table predefined, RLE or an FSE description (AL 5-9, up to
    255 symbols, -1 probabilities), sometimes damaged (AL > 9, truncated, no
    bitstream left); three raw literals and 1-5 sequences of random bits."""
    modes, tables = 0, b""
    for k, shift in enumerate((6, 4, 2)):              # LL, OF, ML
        m = r.choice([0, 1, 2, 2])
        modes |= m << shift
        if m == 1:
            tables += bytes([r.randrange(64) if r.random() < 0.9 else r.randrange(256)])
        elif m == 2:
            al = r.randint(5, 9)
            nsym = r.choice([r.randint(2, 36), r.randint(2, 64), r.randint(65, 255)])
            t = _ncount(al, _random_probs(r, al, nsym))
            if r.random() < 0.05:
                t = bytes([(t[0] & 0xF0) | 0x0F]) + t[1:]   # AL 20
            tables += t
    nseq = r.choice([1, 2, 5])
    bitstream = b"" if r.random() < 0.05 else \
        bytes(r.randrange(256) for _ in range(r.randrange(2, 16))) + bytes([r.randrange(1, 256)])
    seqs = bytes([nseq, modes]) + tables + bitstream
    if r.random() < 0.05:
        seqs = seqs[: r.randrange(2, len(seqs))]          # truncated inside the descriptions
    content = bytes([(3 << 3) | 0]) + b"xyz" + seqs
    hdr = ((len(content) << 3) | (2 << 1) | 1).to_bytes(3, "little")
    return b"\x28\xb5\x2f\xfd" + bytes([0x00, 0x00]) + hdr + content


def test_fused_table_builds():
    """zd_k_fused builds the sequence tables on its K4 waves (fz_tables,
    fz_build_fse), not zd_k_tables: crafted frames (predefined / RLE / FSE
    tables of AL 5-9 and up to 255 symbols, -1 probabilities, damaged
    descriptions, deep OF tables for the redo pass) each decoded as the last
    frame of a 300-frame plan, which takes the fused path, and on the
    two-launch pipeline (ZD_F_NO_FUSE: zd_k_tables_seqw, and with
    ZD_F_K1_LANES K1's lanes); status and output as the oracle's."""
    from zstd_decompressor import _lib
    r = random.Random(4242)
    filler = gen.frames(gen.text(299 * 2048, seed=51), 2048, 3)
    from zstd_decompressor.batch import Plan
    for i in range(40):
        data = filler + _table_frame(r)
        plan = Plan(data)
        assert plan.info.executors & _lib.EXEC_FUSED, "the 300-frame plan takes zd_k_fused"
        plan.close()
        for flags in (0, _lib.F_NO_FUSE, _lib.F_NO_FUSE | _lib.F_K1_LANES):
            assert_parity(data, False, f"table frame #{i} flags={flags}", flags=flags)


def test_plan_decompress_reuses_the_plan(resources):
    """zd_plan_decompress: host in / host out with a plan made once (the
    INTEGRATION.md decompress() pattern), equal to the oracle's output."""
    import ctypes as C
    from zstd_decompressor import _lib
    from zstd_decompressor.batch import Plan
    L = _lib.lib()
    for name, data in resources.items():
        ost, oout = oracle.decompress_status(data)
        plan = Plan(data)
        cap = max(plan.info.out_bytes, 1)
        buf = (C.c_uint8 * cap)()
        n = C.c_size_t()
        p, nb, keep = _lib.buf(data)
        st = L.zd_plan_decompress(plan._h, p, nb, buf, cap, C.byref(n))
        assert st == ost, name
        assert bytes(buf[: n.value]) == oout, name
        plan.close()


def test_one_round_plan():
    """A plan of 3,000 frames of 8 KiB (one round of K3 chains and of K2
    blocks, like one rank's share of C4 on 8 GPUs): round trip, then
    corruptions inside the plan against the oracle."""
    r = random.Random(78)
    src = gen.text(3000 * 8192, seed=14)
    base = gen.frames(src, 8192, 3)
    from zstd_decompressor import decompress
    from zstd_decompressor.batch import frames_index
    assert decompress(base) == src
    spans = [(f["src_offset"], f["src_size"]) for f in frames_index(base)[0]]
    assert len(spans) == 3000
    for it in range(8):
        d = bytearray(base)
        o, n = spans[r.randrange(100, 2900)]
        for _ in range(r.randrange(1, 4)):
            d[o + r.randrange(n)] = r.randrange(256)
        assert_parity(bytes(d), False, f"per-CU plan corrupt #{it}")


def _ncount(al, probs):
    """FSE table description (the inverse of parse_fse_table, fse.rs:16-69):
    probabilities of symbols 0.. (-1 = "less than one"), LSB-first bits."""
    bits, nbits = 0, 0

    def put(v, n):
        nonlocal bits, nbits
        bits |= v << nbits
        nbits += n
    put(al - 5, 4)
    remaining, i = 1 << al, 0
    while remaining > 0:
        d = probs[i] + 1
        nb = (remaining + 1).bit_length()                   # highbit(remaining + 1) + 1
        low = (1 << (nb - 1)) - 1
        thr = (1 << nb) - 1 - (remaining + 1)
        if d < thr:
            put(d, nb - 1)
        elif d <= low:
            put(d, nb)
        else:
            put(d + thr, nb)
        remaining -= abs(probs[i])
        i += 1
        if probs[i - 1] == 0:                               # repeat flags for the zeros that follow
            z = 0
            while i + z < len(probs) and probs[i + z] == 0:
                z += 1
            i += z
            while True:
                put(min(z, 3), 2)
                if z < 3:
                    break
                z -= 3
    assert i == len(probs), (i, len(probs))
    return bits.to_bytes((nbits + 7) // 8, "little")


def test_k1_large_tables():
    """Sequence tables with more than 64 symbols (LL codes past the maximum):
    K1's first pass flags the block and the large-scratch pass builds it
    (zd_kernels.hip zd_k_tables<true>, under ZD_F_K1_LANES), or the
    wave-per-block build does (zd_k_tables_seqw, the default for small
    plans); status and output match the oracle."""
    from zstd_decompressor import _lib
    r = random.Random(77)
    for nsym, al in ((70, 6), (65, 7), (100, 7), (255, 8)):
        probs = [1] * (nsym - 1) + [(1 << al) - (nsym - 1)]   # the last symbol takes the rest
        if probs[-1] <= 0:
            probs = [1] * ((1 << al) - 1) + [0] * (nsym - (1 << al)) + [1]
        assert sum(abs(p) for p in probs) == 1 << al and len(probs) == nsym
        table = _ncount(al, probs)
        for trial in range(6):
            bitstream = bytes(r.randrange(256) for _ in range(r.randrange(3, 12))) + bytes([r.randrange(1, 256)])
            nseq = r.choice([1, 2, 5])
            seqs = bytes([nseq, 0x80]) + table + bitstream       # LL FSE, OF/ML predefined
            lits = bytes([(3 << 3) | 0]) + b"xyz"               # raw literals, 3 bytes
            content = lits + seqs
            hdr = ((len(content) << 3) | (2 << 1) | 1).to_bytes(3, "little")
            frame = b"\x28\xb5\x2f\xfd" + bytes([0x00, 0x00]) + hdr + content
            for flags in (0, _lib.F_K1_LANES):
                assert_parity(frame, False, f"nsym {nsym} al {al} trial {trial} flags {flags}", flags=flags)


def _deep_tree_frame(r, nbytes, weights=None):
    """One frame, one compressed block: a Huffman tree of direct weights
    (default maxBits 12: weights 12, 11, ..., 1 and the implied last symbol,
    a complete tree: every bit pattern decodes) over a random literal
    bitstream, then one sequence from random bits with the predefined tables."""
    if weights is None:
        weights = list(range(12, 0, -1))                   # symbols 0..11; symbol 12 implied
    w = list(weights) + [0] * (len(weights) & 1)
    desc = bytes([127 + len(weights)]) + bytes((w[i] << 4) | w[i + 1] for i in range(0, len(w), 2))
    stream = bytes(r.randrange(256) for _ in range(nbytes - 1)) + bytes([r.randrange(1, 256)])
    comp = len(desc) + len(stream)
    regen = 1023                                            # >= what the stream decodes (the reference ignores it, D8)
    lh = (2 | (0 << 2) | (regen << 4) | (comp << 14)).to_bytes(3, "little")   # compressed, 1 stream
    seqs = bytes([1, 0x00]) + bytes(r.randrange(256) for _ in range(4)) + bytes([r.randrange(1, 256)])
    content = lh + desc + stream + seqs                     # one sequence, predefined tables
    hdr = ((len(content) << 3) | (2 << 1) | 1).to_bytes(3, "little")
    return b"\x28\xb5\x2f\xfd" + bytes([0x00, 0x50]) + hdr + content


def test_k2_deep_trees_beside_libzstd_frames():
    """12-bit Huffman trees (K2 reads their LUTs from HBM, and so does every
    block of its workgroup) in between libzstd frames with <= 11-bit trees,
    whose LUTs hold K2's shifted width field (zd_kernels.hip lut_field)."""
    r = random.Random(9)
    deep_ok, deep_err = [], []
    while len(deep_ok) < 8 or len(deep_err) < 8:         # frames the reference decodes, and ones it rejects
        f = _deep_tree_frame(r, r.randrange(20, 200))
        (deep_err if oracle.decompress_status(f, False)[0] else deep_ok).append(f)
    src = gen.text(300_000, seed=4)
    parts = []
    for i in range(24):
        parts.append(deep_ok[i // 3] if i % 3 == 1 else gen.frames(src[i * 12_000:(i + 1) * 12_000], 12_000, 3))
    ost, _ = assert_parity(b"".join(parts), False, "deep trees + libzstd frames")
    assert ost == 0
    for i, f in enumerate(deep_err[:8]):
        assert_parity(f, False, f"deep tree, rejected #{i}")


def test_k2_trees_deeper_than_the_lut():
    """Trees of maxBits 13..21 (non-conforming: zstd stops at 11) have no LUT;
    K1 keeps their codes as intervals and K2 decodes them symbol by symbol
    (zd_kernels.hip deep_build / huf_stream_deep).  Complete trees (weights
    p..1) and random weights (absent tree nodes at any depth: the reference
    panics there, or runs out of bits first), alone and inside a plan of
    libzstd frames; streams that decode past Regenerated_Size re-plan their
    frame with room for the literals (zd_plan_decompress)."""
    r = random.Random(23)
    ok, frames = [], []
    for p in range(13, 16):                 # complete trees: a frame of each depth the reference decodes
        for _ in range(100):
            f = _deep_tree_frame(r, r.randrange(20, 300), list(range(p, 0, -1)))
            frames.append(f)
            if oracle.decompress_status(f, False)[0] == 0:
                ok.append(f)
                break
    assert len(ok) == 3
    for _ in range(40):
        n = r.randrange(2, 128)
        weights = [r.choice([0, 0, r.randrange(1, 16)]) for _ in range(n)]
        weights[r.randrange(n)] = r.randrange(12, 16)
        frames.append(_deep_tree_frame(r, r.randrange(20, 300), weights))
    for i, f in enumerate(frames):
        assert_parity(f, False, f"deep tree #{i}")
    src = gen.text(200_000, seed=5)
    parts = []
    for i in range(9):
        parts.append(ok[i // 3] if i % 3 == 1 else gen.frames(src[i * 12_000:(i + 1) * 12_000], 12_000, 3))
    ost, _ = assert_parity(b"".join(parts), False, "deep trees inside libzstd frames")
    assert ost == 0


# FSE-compressed Huffman weights decoding to 7,709 nonzero weights (maxBits 13):
# more leaves than a LUT slot's 7,680 symbol bytes (tests/golden/make_deep_tree_desc.py)
DEEP_DESC_7709 = bytes.fromhex(
    "7621fc01f0bfd64950ebd9ef23d79f8cf8023d4fd669ffba7efbdffbae8bcaa6ae366df908c7266acb382b4d79de8c"
    "fac3345fe9099c6a0b85c60ef9beef7bb5c5eba739082a8c150f08ff8feb5c1d9bc050f0fda7c7fbc351db16d35479"
    "bbbe61212d2594467f7676fe5b7f2288477b40d32af17affe0")


def _big_tree_frame(r, codes, n):
    """One frame, one compressed block: DEEP_DESC_7709's tree over n literals
    encoded with its codes (insertion order of huffman.rs:132-175; the first
    literal's code right under the marker bit), then one sequence from random
    bits with the predefined tables."""
    keys = list(codes)
    v = 1
    for _ in range(n):
        c, w = codes[r.choice(keys)]
        v = (v << w) | c
    stream = v.to_bytes((v.bit_length() + 7) // 8, "little")
    comp = len(DEEP_DESC_7709) + len(stream)
    lh = (2 | (0 << 2) | (n << 4) | (comp << 14)).to_bytes(3, "little")   # compressed, 1 stream
    seqs = bytes([1, 0x00]) + bytes(r.randrange(256) for _ in range(4)) + bytes([r.randrange(1, 256)])
    content = lh + DEEP_DESC_7709 + stream + seqs
    hdr = ((len(content) << 3) | (2 << 1) | 1).to_bytes(3, "little")
    return b"\x28\xb5\x2f\xfd" + bytes([0x00, 0x50]) + hdr + content


def test_k2_tree_past_the_lut_slot():
    """A deep tree with more leaves (7,709) than a LUT slot's symbol bytes:
    K1's huge pass keeps its symbols in the plan's deep pool (zd_kernels.hip
    deep_build, DEEP_IN_POOL) and K2 decodes from there.  Frames that decode
    and frames the reference rejects (its sequence is random), alone and many
    of them in one plan beside libzstd frames (several trees in the pool)."""
    _, widths = oracle.huffman_widths(DEEP_DESC_7709)
    p = max(widths)
    assert p == 13 and sum(1 for w in widths if w) > 7680
    codes, pos = {}, 0
    for w in range(p, 0, -1):                      # longest first, ascending symbols, aligned slots
        S = 1 << (p - w)
        al = (pos + S - 1) & ~(S - 1)
        for i in (i for i, x in enumerate(widths) if x == w):
            if al + S > 1 << p:
                break
            codes[i] = (al >> (p - w), w)
            al += S
        pos = al
    r = random.Random(31)
    ok = []
    for i in range(120):
        f = _big_tree_frame(r, codes, r.randrange(100, 500))
        ost, _ = assert_parity(f, False, f"tree of 7,709 leaves #{i}")
        if ost == 0:
            ok.append(f)
    assert len(ok) >= 3
    src = gen.text(200_000, seed=6)
    parts = []
    for i in range(12):
        parts.append(ok[i % len(ok)] if i % 2 else gen.frames(src[i * 12_000:(i + 1) * 12_000], 12_000, 3))
    ost, _ = assert_parity(b"".join(parts), False, "trees of 7,709 leaves inside libzstd frames")
    assert ost == 0


def _tree_codes_7709():
    _, widths = oracle.huffman_widths(DEEP_DESC_7709)
    p = max(widths)
    codes, pos = {}, 0
    for w in range(p, 0, -1):
        S = 1 << (p - w)
        al = (pos + S - 1) & ~(S - 1)
        for i in (i for i, x in enumerate(widths) if x == w):
            if al + S > 1 << p:
                break
            codes[i] = (al >> (p - w), w)
            al += S
        pos = al
    return codes


def _tree_block(r, codes, n, treeless, last, seqbits):
    """One compressed block: n literals under DEEP_DESC_7709's tree (its
    description in the block, or Treeless: the previous block's tree,
    literals.rs:88-206 type 3), then one sequence of the given bits."""
    keys = list(codes)
    v = 1
    for _ in range(n):
        c, w = codes[r.choice(keys)]
        v = (v << w) | c
    stream = v.to_bytes((v.bit_length() + 7) // 8, "little")
    desc = b"" if treeless else DEEP_DESC_7709
    comp = len(desc) + len(stream)
    lh = ((3 if treeless else 2) | (0 << 2) | (n << 4) | (comp << 14)).to_bytes(3, "little")
    content = lh + desc + stream + bytes([1, 0x00]) + seqbits
    return ((len(content) << 3) | (2 << 1) | int(last)).to_bytes(3, "little") + content


def test_context_deep_pool_tree_then_treeless():
    """Block.decode(ctx) of a block whose tree keeps its symbols in the plan's
    deep pool (7,709 leaves), then Treeless blocks reusing that tree: the
    context persists the pool with the LUT slot (block.rs:74-99 through one
    DecodingContext), against the oracle's decode of the same frame and the
    batch path's."""
    from zstd_decompressor import ForwardByteParser, Block, DecodingContext, MAX_WIN_SIZE
    codes = _tree_codes_7709()
    r = random.Random(57)
    head = b"\x28\xb5\x2f\xfd" + bytes([0x00, 0x50])
    for trial in range(2):
        blocks = []
        for k in range(3):
            # the block's sequence: random bits until the frame so far decodes
            for attempt in range(2000):
                n = r.randrange(100, 400)
                seed = r.randrange(1 << 30)
                bits = bytes(random.Random(seed).randrange(256) for _ in range(4)) + bytes([r.randrange(1, 256)])
                cand = _tree_block(random.Random(seed), codes, n, k > 0, True, bits)
                if oracle.decompress_status(head + b"".join(blocks) + cand, False)[0] == 0:
                    blocks.append(_tree_block(random.Random(seed), codes, n, k > 0, k == 2, bits))
                    break
            else:
                pytest.fail(f"no decodable sequence for block {k}")
        frame = head + b"".join(blocks)
        ost, expect = oracle.decompress_status(frame, False)
        assert ost == 0
        assert_parity(frame, False, f"deep tree + Treeless #{trial}")
        p = ForwardByteParser(frame)
        p.slice(6)
        ctx = DecodingContext(MAX_WIN_SIZE)
        while True:
            b, last = Block.parse(p)
            b.decode(ctx)
            if last:
                break
        assert ctx.decoded == expect, f"trial {trial}: context output differs"
        ctx.close()

def _pair_table_kind(weights):
    """Which pair-table entries a tree of direct weights gives K2
    (zd_kernels.hip PR_*): None when the reference panics building it, else
    (p, L, long) -- maxBits, the leading 10-bit prefixes split into 11-bit
    halves, and whether a deep prefix lies past them (PR_LONG).  Restates
    from_weights + insert (huffman.rs:132-203) as K1 places the codes:
    longest first, each width from the next aligned slot; gaps are absent
    nodes."""
    ws = [w for w in weights if w]
    if not ws or max(ws) > 32:
        return None
    total = sum(1 << (w - 1) for w in ws)
    p = total.bit_length() - 1
    if (1 << p) < total:
        p += 1
    rest = (1 << p) - total
    if rest == 0 or rest > 255 or max(ws) > p + 1:
        return None
    manq = rest.bit_length()
    if manq > p + 1 or p > 11:
        return None
    cnt = {}
    for w in list(ws) + [manq]:
        cnt[p + 1 - w] = cnt.get(p + 1 - w, 0) + 1
    T, pos, width = 1 << p, 0, [0] * (1 << p)
    holes = []
    for w in range(p, 0, -1):
        if not cnt.get(w):
            continue
        S = 1 << (p - w)
        al = (pos + S - 1) & ~(S - 1)
        holes.append((pos, al))
        k = min(cnt[w], (T - al) // S)
        for e in range(al, al + k * S):
            width[e] = w
        pos = al + k * S
    holes.append((pos, T))
    for a, b in holes:
        for e in range(a, b):
            k = p
            while k > 0 and not ((e & ~((1 << k) - 1)) >= a and (e & ~((1 << k) - 1)) + (1 << k) <= b):
                k -= 1
            width[e] = p - k
    if p < 11:
        return p, 0, False
    deep = [width[2 * i] > 10 or width[2 * i + 1] > 10 for i in range(1024)]
    L = next((i for i, d in enumerate(deep) if not d), 1024)
    return p, min(L, 128), any(deep[i] for i in range(min(L, 128), 1024))


def test_k2_pair_tables():
    """K2's pair tables (zd_k_huf_pairs, huf_stream_pr): trees of maxBits
    1..11 with no 11-bit codes (no split prefixes) and with split leading
    prefixes, complete (frames the reference decodes, so the literal bytes
    are compared) and incomplete (absent nodes: the reference panics or runs
    out of bits), over streams of 12 bytes (the exact path alone) to 400 (the
    fast loop), each frame against the oracle, alone and beside libzstd
    frames.  (Deep prefixes past the leading run -- PR_LONG -- need more than
    256 leaves, K1's huge-tree pass: a tree description of direct weights
    cannot reach them, and _pair_table_kind never reports one here.)"""
    r = random.Random(31)
    want = {("short", True): 6, ("split", True): 6, ("short", False): 4, ("split", False): 4}
    got = {k: [] for k in want}
    for _ in range(40000):
        if all(len(got[k]) >= want[k] for k in want):
            break
        if r.random() < 0.5:
            n = r.randrange(2, 128)
            top = r.choice([4, 8, 11, 12])
            weights = [r.choice([0, r.randrange(1, top)]) for _ in range(n)]
        else:                                             # a complete code with 11-bit codes: split leaves
            lens = [0]
            while len(lens) < r.randrange(8, 120) or max(lens) < 11:
                cand = [i for i, l in enumerate(lens) if l < 11]
                i = r.choice(cand) if r.random() < 0.6 else max(cand, key=lambda c: lens[c])
                lens[i] += 1
                lens.append(lens[i])
            r.shuffle(lens)
            weights = [12 - l for l in lens[:-1]]         # the last symbol is the implied one
        kind = _pair_table_kind(weights)
        if kind is None:
            continue
        p, L, lng = kind
        assert not lng
        total = sum(1 << (w - 1) for w in weights if w)
        rest = (1 << p) - total
        complete = rest & (rest - 1) == 0                 # the implied symbol fills the tree
        k = ("split" if L else "short", complete)
        if len(got[k]) >= want[k]:
            continue
        f = _deep_tree_frame(r, 400, weights)
        if complete and oracle.decompress_status(f, False)[0] != 0:
            continue                                      # (the random sequence failed)
        got[k].append((weights, f))
    assert all(len(got[k]) >= want[k] for k in want), {k: len(v) for k, v in got.items()}
    frames = []
    for k in want:
        for weights, f in got[k]:
            frames += [f, _deep_tree_frame(r, 12, weights), _deep_tree_frame(r, 60, weights)]
    for i, f in enumerate(frames):
        assert_parity(f, False, f"pair table #{i}")
    src = gen.text(200_000, seed=6)
    parts = []
    for i, f in enumerate(frames[::3]):
        parts.append(f)
        parts.append(gen.frames(src[i * 5_000:(i + 1) * 5_000], 5_000, 3))
    assert_parity(b"".join(parts), False, "pair tables beside libzstd frames")


@pytest.mark.parametrize("shape", ["one_frame", "forked_300_frames", "block_parallel"])
def test_hip_graph_capture_replay(shape):
    """zd_decode_async is graph-safe (include/zd.h): no allocation, no host
    memory read (states reset from device-resident copies), the second
    stream made at plan time.  Capture it in a HIP graph, clear the output,
    replay: same bytes as the source."""
    import torch
    from zstd_decompressor import _lib
    from zstd_decompressor.batch import Plan
    flags = 0
    if shape == "one_frame":
        src = gen.text(1 << 20, seed=61)
        data = libzstd.compress(src, 3)
    elif shape == "forked_300_frames":
        src = gen.text(300 * 4096, seed=62)
        data = gen.frames(src, 4096, 3)
    else:
        src = gen.text(3 << 20, seed=63)
        data = gen.frames(src, 1 << 20, 9)
        flags = _lib.F_BLOCK_PARALLEL
    plan = Plan(data, False, flags)
    n = plan.info.out_bytes
    dev = torch.device("cuda", 0)
    d_src = torch.zeros(len(data) + 64, dtype=torch.uint8, device=dev)
    d_src[: len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    d_dst = torch.zeros(n + 64, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):          # warm-up outside the capture
        plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), n, s.cuda_stream)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), n, s.cuda_stream)
    d_dst.zero_()
    torch.cuda.synchronize(dev)
    g.replay()
    torch.cuda.synchronize(dev)
    st, total, _, _, _ = plan.results(d_dst.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    assert st == 0 and total == len(src)
    assert bytes(d_dst[:total].cpu().numpy().tobytes()) == src
    plan.close()
