"""Content checksums (XXH64, seed 0): an extra beyond the reference, which
computes the hash in frame.rs:239-255 but never enforces it.
The shared XXH64 pieces (zd_common.h) are checked on the host against the
`xxhash` package; the GPU pass (zd_plan_checksums) against libzstd's stored
checksums and `xxhash`.  Decode status is never affected by a mismatch."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

XXH_HOST = r'''
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "zstd-decompressor_amd/csrc/zd_common.h"
using namespace zd;
int main(int argc, char** argv) {
  // xxh64 of the byte strings i*7 % 251 of lengths given on the command line
  for (int a = 1; a < argc; a++) {
    size_t n = strtoul(argv[a], 0, 10);
    std::vector<uint8_t> d(n);
    for (size_t i = 0; i < n; i++) d[i] = (uint8_t)(i * 7 % 251);
    uint64_t v[4] = {xx_acc_init(0), xx_acc_init(1), xx_acc_init(2), xx_acc_init(3)};
    size_t s = 0;
    for (; s + 32 <= n; s += 32)
      for (int k = 0; k < 4; k++) {
        uint64_t w = 0;
        for (int b = 7; b >= 0; b--) w = (w << 8) | d[s + 8 * k + b];
        v[k] = xx_round(v[k], w);
      }
    printf("%llu\n", (unsigned long long)xx_finish(n, v, d.data() + s, (uint32_t)(n - s)));
  }
}
'''


def test_xxh64_host_pieces(tmp_path):
    xxhash = pytest.importorskip("xxhash")
    src = tmp_path / "x.cpp"
    src.write_text(XXH_HOST)
    exe = tmp_path / "x"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", ROOT, "-o", str(exe), str(src)])
    lens = [0, 1, 3, 4, 7, 8, 15, 31, 32, 33, 63, 64, 100, 1000, 131072]
    out = subprocess.run([str(exe)] + [str(n) for n in lens], capture_output=True, text=True, check=True).stdout.split()
    for n, got in zip(lens, out):
        d = bytes(i * 7 % 251 for i in range(n))
        assert int(got) == xxhash.xxh64(d, seed=0).intdigest(), n


@pytest.mark.gpu
def test_gpu_checksums():
    xxhash = pytest.importorskip("xxhash")
    import torch
    from corpus import gen
    from zstd_decompressor.batch import Plan, frames_index
    src = gen.text(600_000, seed=21)
    data = bytearray(gen.frames(src, 100_000, 3, checksum=True) + gen.frames(src[:50_000], 100_000, 3))
    frames, _, _, _ = frames_index(bytes(data))
    # corrupt the stored checksum of frame 2 (the last 4 bytes of the frame)
    f2 = frames[2]
    end = f2["src_offset"] + f2["src_size"]
    data[end - 1] ^= 0x5A
    data = bytes(data)
    plan = Plan(data)
    d_src = torch.zeros(len(data) + 64, dtype=torch.uint8, device="cuda")
    d_src[: len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    d_dst = torch.empty(plan.info.out_bytes + 64, dtype=torch.uint8, device="cuda")
    plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), plan.info.out_bytes)
    st, total, fst, flen, _ = plan.results(d_dst.data_ptr())
    assert st == 0                                     # the reference never enforces checksums
    ok, h = plan.checksums(d_dst.data_ptr())
    out = bytes(d_dst[:total].cpu().numpy().tobytes())
    pos = 0
    for i, f in enumerate(frames):
        piece = out[pos: pos + flen[i]]
        pos += flen[i]
        assert h[i] == xxhash.xxh64(piece, seed=0).intdigest(), i
        if f["has_checksum"]:
            assert ok[i] == (0 if i == 2 else 1), (i, ok[i])
        else:
            assert ok[i] == -1
