"""K4 pass 0 (zd_k_execute, the merged 16-byte chunks of execute_sequences,
decoding_context.rs:95-98) is correct only if each lane's chunk is written by
ONE ds_write_b128: where lanes' chunks overlap, one wave-wide LDS store leaves
each byte to the highest lane writing it (tools/lds_order_check,
test_lds_order.py pin that hardware rule).  A store split into two
ds_write_b64 would let a lower lane's second half overwrite a higher lane's
first half.  This checks the code generation, on the CPU:

1. zd_kernels.hip compiled for gfx950 with the pass-0 store bracketed by asm
   markers (-DZD_ISA_MARKS=1): every bracket holds exactly one LDS store, a
   ds_write_b128;
2. the shipped lib/libzd.so's gfx950 code object: zd_k_execute has the same
   LDS store instructions, by kind and count, as that marked build, so the
   markers changed nothing the check relies on.
"""
import collections
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zstd-decompressor_amd", "csrc")
LIB = os.path.join(ROOT, "zstd-decompressor_amd", "lib", "libzd.so")
HIPCC = "/opt/rocm/bin/hipcc"
OBJDUMP = "/opt/rocm/llvm/bin/llvm-objdump"
K4 = "_ZN2zd12zd_k_execute"
STORE = re.compile(r"\b(ds_(?:write|store)\w*)")

pytestmark = pytest.mark.skipif(not (os.path.exists(HIPCC) and os.path.exists(OBJDUMP)), reason="no ROCm toolchain")


def _function(lines, start_pred, end_pred):
    a = next(i for i, l in enumerate(lines) if start_pred(l))
    b = next(i for i in range(a + 1, len(lines)) if end_pred(lines[i]))
    return lines[a:b]


def _stores(lines):
    c = collections.Counter()
    for l in lines:
        t = l.split(";")[0] if not l.lstrip().startswith(";") else ""
        m = STORE.search(t)
        if m:
            c[m.group(1)] += 1
    return c


@pytest.fixture(scope="module")
def marked(tmp_path_factory):
    d = tmp_path_factory.mktemp("isa")
    out = d / "k.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result",
                    "--cuda-device-only", "-S", "-DZD_ISA_MARKS=1", os.path.join(CSRC, "zd_kernels.hip"),
                    "-I", CSRC, "-o", str(out)], check=True, capture_output=True, timeout=600)
    L = out.read_text().split("\n")
    return _function(L, lambda l: l.startswith(K4 + "E") and ":" in l, lambda l: l.startswith(".Lfunc_end"))


def test_pass0_put_is_one_ds_write_b128(marked):
    opens = [i for i, l in enumerate(marked) if "ZDPUT<" in l]
    closes = [i for i, l in enumerate(marked) if "ZDPUT>" in l]
    assert opens and len(opens) == len(closes)
    for a, b in zip(opens, closes):
        assert a < b
        st = _stores(marked[a + 1:b])
        assert st == collections.Counter({"ds_write_b128": 1}), (a, st, marked[a:b + 1])


def test_shipped_library_matches_the_marked_build(marked, tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("lib/libzd.so not built")
    so = tmp_path / "libzd.so"
    shutil.copy(LIB, so)
    subprocess.run([OBJDUMP, "--offloading", str(so)], check=True, capture_output=True, cwd=tmp_path, timeout=120)
    co = [p for p in os.listdir(tmp_path) if "gfx950" in p]
    assert co, os.listdir(tmp_path)
    dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", str(tmp_path / co[0])], check=True, capture_output=True,
                         text=True, timeout=300).stdout.split("\n")
    k4 = _function(dis, lambda l: re.match(r"^[0-9a-f]+ <" + K4 + r"E", l) is not None,
                   lambda l: re.match(r"^[0-9a-f]+ <", l) is not None)
    shipped = _stores(k4)
    assert shipped["ds_write_b128"] > 0
    assert shipped == _stores(marked), (shipped, _stores(marked))
