"""Static instruction counts per K4 phase: compile zd_kernels.hip with the
K4_PHASE markers turned into asm comments and count VALU / SALU / LDS / VMEM
instructions between them in zd_k_execute's batch loop.
usage: python scripts/k4_isa_phases.py [extra hipcc defines...]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zstd-decompressor_amd", "csrc")
src = open(os.path.join(CSRC, "zd_kernels.hip")).read()
src = src.replace('#define K4_PHASE(i) do { } while (0)', '#define K4_PHASE(i) asm volatile("; K4PH " #i)')
open("/tmp/kph.hip", "w").write(src)
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                       "/tmp/kph.hip", "-I", CSRC, "-o", "/tmp/kph.s"] + sys.argv[1:], stderr=subprocess.DEVNULL)
L = open("/tmp/kph.s").read().split("\n")
a = next(i for i, l in enumerate(L) if l.startswith("_ZN2zd12zd_k_execute"))
b = next(i for i in range(a, len(L)) if L[i].startswith(".Lfunc_end"))
marks = [i for i in range(a, b) if "K4PH" in L[i]]
# the batch loop: from the header containing the first marker to the last branch back to it
hdr = max(i for i in range(a, marks[0]) if re.match(r"\.LBB\d+_\d+:", L[i]))
name = L[hdr].split(":")[0]
end = max(i for i in range(a, b) if re.search(r"s_(cbranch_\w+|branch)\s+" + re.escape(name) + r"\b", L[i]))
def cnt(x, y):
    c = dict(v=0, s=0, ds=0, g=0, nop=0, br=0)
    for l in L[x:y]:
        t = l.strip()
        if not t or t[0] in ";." or ":" in t.split()[0]:
            continue
        op = t.split()[0]
        k = ("nop" if op.startswith("s_nop") else "br" if op.startswith(("s_cbranch", "s_branch")) else
             "v" if op.startswith("v_") else "ds" if op.startswith("ds_") else
             "g" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else "s" if op.startswith("s_") else None)
        if k:
            c[k] += 1
    return c
pts = [hdr] + marks + [end + 1]
tot = cnt(hdr, end + 1)
for x, y in zip(pts, pts[1:]):
    print(L[x].strip()[:12].ljust(12), cnt(x, y))
print("loop total", tot)
