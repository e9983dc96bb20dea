"""Planner regression check (host only, no GPU): the descriptor arrays two
libzd builds make for the same inputs (ZD_PLAN_DUMP), byte for byte.
usage: python tools/plan_compare.py OLD_LIBZD.so NEW_LIBZD.so
(plan creation stops at the device allocation without a GPU; the dump is
written before it).  The NEW build plans two other inputs first, so its
process caches are warm."""
import ctypes as C, os, sys, random, subprocess, hashlib, json
OLD, NEW = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'zstd-decompressor_amd'))
def dump(lib, data, flags, out):
    code = f"""
NEW_LIB = {NEW!r}
import ctypes as C, os, sys
os.environ['ZD_PLAN_DUMP'] = {out!r}
L = C.CDLL({lib!r})
data = open('/tmp/plan_in.bin','rb').read()
P = C.c_void_p()
L.zd_plan_create.argtypes = [C.c_char_p, C.c_size_t, C.c_uint32, C.c_void_p]
if {lib!r} == NEW_LIB:
    pre = open('/tmp/plan_pre.bin','rb').read()
    L.zd_plan_create(pre, len(pre), 0, C.byref(P))
    L.zd_plan_create(pre[:len(pre)//3], len(pre)//3, 0, C.byref(P))
r = L.zd_plan_create(data, len(data), {flags}, C.byref(P))
"""
    subprocess.run([sys.executable, '-c', code], check=True)
    return open(out, 'rb').read()
def cases():
    from corpus import gen as g2, libzstd as lz2
    if not os.path.exists('/tmp/c4set.zst'):
        open('/tmp/c4set.zst', 'wb').write(g2.frames(g2.text(256 << 20, seed=0x5EED), 128 << 10, 3))
    yield 'c4x4', open('/tmp/c4set.zst','rb').read() * 4
    skip = (0x184D2A53).to_bytes(4,'little') + (5).to_bytes(4,'little') + b'abcde'
    yield 'bigmix', open('/tmp/c4set.zst','rb').read() * 2 + lz2.compress(g2.text(6 << 20, seed=4), 3) + skip + g2.c2_raw_rle(4 << 20) + open('/tmp/c4set.zst','rb').read()
    if os.environ.get('ONLY_BIG'): return
    from corpus import gen, libzstd
    kat = json.load(open(os.path.join(ROOT, 'tests/golden/kat.json')))
    for c in kat['frames']:
        yield 'kat', bytes(c['data'])
    for f in os.listdir(os.path.join(ROOT, 'tests/golden/resources')):
        yield f, open(os.path.join(ROOT, 'tests/golden/resources', f), 'rb').read()
    t = gen.text(3 << 20, seed=1)
    yield 'frames128k', gen.frames(t, 128 << 10, 3)
    yield 'frames1m_L9', gen.frames(t, 1 << 20, 9)
    yield 'frames1m_L19', gen.frames(gen.binary(2 << 20, seed=3), 1 << 20, 19)
    yield 'single', libzstd.compress(t, 3)
    yield 'c2', gen.c2_raw_rle(8 << 20)
    yield 'chk', gen.frames(t[:600000], 300000, 3, checksum=True)
    big = gen.frames(gen.text(8 << 20, seed=5), 128 << 10, 3)
    yield 'big_x4', big * 4                        # >= 4 MiB: parallel walk
    mixed = big + libzstd.compress(t, 3) + big     # a frame spanning several ranges
    yield 'mixed', mixed
    r = random.Random(7)
    for i in range(40):
        d = bytearray(big * 2)
        for _ in range(r.randrange(1, 4)):
            d[r.randrange(len(d))] = r.randrange(256)
        if r.random() < 0.3:
            d = d[:r.randrange(len(d))]
        yield f'corrupt{i}', bytes(d)
    # magic numbers planted inside data
    d = bytearray(big * 2)
    for _ in range(50):
        p = r.randrange(len(d) - 4); d[p:p+4] = (0xFD2FB528).to_bytes(4, 'little')
    yield 'planted', bytes(d)
bad = 0
from corpus import gen as _g
open('/tmp/plan_pre.bin','wb').write(_g.frames(_g.xml(12 << 20, seed=9), 1 << 20, 9) + _g.frames(_g.text(4 << 20, seed=2), 128<<10, 1))
for name, data in cases():
    open('/tmp/plan_in.bin', 'wb').write(data)
    for flags in (0, 1, 2, 4):
        a = dump(OLD, data, flags, '/tmp/d_old.bin')
        b = dump(NEW, data, flags, '/tmp/d_new.bin')
        if a != b:
            bad += 1
            print('DIFF', name, flags, len(data), len(a), len(b))
print('done, diffs:', bad)
