"""The command line (zstd_decompressor/__main__.py) against the reference CLI
behaviour (src/main.rs:7-60): stdout / -o output, -p for skippable payloads,
the first failing frame -> exit 1 with nothing written, non-UTF-8 output ->
exit 101 (the reference's `String::from_utf8(res).unwrap()` panic), --info
listing frames.  Expected bytes come from the oracle (the CPU restatement)."""
import os
import subprocess
import sys

import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "zstd-decompressor_amd")
RES = os.path.join(ROOT, "tests", "golden", "resources")


def cli(*args, timeout=300):
    env = dict(os.environ, PYTHONPATH=PKG + os.pathsep + ROOT)
    return subprocess.run([sys.executable, "-m", "zstd_decompressor", *args], cwd=ROOT, env=env,
                          capture_output=True, timeout=timeout)


def test_info_lists_frames():
    r = cli("-i", os.path.join(RES, "romeo3.txt.zst"))
    assert r.returncode == 0
    lines = r.stdout.decode().splitlines()
    assert len(lines) == 3 and all(l.startswith("ZStandardFrame(") for l in lines)
    r = cli("--info", os.path.join(RES, "skippables.zst"))
    assert r.returncode == 0 and all(l.startswith("SkippableFrame(") for l in r.stdout.decode().splitlines())


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["moby-dick.txt.zst", "romeo.txt.zst", "romeo3.txt.zst", "welcome.zst", "skippables.zst"])
def test_cli_outputs(name, tmp_path):
    path = os.path.join(RES, name)
    data = open(path, "rb").read()
    for p in (False, True):
        want = oracle.decompress(data, p)
        r = cli(*(["-p"] if p else []), path)
        assert r.returncode == 0, r.stderr
        assert r.stdout == want
    out = tmp_path / "o.txt"
    r = cli(path, "-o", str(out))
    assert r.returncode == 0 and r.stdout == b"" and out.read_bytes() == oracle.decompress(data, False)


@pytest.mark.gpu
def test_cli_errors(tmp_path):
    from corpus import gen
    bad = tmp_path / "bad.zst"
    data = bytearray(open(os.path.join(RES, "romeo3.txt.zst"), "rb").read())
    data[4] |= 0x08                                   # reserved bit of the first frame header
    bad.write_bytes(bytes(data))
    r = cli(str(bad))
    assert r.returncode == 1 and r.stdout == b""
    binf = tmp_path / "bin.zst"
    binf.write_bytes(gen.frames(bytes(range(256)) * 64, 1 << 20, 3))
    r = cli(str(binf))
    assert r.returncode == 101 and r.stdout == b""
