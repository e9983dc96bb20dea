"""End-to-end pins of the reference's own sample inputs.

The reference ships `resources/*.zst` (copied byte-identical into
tests/golden/resources/) but no test of its own decodes them.  SURVEY §8c
records the SHA-256 of what the CLI (src/main.rs:43-58) writes for each, with
and without `-p/--print-skippable`; these digests were computed with libzstd
1.4.8 in the survey container (an RFC decoder that equals the reference on
these in-domain frames) and agree with the oracle.  The CPU test
pins the oracle to them; the `-m gpu` test pins the HIP path.
"""
import hashlib

import pytest

from oracle import oracle

DIGESTS = {
    # name: {print_skippable: (length, sha256)}
    "moby-dick.txt.zst": {False: (1276235, "61d5ab6a3910fab66eabc9d2fc708b68b756199cb754fd5ff51751dbe5f766cd"),
                          True: (1276235, "61d5ab6a3910fab66eabc9d2fc708b68b756199cb754fd5ff51751dbe5f766cd")},
    "romeo.txt.zst": {False: (942, "4854f5102035d288e8b8d6727cf25e0a44369e0a2dbaed7c02093bf3020979da"),
                      True: (942, "4854f5102035d288e8b8d6727cf25e0a44369e0a2dbaed7c02093bf3020979da")},
    "romeo3.txt.zst": {False: (2826, "51f5cdec8285f7686b0d75ebef96b6dbcd06e3ac0019b6b5c6595c132ff6295c"),
                       True: (2826, "51f5cdec8285f7686b0d75ebef96b6dbcd06e3ac0019b6b5c6595c132ff6295c")},
    "welcome.zst": {False: (126, "bc085b6464ec352b6fa9755b2bfdf8489775961027b3df432cb70e75d7d84242"),
                    True: (174, "7bcd1011853f3205233ec50a1194b15fdb4a5c36a884ac4b0d944785eac861d0")},
    # skippables only: nothing without -p; the payloads 10 20 30 42 with it
    "skippables.zst": {False: (0, "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
                       True: (4, "a3064ba7dbd296dbf1b6b3fd5d0201ffb96fa4a401a566438b8471f4621e0486")},
}


def _check(name, p, out):
    n, digest = DIGESTS[name][p]
    assert len(out) == n, f"{name} -p={p}: {len(out)} bytes, expected {n}"
    assert hashlib.sha256(out).hexdigest() == digest, f"{name} -p={p}: digest differs"


def test_oracle_resource_digests(resources):
    assert set(resources) == set(DIGESTS)
    for name, data in resources.items():
        for p in (False, True):
            st, out = oracle.decompress_status(data, p)
            assert st == 0, (name, p, st)
            _check(name, p, out)
    assert oracle.decompress(resources["skippables.zst"], True) == bytes([0x10, 0x20, 0x30, 0x42])


@pytest.mark.gpu
def test_gpu_resource_digests(resources):
    from zstd_decompressor.batch import decompress_status
    for name, data in resources.items():
        for p in (False, True):
            st, out = decompress_status(data, p)
            assert st == 0, (name, p, st)
            _check(name, p, out)
