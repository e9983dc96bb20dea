"""Seeded synthetic corpora for the configs of BASELINE.json.

Nothing here decodes: libzstd is only the compressor.  Inputs are built from
the reference's own sample text (tests/golden/resources/moby-dick.txt.zst,
decoded once by libzstd) so that the GPU box, which has no /root/reference,
can regenerate them.

  c2_raw_rle()        single 64 MiB frame, 512 alternating raw/RLE blocks
  text(n, seed)       enwik-style wiki-XML text (word spans + markup)
  xml(n, seed)        Silesia-xml proxy
  binary(n, seed)     Silesia-mozilla proxy (pseudo-ELF/tar bytes)
  frames(data, chunk, level)  independent frames of `chunk` bytes each
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import struct

import numpy as np

from . import libzstd

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
_MOBY = os.path.join(_ROOT, "tests", "golden", "resources", "moby-dick.txt.zst")
SEED = 0x5EED

_words_cache = None


def _words():
    """(word bytes table, offsets, lengths) from the decoded moby-dick text."""
    global _words_cache
    if _words_cache is None:
        raw = open(_MOBY, "rb").read()
        txt = libzstd.decompress_frame(raw, libzstd.frame_content_size(raw))
        ws = txt.split()
        lens = np.fromiter((len(w) for w in ws), dtype=np.int64, count=len(ws))
        offs = np.zeros(len(ws) + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        _words_cache = (np.frombuffer(b"".join(ws), dtype=np.uint8), offs, lens)
    return _words_cache


def _gather_words(rng, nbytes: int) -> np.ndarray:
    """~nbytes of text made of random spans of 1-12 consecutive source words."""
    table, offs, lens = _words()
    nw = len(lens)
    est = int(nbytes / 5.5) + 64
    nspan = est // 6 + 1
    starts = rng.integers(0, nw - 13, size=nspan)
    slen = rng.integers(1, 13, size=nspan)
    idx = np.repeat(starts, slen) + (np.arange(slen.sum()) - np.repeat(np.cumsum(slen) - slen, slen))
    wl = lens[idx] + 1                       # word + separator
    total = int(wl.sum())
    out_pos = np.cumsum(wl) - wl
    # byte gather: for every output byte, its source byte
    word_of_byte = np.repeat(np.arange(len(idx)), wl)
    k = np.arange(total) - out_pos[word_of_byte]
    src = offs[idx][word_of_byte] + k
    is_sep = k == lens[idx][word_of_byte]
    out = np.empty(total, dtype=np.uint8)
    out[~is_sep] = table[src[~is_sep]]
    sep = np.where(rng.random(int(is_sep.sum())) < 0.08, 10, 32).astype(np.uint8)
    out[is_sep] = sep
    return out[:nbytes] if total >= nbytes else out


def text(nbytes: int, seed: int = SEED) -> bytes:
    """enwik-style: <page> records of wiki markup around word-span prose."""
    rng = np.random.default_rng(seed)
    pieces, total, page = [], 0, int(rng.integers(1, 10 ** 6))
    while total < nbytes:
        body = _gather_words(rng, int(rng.integers(1500, 9000))).tobytes()
        page += int(rng.integers(1, 40))
        title = _gather_words(rng, int(rng.integers(8, 40))).tobytes().replace(b"\n", b" ").strip()
        head = (b"  <page>\n    <title>" + title + b"</title>\n    <id>" + str(page).encode() +
                b"</id>\n    <revision>\n      <id>" + str(page * 7 + 13).encode() +
                b"</id>\n      <timestamp>2006-0" + str(int(rng.integers(1, 10))).encode() +
                b"-1" + str(int(rng.integers(0, 10))).encode() + b"T0" + str(int(rng.integers(0, 10))).encode() +
                b":34:56Z</timestamp>\n      <text xml:space=\"preserve\">")
        tail = b"</text>\n    </revision>\n  </page>\n"
        # sprinkle wiki links / emphasis
        if len(body) > 64:
            j = int(rng.integers(0, len(body) - 32))
            body = body[:j] + b"[[" + body[j:j + 12].replace(b"\n", b" ") + b"]]" + body[j + 12:]
        pieces += [head, body, tail]
        total += len(head) + len(body) + len(tail)
    return b"".join(pieces)[:nbytes]


def xml(nbytes: int, seed: int = SEED + 1) -> bytes:
    rng = np.random.default_rng(seed)
    names = [w for w in _gather_words(rng, 20000).tobytes().split() if w.isalpha()][:500] or [b"x"]
    pieces, total, i = [b'<?xml version="1.0"?>\n<table>\n'], 0, 0
    while total < nbytes:
        n = int(rng.integers(50, 200))
        ids = rng.integers(0, 10 ** 6, size=n)
        vals = rng.integers(0, 10 ** 4, size=n)
        kinds = rng.integers(0, len(names), size=n)
        rows = b"".join(b'  <row id="%d" name="%s" value="%d.%02d" flag="%s"/>\n'
                        % (ids[r], names[kinds[r]], vals[r] // 100, vals[r] % 100,
                           b"true" if vals[r] & 1 else b"false") for r in range(n))
        pieces.append(rows)
        total += len(rows)
        i += 1
    pieces.append(b"</table>\n")
    return b"".join(pieces)[:nbytes]


def binary(nbytes: int, seed: int = SEED + 2) -> bytes:
    """Pseudo-ELF: Zipf-distributed 'instruction' byte strings, LE addresses,
    zero padding and embedded strings."""
    rng = np.random.default_rng(seed)
    vocab = [rng.integers(0, 256, size=int(rng.integers(1, 9)), dtype=np.uint8).tobytes() for _ in range(600)]
    p = 1.0 / np.arange(1, len(vocab) + 1) ** 1.1
    p /= p.sum()
    strings = [w for w in _gather_words(rng, 8000).tobytes().split()][:300]
    out, total = [b"\x7fELF\x02\x01\x01\x00" + bytes(8)], 16
    while total < nbytes:
        r = rng.random()
        if r < 0.80:
            ks = rng.choice(len(vocab), size=64, p=p)
            addr = rng.integers(0x400000, 0x480000, size=64)
            chunk = b"".join(vocab[k] + (struct.pack("<I", int(a)) if (k & 3) == 0 else b"") for k, a in zip(ks, addr))
        elif r < 0.9:
            chunk = bytes(int(rng.integers(4, 256)))
        else:
            chunk = b"\0".join(strings[int(i)] for i in rng.integers(0, len(strings), size=8)) + b"\0"
        out.append(chunk)
        total += len(chunk)
    return b"".join(out)[:nbytes]


def c2_raw_rle(total: int = 64 << 20, block: int = 128 << 10, seed: int = SEED + 3,
               with_content: bool = False):
    """C2: one frame, not single-segment (window descriptor 0x68 = 8 MiB),
    4-byte FCS, alternating Raw (random bytes) / RLE (byte = index & 0xFF)
    blocks, no checksum.  with_content: (frame bytes, the content they carry)."""
    rng = np.random.default_rng(seed)
    nb = total // block
    out = [struct.pack("<I", 0xFD2FB528), bytes([0x80, 0x68]), struct.pack("<I", total)]
    content = []
    for i in range(nb):
        last = 1 if i == nb - 1 else 0
        if i % 2 == 0:
            out.append(struct.pack("<I", last | (0 << 1) | (block << 3))[:3])
            raw = rng.integers(0, 256, size=block, dtype=np.uint8).tobytes()
            out.append(raw)
            content.append(raw)
        else:
            out.append(struct.pack("<I", last | (1 << 1) | (block << 3))[:3])
            out.append(bytes([i & 0xFF]))
            content.append(bytes([i & 0xFF]) * block)
    if with_content:
        return b"".join(out), b"".join(content)
    return b"".join(out)


def frames(data: bytes, chunk: int, level: int = 3, threads: int | None = None,
           checksum: bool = False, window_log: int = 0, content_size: bool = True) -> bytes:
    """Independent frames of `chunk` decompressed bytes each (last may be short)."""
    parts = [data[i:i + chunk] for i in range(0, len(data), chunk)]
    threads = threads or min(16, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(threads) as ex:
        out = list(ex.map(lambda p: libzstd.compress(p, level, checksum, window_log, content_size), parts))
    return b"".join(out)


def replicate(frame_set: bytes, times: int) -> bytes:
    return frame_set * times
