"""Command line, mirroring the reference CLI (src/main.rs:7-60):

    python -m zstd_decompressor FILE [-i/--info] [-o/--output FILE] [-p/--print-skippable]

Decodes every frame of FILE on the GPU (the HIP pipeline behind zd_decompress)
and writes the concatenated output to stdout or --output.  As in the
reference: skippable frames are dropped unless -p; the first failing frame
ends the run with its error (exit status 1, nothing written); the output must
be UTF-8 (the reference's `String::from_utf8(res).unwrap()` panics otherwise:
exit status 101).  --info prints one line per frame instead (the reference
prints the parsed frames with `{:#x?}`).  Extra, beyond the reference:
--check-checksums verifies Content_Checksum (XXH64) on the GPU and reports
mismatches on stderr (the reference computes and never enforces it).
"""
from __future__ import annotations

import argparse
import sys

from . import _lib
from .batch import Plan, frames_index


def _info(data: bytes) -> int:
    frames, blocks, st, _ = frames_index(data)
    for f in frames:
        if f["kind"] == 1:
            print(f"SkippableFrame(Skippable {{ magic: {f['magic']:#x}, data: {f['src_size'] - 8:#x} bytes }})")
            continue
        bs = blocks[f["first_block"]: f["first_block"] + f["num_blocks"]]
        kinds = ["Raw", "RLE", "Compressed"]
        cs = None if f["content_size"] == (1 << 64) - 1 else f["content_size"]
        did = None if f["dict_id"] == (1 << 64) - 1 else f["dict_id"]
        blist = ", ".join("%s(%#x)" % (kinds[b["type"]], b["block_size"]) for b in bs)
        chk = hex(f["checksum"]) if f["has_checksum"] else None
        print(f"ZStandardFrame(ZStandard {{ header: Header {{ content_checksum_flag: {bool(f['has_checksum'])}, "
              f"window_size: {f['window_size']:#x}, dictionnary_id: {did}, content_size: {cs} }}, "
              f"blocks: [{blist}], checksum: {chk} }})")
    if st != 0:
        print(f"Error: {_lib.status_name(st)}", file=sys.stderr)
        return 1
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="zstd_decompressor", description="ZStandard decoder on MI355X (HIP)")
    ap.add_argument("filename", help="ZStandard file input, decompress it and output to stdout")
    ap.add_argument("-i", "--info", action="store_true", help="Dump information about frames instead of the output")
    ap.add_argument("-o", "--output", metavar="filename", help="Output to given file (overwriting) instead of stdout")
    ap.add_argument("-p", "--print-skippable", action="store_true", help="Output Skippable frames as well")
    ap.add_argument("--check-checksums", action="store_true",
                    help="verify Content_Checksum (XXH64) on the GPU; mismatches go to stderr (not in the reference)")
    a = ap.parse_args(argv)
    data = open(a.filename, "rb").read()
    if a.info:
        return _info(data)
    import torch
    plan = Plan(data, a.print_skippable)
    dev = torch.device("cuda", torch.cuda.current_device())
    d_src = torch.zeros(len(data) + 64, dtype=torch.uint8, device=dev)
    if data:
        d_src[: len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    cap = max(int(plan.info.out_bytes), 1)
    d_dst = torch.empty(cap + 64, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    plan.decode_async(d_src.data_ptr(), d_dst.data_ptr(), cap, s)
    st, total, _, _, first = plan.results(d_dst.data_ptr(), s)
    if st != 0:
        print(f"Error: frame {first}: {_lib.status_name(st)}", file=sys.stderr)
        return 1
    if a.check_checksums:
        ok, _ = plan.checksums(d_dst.data_ptr(), s)
        for i, v in enumerate(ok):
            if v == 0:
                print(f"Warning: Bad checksum ! (frame {i})", file=sys.stderr)
    out = bytes(d_dst[:total].cpu().numpy().tobytes())
    try:
        text = out.decode("utf-8")
    except UnicodeDecodeError as e:
        print(f"thread 'main' panicked: called `Result::unwrap()` on an `Err` value: FromUtf8Error {{ {e} }}",
              file=sys.stderr)
        return 101
    if a.output:
        with open(a.output, "w", encoding="utf-8", newline="") as fo:
            fo.write(text)
    else:
        sys.stdout.write(text)
        sys.stdout.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
