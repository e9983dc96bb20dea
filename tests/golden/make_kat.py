"""Writes tests/golden/kat.json: the reference's own known-answer tests for the
hot path, transcribed as data (inputs + expected outputs).

Each entry cites the reference test it was transcribed from
(paths relative to the reference repo, AchilleBailly/zstd-decompressor).
Run: python tests/golden/make_kat.py
"""
import json
import os

NOT_ENOUGH_BYTES, NOT_ENOUGH_BITS, MAX_BITS, EMPTY_INPUT, NULL_BYTE = -1, -2, -3, -4, -5
RESERVED_BLOCK, UNRECOGNIZED_MAGIC, FRAME_RESERVED, MISSING_CHECKSUM, WINDOW_TOO_BIG = -50, -60, -61, -64, -66

ALT_TABLE = [[0, 1, 0], [3, 2, 1], [1, 0, 1], [0, 2, 1]]  # (output, baseline, bits_to_read), al 2

kat = {
    # --- parsing.rs: ForwardBitParser (LSB-first) ---
    "forward_bits": [
        {"src": "tests/parsing.rs:138-146", "data": [75, 0b0000_1111], "takes": [12], "vals": [(15 << 8) + 75], "len_after": 4},
        {"src": "tests/parsing.rs:148-158", "data": [0b0101_1010, 0b1100_0011], "takes": [3, 3, 4, 6],
         "vals": [0b010, 0b011, 0b1101, 0b110000], "len_after": 0},
        {"src": "tests/parsing.rs:128-136", "data": [75], "takes": [8], "vals": [75], "len_after": 0},
        {"src": "tests/parsing.rs:160-171", "data": [1] * 10, "takes": [67], "error": MAX_BITS, "err_a": 67, "len_after": 80},
        {"src": "tests/parsing.rs:173-187", "data": [1] * 6, "takes": [60], "error": NOT_ENOUGH_BITS, "err_a": 60, "err_b": 48, "len_after": 48},
        {"src": "tests/parsing.rs:80-87", "data": [], "takes": [], "error": EMPTY_INPUT},
    ],
    # --- parsing.rs: BackwardBitParser (reverse, skip padding + marker, MSB-first) ---
    "backward_bits": [
        {"src": "tests/parsing.rs:220-227", "data": [0], "takes": [], "error": NULL_BYTE},
        {"src": "tests/parsing.rs:229-236", "data": [], "takes": [], "error": EMPTY_INPUT},
        {"src": "tests/parsing.rs:238-245", "data": [1], "takes": [], "len_before": 0},
        {"src": "tests/parsing.rs:247-254", "data": [2], "takes": [], "len_before": 1},
        {"src": "tests/parsing.rs:265-273", "data": [0x5F, 1], "takes": [], "len_before": 8},
        {"src": "tests/parsing.rs:275-283", "data": [0x5F, 0xFF], "takes": [], "len_before": 15},
        {"src": "tests/parsing.rs:285-294", "data": [0x5F, 1], "takes": [8], "vals": [0b0101_1111], "len_after": 0},
        {"src": "tests/parsing.rs:296-304", "data": [0b0000_1111, 0b0111_0101, 1], "takes": [12], "vals": [0b0111_0101_0000], "len_after": 4},
        {"src": "tests/parsing.rs:306-317", "data": [0b0101_1010, 0b1100_0011, 1], "takes": [3, 3, 4, 6],
         "vals": [0b110, 0, 0b1101, 0b011010], "len_after": 0},
        {"src": "tests/parsing.rs:319-330", "data": [1] * 10, "takes": [67], "error": MAX_BITS, "err_a": 67, "len_after": 72},
        {"src": "tests/parsing.rs:332-346", "data": [1] * 6, "takes": [60], "error": NOT_ENOUGH_BITS, "err_a": 60, "err_b": 40, "len_after": 40},
    ],
    # --- decoders/fse.rs ---
    "parse_fse_table": [
        {"src": "tests/decoders/fse.rs:7-16", "data": [0x30, 0x6F, 0x9B, 0x03], "al": 5,
         "dist": [18, 6, 2, 2, 2, 1, 1], "bits_left": 6},
    ],
    "fse_from_distribution": [
        {"src": "tests/decoders/fse.rs:19-30", "al": 5, "dist": [18, 6, 2, 2, 2, 1, 1],
         "states": {"12": [1, 0x18, 3]}},
    ],
    "fse_table_parse": [
        {"src": "tests/decoders/fse.rs:33-58",
         "data": [0x21, 0x9D, 0x51, 0xCC, 0x18, 0x42, 0x44, 0x81, 0x8C, 0x94, 0xB4, 0x50, 0x1E],
         "states": {"63": [24, 0x10, 4], "44": [0, 0x34, 2]}},
    ],
    "fse_decode": [
        {"src": "tests/decoders/fse.rs:72-114", "table": ALT_TABLE, "al": 2, "stream": [0b1010_0000, 0b1111_0000],
         "symbols": [0, 0, 1, 0, 3, 1, 0, 3, 0, 1, 3]},
    ],
    "alternating_decode": [
        {"src": "tests/decoders/alternating.rs:58-77", "table": ALT_TABLE, "al": 2,
         "stream": [0b1001_1000, 0b0000_0001, 0b1111_1110],
         "symbols": [0, 0, 0, 0, 1, 1, 0, 0, 3, 3, 1, 1, 0, 0, 3, 3, 0, 0, 1, 1, 3, 3]},
    ],
    # --- decoders/huffman.rs ---
    "huffman_weights_decode": [
        {"src": "tests/decoders/huffman.rs:54-66 and tests/parsing.rs:205-218",
         "weights": [0] * 65 + [1, 2], "stream": [0x97, 0x01], "out": "BABCBB"},
    ],
    "huffman_parse_decode": [
        {"src": "tests/decoders/huffman.rs:68-95",
         # 127+67 header then 65 zeros, 1, 2 packed two 4-bit weights per byte (high nibble first)
         "desc": [127 + 67] + [0] * 32 + [(0 << 4) | 1, (2 << 4)], "stream": [0x97, 0x01], "out": "BABCBB"},
    ],
    "huffman_widths": [
        {"src": "tests/decoders/huffman.rs:7-16 (example_tree: A=2, B=1, C=2 bits)",
         "desc": [127 + 67] + [0] * 32 + [(0 << 4) | 1, (2 << 4)], "widths_at": {"65": 2, "66": 1, "67": 2}},
    ],
    # --- decoding_context.rs inline KAT ---
    "execute_sequences": [
        {"src": "src/decoding_context.rs:109-122", "seqs": [[3, 5, 3], [2, 11, 1]],
         "literals": [0x61, 0x62, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68],
         "out": [0x61, 0x62, 0x63, 0x62, 0x63, 0x62, 0x64, 0x65, 0x61, 0x66, 0x67, 0x68]},
    ],
    # --- frame.rs inline tests + tests/frame.rs header tests ---
    "window_descriptor": [
        {"src": "src/frame.rs:282-289", "byte": 0x00, "window": 1 << 10},
        {"src": "src/frame.rs:291-299", "byte": 0xFF, "window": (1 << 41) + 7 * (1 << 38)},
        {"src": "src/frame.rs:301-309", "byte": 0x01, "window": (1 << 10) + 1024 // 8},
    ],
    "header_parse": [
        {"src": "tests/frame.rs:155-168", "data": [0b01_1_0_0_0_00, 0xCC, 0xCC],
         "checksum": False, "window": 0xCCCC + 256, "fcs": 0xCCCC + 256, "dict": None},
        {"src": "tests/frame.rs:171-187", "data": [0b01_0_0_0_0_00, 0x00, 0xCC, 0xDD],
         "checksum": False, "window": 1024, "fcs": 0xDDCC + 256, "dict": None},
        {"src": "tests/frame.rs:190-199", "data": [0b01_0_0_1_0_00], "error": FRAME_RESERVED},
        {"src": "tests/frame.rs:202-220", "data": [0b01_0_0_0_0_10, 0x00, 0xEF, 0xAB, 0xCC, 0xDD],
         "checksum": False, "window": 1024, "fcs": 0xDDCC + 256, "dict": 0xABEF},
        {"src": "tests/frame.rs:223-257",
         "data": [0b11_0_0_0_0_11, 0x00, 0xEF, 0xAB, 0xEF, 0xAB, 0xCC, 0xDD, 0xCC, 0xDD, 0xCC, 0xDD, 0xCC, 0xDD],
         "checksum": False, "window": 1024, "fcs": 0xDDCCDDCCDDCCDDCC, "dict": 0xABEFABEF},
    ],
    # Whole inputs through Frame::parse/decode (CLI-style iteration).
    "frames": [
        {"src": "tests/frame.rs:6-14,40-49,72-78", "data": [0x53, 0x2A, 0x4D, 0x18, 0x03, 0, 0, 0, 0x10, 0x20, 0x30],
         "skippable_out": [0x10, 0x20, 0x30], "out": []},
        {"src": "tests/frame.rs:16-38,51-61 (single segment, checksum 1, raw block)",
         "data": [0x28, 0xB5, 0x2F, 0xFD, 0b01_1_0_0_1_00, 0x04, 0x00, 0x21, 0x0, 0x0, 0x10, 0x20, 0x30, 0x40, 0x01, 0, 0, 0],
         "out": [0x10, 0x20, 0x30, 0x40]},
        {"src": "tests/frame.rs:63-70", "data": [0x10, 0x20, 0x30, 0x40], "error": UNRECOGNIZED_MAGIC, "err_a": 0x40302010},
        {"src": "tests/frame.rs:88-107", "data": [0x53, 0x2A, 0x4D, 0x18, 0x03, 0, 0, 0, 0x10, 0x20],
         "error": NOT_ENOUGH_BYTES, "err_a": 3, "err_b": 2},
        {"src": "tests/frame.rs:109-127", "data": [0x53, 0x2A, 0x4D, 0x18, 0x03, 0, 0],
         "error": NOT_ENOUGH_BYTES, "err_a": 4, "err_b": 3},
        {"src": "tests/frame.rs:129-146", "data": [0x53, 0x2A, 0x4D], "error": NOT_ENOUGH_BYTES, "err_a": 4, "err_b": 3},
        {"src": "tests/frame.rs:316-343 (checksum flag but no checksum)",
         "data": [0x28, 0xB5, 0x2F, 0xFD, 0b01_1_0_0_1_00, 0x04, 0x00, 0x21, 0x0, 0x0, 0x10, 0x20, 0x30, 0x40, 0x42],
         "error": MISSING_CHECKSUM},
        {"src": "tests/frame.rs:345-372 (window 0xff too big)",
         "data": [0x28, 0xB5, 0x2F, 0xFD, 0b01_0_0_0_1_00, 0xFF, 0x04, 0x05, 0x21, 0x0, 0x0, 0x10, 0x20, 0x30, 0x40, 0x42],
         "error": WINDOW_TOO_BIG},
        {"src": "tests/frame.rs:376-398 (two skippable frames)",
         "data": [0x53, 0x2A, 0x4D, 0x18, 0x03, 0, 0, 0, 0x10, 0x20, 0x30, 0x51, 0x2A, 0x4D, 0x18, 0x04, 0, 0, 0,
                  0x10, 0x20, 0x30, 0x40],
         "skippable_out": [0x10, 0x20, 0x30, 0x10, 0x20, 0x30, 0x40], "out": []},
        {"src": "tests/block.rs:12-26 (raw last block inside a frame)",
         "data": [0x28, 0xB5, 0x2F, 0xFD, 0b00_1_0_0_0_00, 0x04, 0x21, 0x0, 0x0, 0x10, 0x20, 0x30, 0x40],
         "out": [0x10, 0x20, 0x30, 0x40]},
        {"src": "tests/block.rs:28-49 (RLE block 0x42 x 196612, then a raw last block)",
         "data": [0x28, 0xB5, 0x2F, 0xFD, 0b00_0_0_0_0_00, 0x68, 0x22, 0x0, 0x18, 0x42, 0x09, 0x0, 0x0, 0x50],
         "out_rle": [0x42, 196612, 0x50]},
        {"src": "tests/block.rs:51-61 (reserved block type)",
         "data": [0x28, 0xB5, 0x2F, 0xFD, 0b00_1_0_0_0_00, 0x04, 0x27, 0x0, 0x0, 0x10, 0x20, 0x30, 0x40, 0x50],
         "error": RESERVED_BLOCK},
        {"src": "tests/block.rs:63-79 (truncated raw block)",
         "data": [0x28, 0xB5, 0x2F, 0xFD, 0b00_1_0_0_0_00, 0x04, 0x21, 0x0, 0x0, 0x10, 0x20, 0x30],
         "error": NOT_ENOUGH_BYTES, "err_a": 4, "err_b": 3},
        {"src": "tests/decoders/sequence.rs:6-31 (fuzz regression: must not panic)",
         "data": [40, 181, 47, 253, 0, 10, 165, 0, 0, 85, 47, 0, 252, 59, 64, 44, 0, 51, 29, 44, 47, 10,
                  40, 0, 181, 181, 40, 181, 47, 253],
         "no_panic": True},
    ],
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat.json")
    with open(out, "w") as f:
        json.dump(kat, f, indent=1)
    print("wrote", out)
