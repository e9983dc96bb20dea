/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Not part of the product.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it, and only as the checker (or the timed CPU baseline), never as a
 * decode path of the product.
 *
 * A plain-C restatement of the reference Rust decoder
 * (AchilleBailly/zstd-decompressor, zstd-decompressor/src/…), function by
 * function, reference semantics included.
 * Parity pinning: the reference cannot be built here (no Rust toolchain),
 * so this restatement is pinned by (1) the reference's own known-answer
 * tests transcribed in tests/golden/kat.json and (2) libzstd 1.4.8 output on
 * in-domain frames (tests/golden/ sha256 files, tests/golden/make_golden.py).
 */
#ifndef ZD_ORACLE_H
#define ZD_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Error detail: code plus the payload some reference variants carry
 * (NotEnoughBytes/NotEnoughBits{requested, available},
 * MaximumReadableBitsExceeded(n), LargeAccuracyLog(al), UnrecognizedMagic). */
typedef struct zdo_err { int code; int64_t a, b; } zdo_err;

/* CLI semantics (src/main.rs:43-58): decode every frame of src, appending
 * ZStandard outputs (and skippable payloads when print_skippable); stops at
 * the first error.  *out is malloc'd (free with zdo_free) and holds the bytes
 * produced before the failure, if any.  *frames receives the number of frames
 * iterated successfully. */
int zdo_decompress(const uint8_t* src, size_t n, int print_skippable,
                   uint8_t** out, size_t* out_len, size_t* frames, zdo_err* err);

/* Frame::parse + Frame::decode for one frame at src (frame.rs:61-84). */
int zdo_frame_decode(const uint8_t* src, size_t n, size_t* consumed,
                     uint8_t** out, size_t* out_len, int* is_skippable, zdo_err* err);

void zdo_free(void* p);

/* ---- component-level entry points (reference KATs) ---- */
/* ForwardBitParser (parsing.rs:114-189): performs takes[i] bits reads. */
int zdo_forward_bits(const uint8_t* d, size_t n, const uint32_t* takes, size_t nt,
                     uint64_t* vals, uint64_t* len_after, zdo_err* err);
/* BackwardBitParser (parsing.rs:191-259). len_before = readable after new(). */
int zdo_backward_bits(const uint8_t* d, size_t n, const uint32_t* takes, size_t nt,
                      uint64_t* vals, uint64_t* len_before, uint64_t* len_after, zdo_err* err);
/* parse_fse_table (fse.rs:16-69); dist has room for 256 entries. */
int zdo_parse_fse_table(const uint8_t* d, size_t n, uint8_t* al, int16_t* dist,
                        size_t* nsym, uint64_t* bits_left, zdo_err* err);
/* FseTable::from_distribution (fse.rs:110-202); out: 3 u16 per state
 * (output, baseline, bits_to_read), 1<<al states. */
int zdo_fse_from_distribution(uint8_t al, const int16_t* dist, size_t n, uint16_t* out, zdo_err* err);
/* FseDecoder over an explicit table (fse.rs:230-323): initialize, then
 * nsym x (symbol, update_bits). table: 3 u16 per state. */
int zdo_fse_decode(const uint16_t* table, uint8_t al, const uint8_t* stream, size_t n,
                   size_t nsym, uint16_t* syms, zdo_err* err);
/* AlternatingDecoder (alternating.rs) over an explicit table: initialize,
 * then nsym x (symbol, update_bits). */
int zdo_alternating_decode(const uint16_t* table, uint8_t al, const uint8_t* stream, size_t n,
                           size_t nsym, uint16_t* syms, zdo_err* err);
/* HuffmanDecoder::from_weights + decode until the stream is empty
 * (huffman.rs:177-218, literals.rs:78-80). */
int zdo_huffman_weights_decode(const uint8_t* weights, size_t nw, const uint8_t* stream, size_t n,
                               uint8_t* out, size_t cap, size_t* nout, zdo_err* err);
/* HuffmanDecoder::parse (huffman.rs:80-130) from a tree description, then
 * decode the stream until empty. */
int zdo_huffman_parse_decode(const uint8_t* desc, size_t dn, size_t* consumed,
                             const uint8_t* stream, size_t n,
                             uint8_t* out, size_t cap, size_t* nout, zdo_err* err);
/* Huffman code widths (0 = absent) for the symbols of a tree description,
 * as from_weights computes them (huffman.rs:177-203); widths has 256+ room. */
int zdo_huffman_widths(const uint8_t* desc, size_t dn, uint8_t* widths, size_t* nwidths,
                       size_t* consumed, zdo_err* err);
/* DecodingContext::execute_sequences on a fresh context
 * (decoding_context.rs:78-106); seqs = nseq triples (ll, offset_value, ml). */
int zdo_execute_sequences(const uint64_t* seqs, size_t nseq, const uint8_t* lits, size_t nl,
                          uint8_t* out, size_t cap, size_t* nout, zdo_err* err);
/* Header::parse (frame.rs:111-177): fields out[0..4] = checksum_flag,
 * window_size, dict_id (UINT64_MAX none), content_size (UINT64_MAX none). */
int zdo_header_parse(const uint8_t* d, size_t n, uint64_t out[4], size_t* consumed, zdo_err* err);
/* Sequences of one compressed block inside a frame: decode blocks of the
 * frame at src up to block `block_index`, return that block's decoded
 * (ll, offset_value, ml) triples and literals (stage-level parity). */
int zdo_block_stages(const uint8_t* src, size_t n, size_t block_index,
                     uint64_t** seqs, size_t* nseq, uint8_t** lits, size_t* nlits, zdo_err* err);

#ifdef __cplusplus
}
#endif
#endif
