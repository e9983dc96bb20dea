// zd_common.h — descriptors shared by the host planner (zd_host.cpp) and the
// gfx950 kernels (zd_kernels.hip).  Layout is plain-old-data, 8-byte aligned,
// uploaded once per plan.
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define ZD_HD __host__ __device__
#else
#define ZD_HD
#endif

namespace zd {

constexpr int LUT_MAX_BITS = 12;                 // Huffman LUT covers maxBits <= 12
constexpr int LUT_ENTRIES = 1 << LUT_MAX_BITS;   // u16 entries per LUT slot
constexpr int FSE_MAX_AL = 9;                    // MAX_AL (fse.rs:13)
constexpr int FSE_ENTRIES = 1 << FSE_MAX_AL;     // u32 entries per table
constexpr int MAX_WEIGHTS = 2048;                // cap on FSE-decoded Huffman weights
constexpr uint64_t MAX_WIN_SIZE = 8ull << 20;    // frame.rs:44
constexpr uint32_t MAX_BLOCK_OUT = 128u << 10;   // RFC Block_Maximum_Size (capacity bound only)

// LUT entry: symbol | nbits << 8 | ABSENT (depth of the absent tree node in nbits)
constexpr uint16_t LUT_ABSENT = 0x8000;

// FSE decode entry, 16 bits: symbol (clamped to 63) | nextState << 6.
// FseTable::from_distribution (fse.rs:169-189) gives state u of symbol s
// nextState ns = count(s) + u in [1, 2T); the reference's {bits_to_read,
// baseline} are recovered as nb = AL - highbit(ns), base = (ns << nb) - T.
// Every sequence code above 63 is already past LL/ML/OF maxima (35/52/31) and
// every Huffman weight above 32 already panics, so the clamp keeps behaviour.
constexpr int FSE_TAB = 1 << FSE_MAX_AL;           // u16 entries per table in a slot
// K1's pool for the symbols of deep Huffman trees with more leaves than a
// LUT slot holds (only a weight stream of > 7,680 nonzero weights makes one)
constexpr uint64_t DEEP_POOL_BYTES = 4ull << 20;
constexpr int FSE_SLOT = 3 * FSE_TAB;              // LL | OF | ML
ZD_HD inline uint16_t fse_entry(uint32_t sym, uint32_t ns) { return (uint16_t)((sym > 63 ? 63 : sym) | (ns << 6)); }
ZD_HD inline int hb32(uint32_t v) {
#ifdef __HIP_DEVICE_COMPILE__
  return 31 - __clz(v);
#else
  return 31 - __builtin_clz(v);
#endif
}
ZD_HD inline uint32_t fse_sym(uint16_t e) { return e & 63; }
ZD_HD inline uint32_t fse_nb(uint16_t e, int al) { return (uint32_t)(al - hb32((uint32_t)e >> 6)); }
ZD_HD inline uint32_t fse_base(uint16_t e, int al) {
  uint32_t ns = (uint32_t)e >> 6;
  return (ns << fse_nb(e, al)) - (1u << al);
}

// Sequence codes -> (baseline, extra bits) (decoders/sequence.rs:98-191) as
// arithmetic instead of the reference's linear table search (sequence.rs:36).
// Offsets 16..24 (LL) / 32..42 (ML) above the base: 0,2,4,6 then
// (2 + odd) << (k >> 1).
ZD_HD inline uint32_t code_step(uint32_t k) {
  return ((2u + (k & 1)) << ((k >> 1) & 31)) - (k < 2 ? 2 - k : 0);
}
// (branch-free: selects, no divergent control flow in the per-lane decoders)
ZD_HD inline void ll_code(uint32_t c, uint32_t* base, uint32_t* bits) {
  const uint32_t k = (c - 16) & 15, hi = (c - 19) & 31;
  const uint32_t mb = k < 2 ? 1 : (k >> 1), mbase = 16 + code_step(k);
  *bits = c < 16 ? 0 : (c < 25 ? mb : hi);
  *base = c < 16 ? c : (c < 25 ? mbase : (1u << hi));
}
ZD_HD inline void ml_code(uint32_t c, uint32_t* base, uint32_t* bits) {
  const uint32_t k = (c - 32) & 15, hi = (c - 36) & 31;
  const uint32_t mb = k < 2 ? 1 : (k >> 1), mbase = 35 + code_step(k);
  *bits = c < 32 ? 0 : (c < 43 ? mb : hi);
  *base = c < 32 ? c + 3 : (c < 43 ? mbase : (1u << hi) + 3);
}

// K3's chain-format table entry (16 bits), re-encoded from a sym entry of
// table k (0 LL, 1 OF, 2 ML) when K3 loads it into LDS: nextState (10 bits)
// | extra-bit count of the symbol's code << 10 (5 bits) | K3_BAD for a code
// above the maximum (LL 35, OF 31, ML 52: decoders/sequence.rs:95-97).
constexpr uint32_t K3_BAD = 1u << 15;
ZD_HD inline uint32_t k3_entry(uint32_t e, int k) {
  const uint32_t c = e & 63, ns = (e >> 6) & 1023;
  uint32_t base, eb, bad;
  if (k == 0) { ll_code(c, &base, &eb); bad = c > 35; }
  else if (k == 2) { ml_code(c, &base, &eb); bad = c > 52; }
  else { eb = c; bad = c > 31; }
  return ns | ((eb & 31) << 10) | (bad ? K3_BAD : 0u);
}
// K3's fast chain (zd_kernels.hip seq_chainfl) reads one number per table per
// step: nextState | (extra-bit count + state-bit count) << 10, with the
// count 63 (never reached: <= 31 + 9) marking a code above the maximum.
constexpr uint32_t K3F_BAD = 63u << 10;
ZD_HD inline uint32_t k3f_entry(uint32_t e, int k, int al) {
  const uint32_t c = e & 63, ns = (e >> 6) & 1023;
  uint32_t base, eb;
  bool bad;
  if (k == 0) { ll_code(c, &base, &eb); bad = c > 35; }
  else if (k == 2) { ml_code(c, &base, &eb); bad = c > 52; }
  else { eb = c; bad = c > 31; }
  const uint32_t nb = (uint32_t)(al - hb32(ns));
  return ns | (bad ? K3F_BAD : (eb + nb) << 10);
}

// ---------------------------------------------------------------------------
// Sequence records (K3 -> K4), 8 bytes per sequence:
//   from K3 (FSE chain): for each sequence the bit position of its extra
//     bits (their top, before OF/ML/LL are read) and the LL / ML / OF states;
//     K4 decodes the values (decoders/sequence.rs:41-55).  They come in pairs,
//     sequences 2p and 2p + 1 in 16 bytes (a block's first record index is
//     even), four dwords each written by one lane of K3Q's quad (OF | ML | LL
//     | shadow) with no cross-lane moves:
//       x  OF state of 2p | OF state of 2p+1 << 10 | (pos_2p - pos_2p+1) << 20
//       y  ML states (bits 0-9, 10-19)       z  LL states
//       w  pos_2p
//     (a step reads at most 89 bits, so the position difference fits 12 bits;
//     states are below 2^9).  rec_unpack gives one record of a pair in the
//     consumers' one-word form: pos | (LL | ML << 10 | OF << 20) << 32.
//   direct (zd_execute_sequences, CompBlock::seq_direct): bits 0-16
//     literals_length, 17-34 match_length, 35-63 offset_value, where
//     DIRECT_GIANT stands for any offset_value >= 2^29 - 1 (an offset past
//     every frame the GPU path accepts: ImpossibleValue when used).
// Repeat offsets (decoding_context.rs:50-75) are resolved by K4 in frame
// order with concrete values.
// ---------------------------------------------------------------------------
ZD_HD inline uint64_t rec_unpack(uint32_t x, uint32_t y, uint32_t z, uint32_t w, uint32_t h) {
  const uint32_t sh = 10 * h;
  const uint32_t st = ((z >> sh) & 1023) | (((y >> sh) & 1023) << 10) | (((x >> sh) & 1023) << 20);
  const uint32_t pos = h ? w - (x >> 20) : w;
  return (uint64_t)pos | ((uint64_t)st << 32);
}
// the pair of records (posA, stA), (posB, stB) -- st = LL | ML << 10 | OF << 20
ZD_HD inline void rec_pack(uint32_t posA, uint32_t stA, uint32_t posB, uint32_t stB, uint32_t v[4]) {
  v[0] = (stA >> 20) | ((stB >> 20) << 10) | ((posA - posB) << 20);
  v[1] = ((stA >> 10) & 1023) | (((stB >> 10) & 1023) << 10);
  v[2] = (stA & 1023) | ((stB & 1023) << 10);
  v[3] = posA;
}
// record slots a block of n sequences takes (pairs, and one spare pair that
// the chains write past the last)
ZD_HD inline uint64_t rec_slots(uint32_t n) { return n ? ((uint64_t)(n + 1) & ~1ull) + 2 : 0; }
constexpr uint32_t DIRECT_GIANT = (1u << 29) - 1;
// Output bounds per executor: the streaming K4 keeps int32 frame positions;
// K4J u64 positions and 31-bit distances in its state words, up to 32 GiB a
// frame.  A frame with sequences above both is outside the GPU path's domain
// (ZD_E_OUT_OF_DOMAIN; the reference's own limit is the 8 MiB window).
constexpr uint64_t K4_MAX_FRAME_OUT = 0x7FFF0000ull;
constexpr uint64_t K4J_MAX_FRAME_OUT = 1ull << 35;   // 32 GiB: 128 GiB of K4J state words
constexpr uint64_t OFF_HUGE = ~0ull >> 1;        // a giant offset (never <= a decoded length)

ZD_HD inline uint64_t seq_pack(uint32_t ll, uint32_t ml, uint32_t ofv) {
  return (uint64_t)ll | ((uint64_t)ml << 17) | ((uint64_t)(ofv > DIRECT_GIANT ? DIRECT_GIANT : ofv) << 35);
}
ZD_HD inline uint32_t seq_ll(uint64_t s) { return (uint32_t)(s & 0x1FFFF); }
ZD_HD inline uint32_t seq_ml(uint64_t s) { return (uint32_t)((s >> 17) & 0x3FFFF); }
ZD_HD inline uint32_t seq_off(uint64_t s) { return (uint32_t)(s >> 35); }
// A direct record with a field at its maximum (literals_length >= 2^17 - 1,
// match_length >= 2^18 - 1 or offset_value >= DIRECT_GIANT) is an escape:
// its exact values are the record's DirectSide entry (CompBlock::seq_side,
// same index), so the context API takes any u32 triple.
struct DirectSide { uint32_t ll, ml, ofv, pad; };
constexpr uint64_t DIRECT_ESCAPE = (uint64_t)0x1FFFF | ((uint64_t)0x3FFFF << 17) | ((uint64_t)DIRECT_GIANT << 35);
ZD_HD inline bool seq_escaped(uint64_t s) {
  return seq_ll(s) == 0x1FFFF || seq_ml(s) == 0x3FFFF || seq_off(s) == DIRECT_GIANT;
}
// record i's values (side: the block's DirectSide entries)
ZD_HD inline void seq_values(uint64_t s, uint64_t side, uint32_t i, uint32_t* ll, uint32_t* ml, uint32_t* ofv) {
  if (side && seq_escaped(s)) {
    const DirectSide d = ((const DirectSide*)side)[i];
    *ll = d.ll; *ml = d.ml; *ofv = d.ofv;
  } else {
    *ll = seq_ll(s); *ml = seq_ml(s); *ofv = seq_off(s);
  }
}

// ---------------------------------------------------------------------------
// Repeat-offset codes (u32) for resolving decode_offset (decoding_context.rs:
// 50-75) by a parallel scan (K4F).  A segment of sequences maps the three
// incoming repeat offsets to three outgoing ones, each either a concrete
// value or "incoming slot j minus d" (d decrements of the `3, ll == 0` rule):
//   v <  OFF_SYM                    concrete offset v
//   OFF_SYM + (j << 24) + d         incoming rep[j] - d
//   OFF_GIANT                       an offset >= 2^28: past any frame K4F
//                                   decodes (ImpossibleValue when used)
//   OFF_NULL                        offset_value 0 (NullOffsetError)
//   OFF_UNDERFLOW                   usize underflow of rep0 - 1 (ZD_E_REF_PANIC)
// Maps compose with rc_apply, so the state before every thread's sequences
// is an exclusive scan of the threads' maps.
// ---------------------------------------------------------------------------
constexpr uint32_t OFF_SYM = 1u << 28;
constexpr uint32_t OFF_GIANT = (1u << 29) - 3;
constexpr uint32_t OFF_NULL = (1u << 29) - 2;
constexpr uint32_t OFF_UNDERFLOW = (1u << 29) - 1;

ZD_HD inline void rep_ident(uint32_t r[3]) { r[0] = OFF_SYM; r[1] = OFF_SYM | (1u << 24); r[2] = OFF_SYM | (2u << 24); }
ZD_HD inline uint32_t rep_code(uint64_t v) { return v < OFF_SYM ? (uint32_t)v : OFF_GIANT; }
ZD_HD inline uint64_t rep_value(uint32_t c) { return c < OFF_SYM ? (uint64_t)c : OFF_HUGE; }
ZD_HD inline uint32_t rep_dec1(uint32_t v) {
  // giant stays giant; after an underflow the reference stopped; a symbolic
  // value counts one more decrement; 0 underflows (selects, no branches)
  uint32_t t = v >= OFF_SYM ? v + 1 : v - 1;
  t = v == 0 ? OFF_UNDERFLOW : t;
  return v >= OFF_GIANT ? v : t;
}
// decode_offset on codes: updates r, returns the offset code.  idx = the
// repeat slot an offset_value <= 3 names (RFC 8878 3.1.1.5), 3 = rep0 - 1.
ZD_HD inline uint32_t rep_step(uint32_t r[3], uint32_t ofv, uint32_t ll) {
  const uint32_t r0 = r[0], r1 = r[1], r2 = r[2];
  const bool fresh = ofv > 3;
  const uint32_t idx = ofv - (ll != 0 ? 1u : 0u);
  uint32_t rep = idx == 0 ? r0 : r1;
  rep = idx >= 2 ? r2 : rep;
  rep = idx == 3 ? rep_dec1(r0) : rep;
  const uint32_t v = ofv - 3;
  const uint32_t n0 = fresh ? (v >= OFF_SYM ? OFF_GIANT : v) : rep;
  const uint32_t n1 = (!fresh && idx == 0) ? r1 : r0;
  const uint32_t n2 = (!fresh && idx <= 1) ? r2 : r1;
  const bool null = ofv == 0;
  r[0] = null ? r0 : n0;
  r[1] = null ? r1 : n1;
  r[2] = null ? r2 : n2;
  return null ? OFF_NULL : n0;
}
// code b evaluated with the incoming slots a[3] (which may be codes too)
ZD_HD inline uint32_t rc_apply(uint32_t b, const uint32_t a[3]) {
  if (b < OFF_SYM || b >= OFF_GIANT) return b;
  const uint32_t j = (b - OFF_SYM) >> 24, d = (b - OFF_SYM) & 0xFFFFFFu;
  const uint32_t x = j == 0 ? a[0] : (j == 1 ? a[1] : a[2]);
  if (x >= OFF_GIANT) return x;
  if (x >= OFF_SYM) return x + d;
  return x >= d ? x - d : OFF_UNDERFLOW;
}
// map b after map a (a's outputs feed b's inputs)
ZD_HD inline void rc_compose(const uint32_t a[3], uint32_t b[3]) {
  const uint32_t c0 = rc_apply(b[0], a), c1 = rc_apply(b[1], a), c2 = rc_apply(b[2], a);
  b[0] = c0; b[1] = c1; b[2] = c2;
}

// 64-bit repeat-offset codes for K4J's per-block maps (the K4F codes above
// cap offsets at 2^28; K4J frames go to 4 GiB).  Concrete offsets are below
// 2^33 (offset_value < 2^32, decrements), so these stay exact:
//   v < J_SYM                concrete v; J_UNDER = a value after a usize
//                            underflow (the sequence that underflowed reports
//                            ZD_E_REF_PANIC; what follows in the frame is moot)
//   J_SYM | j << 48 | d      incoming rep[j] - d
constexpr uint64_t J_SYM = 1ull << 63;
constexpr uint64_t J_UNDER = 1ull << 62;
constexpr uint64_t J_DMASK = (1ull << 48) - 1;
ZD_HD inline uint64_t jr_sym(uint32_t j) { return J_SYM | ((uint64_t)j << 48); }
ZD_HD inline uint64_t jr_dec1(uint64_t v) {
  if (v >= J_SYM) return v + 1;
  return (v == 0 || v >= J_UNDER) ? J_UNDER : v - 1;
}
// code b evaluated on the incoming slots a[3] (codes or concrete)
ZD_HD inline uint64_t jr_apply(uint64_t b, const uint64_t a[3]) {
  if (b < J_SYM) return b;
  const uint32_t j = (uint32_t)((b >> 48) & 3);
  const uint64_t d = b & J_DMASK;
  const uint64_t x = j == 0 ? a[0] : (j == 1 ? a[1] : a[2]);
  if (x >= J_SYM) return x + d;
  if (x >= J_UNDER) return J_UNDER;
  return x >= d ? x - d : J_UNDER;
}

// ---------------------------------------------------------------------------
// XXH64 (seed 0) pieces, for the content-checksum pass (frame.rs:239-255: the
// reference computes this hash but never enforces it; verifying it
// is an extra, reported apart from the decode status).
// ---------------------------------------------------------------------------
constexpr uint64_t XP1 = 0x9E3779B185EBCA87ull, XP2 = 0xC2B2AE3D27D4EB4Full, XP3 = 0x165667B19E3779F9ull,
                   XP4 = 0x85EBCA77C2B2AE63ull, XP5 = 0x27D4EB2F165667C5ull;
ZD_HD inline uint64_t xx_rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
ZD_HD inline uint64_t xx_round(uint64_t acc, uint64_t in) { return xx_rotl(acc + in * XP2, 31) * XP1; }
ZD_HD inline uint64_t xx_merge(uint64_t h, uint64_t v) { return (h ^ xx_round(0, v)) * XP1 + XP4; }
ZD_HD inline uint64_t xx_acc_init(int i) { return i == 0 ? XP1 + XP2 : (i == 1 ? XP2 : (i == 2 ? 0 : 0 - XP1)); }
// h from the four accumulators (len >= 32) or XP5 (len < 32), then the tail
// bytes p[0, rem) (rem < 32) and the avalanche
ZD_HD inline uint64_t xx_finish(uint64_t len, const uint64_t v[4], const uint8_t* p, uint32_t rem) {
  uint64_t h;
  if (len >= 32) {
    h = xx_rotl(v[0], 1) + xx_rotl(v[1], 7) + xx_rotl(v[2], 12) + xx_rotl(v[3], 18);
    for (int i = 0; i < 4; i++) h = xx_merge(h, v[i]);
  } else {
    h = XP5;
  }
  h += len;
  uint32_t i = 0;
  for (; i + 8 <= rem; i += 8) {
    uint64_t k = 0;
    for (int b = 7; b >= 0; b--) k = (k << 8) | p[i + b];
    h = xx_rotl(h ^ xx_round(0, k), 27) * XP1 + XP4;
  }
  if (i + 4 <= rem) {
    uint64_t k = (uint64_t)p[i] | ((uint64_t)p[i + 1] << 8) | ((uint64_t)p[i + 2] << 16) | ((uint64_t)p[i + 3] << 24);
    h = xx_rotl(h ^ (k * XP1), 23) * XP2 + XP3;
    i += 4;
  }
  for (; i < rem; i++) h = xx_rotl(h ^ (p[i] * XP5), 11) * XP1;
  h ^= h >> 33;
  h *= XP2;
  h ^= h >> 29;
  h *= XP3;
  h ^= h >> 32;
  return h;
}

// ---------------------------------------------------------------------------
// Error keys.  The reference parses every block of a frame (tables included)
// before decoding any (frame.rs:198-230 then 232-260), and stops at the first
// error in each phase.  A key orders errors the same way; per frame we keep
// the minimum (atomicMin).  phase: 0 parse, 1 decode, 3 limit (GPU cannot
// reproduce the reference here: ZD_E_OUT_OF_DOMAIN / ZD_E_DST_TOO_SMALL).
// ---------------------------------------------------------------------------
constexpr uint64_t KEY_NONE = ~0ull;
enum : uint32_t { PH_PARSE = 0, PH_DECODE = 1, PH_LIMIT = 3 };
// parse stages, in reference order inside Block::parse
enum : uint32_t { PS_STRUCT = 0, PS_HUF_DESC = 1, PS_JUMP = 2, PS_SEQ_HDR = 3, PS_SEQ_TABLES = 4, PS_ALL = 5 };
// decode stages inside Block::decode (block.rs:80-87)
enum : uint32_t { DS_LITERALS = 1, DS_SEQUENCES = 2, DS_EXECUTE = 3 };
// PH_LIMIT stages the host can act on: a frame that decodes past the capacity
// its plan reserved (re-planned with more, zd_plan_decompress), K4J's
// pointer jumping not converging within its rounds (re-planned streaming)
enum : uint32_t { LS_CAPACITY = 7, LS_JROUNDS = 8 };
// sub of the DS_LITERALS out-of-domain key of a block whose streams decoded
// more literals than its slot holds (re-planned with room, zd_plan_decompress)
constexpr uint32_t DS_LIT_OVERFLOW_SUB = 4;
ZD_HD inline uint32_t key_stage(uint64_t k) { return (uint32_t)((k >> 28) & 15); }

ZD_HD inline uint64_t make_key(uint32_t phase, uint32_t block, uint32_t stage, uint32_t sub, int code) {
  return ((uint64_t)(phase & 3) << 62) | ((uint64_t)(block & 0x3FFFFFFFu) << 32) |
         ((uint64_t)(stage & 15) << 28) | ((uint64_t)(sub & 0xFFFFFu) << 8) | (uint64_t)((-code) & 0xFF);
}
ZD_HD inline int key_code(uint64_t k) { return k == KEY_NONE ? 0 : -(int)(k & 0xFF); }
ZD_HD inline uint32_t key_phase(uint64_t k) { return (uint32_t)(k >> 62); }
ZD_HD inline uint32_t key_block(uint64_t k) { return (uint32_t)((k >> 32) & 0x3FFFFFFFu); }

// Literal section types (literals.rs:38-43) and sequence modes (sequences.rs:256-261)
enum : uint8_t { LIT_RAW = 0, LIT_RLE = 1, LIT_COMPRESSED = 2, LIT_TREELESS = 3 };
enum : uint8_t { M_PREDEFINED = 0, M_RLE = 1, M_FSE = 2, M_REPEAT = 3 };

// One per compressed block.  Offsets marked "rel" are relative to `src`
// (first byte of the block content).
struct CompBlock {
  uint64_t src;            // absolute offset of the block content in d_src
  uint64_t lit_out;        // byte offset of this block's literals in the literal workspace
  uint64_t seq_out;        // sequence index of this block's first sequence in the sequence workspace
  uint64_t seq_side;       // direct records (zd_execute_sequences): device address of their DirectSide
                           // entries (values past the packed fields), 0 when none
  uint32_t size;           // Block_Size
  uint32_t frame;          // plan frame index
  uint32_t block_in_frame;
  uint32_t lit_regen;      // Regenerated_Size
  uint32_t lit_data;       // rel: raw literal bytes / Huffman tree description
  uint32_t huf_desc_size;  // bytes of the Huffman tree description (header byte included)
  uint32_t streams;        // rel: first Huffman stream (after the jump table)
  uint32_t stream_size[4]; // Huffman stream sizes after the reference's u16 truncation (literals.rs:115-122)
  uint32_t nseq;           // Number_of_Sequences as the reference computes it (D1 kept)
  uint32_t seq_tables;     // rel: first byte after nbSeq + mode byte
  uint32_t lut_slot;       // Huffman LUT slot this block builds (LIT_COMPRESSED)
  uint32_t fse_slot;       // FSE slot this block builds (nseq > 0)
  uint32_t lit_extra;      // literal slot bytes past Regenerated_Size + 16: a re-planned frame's blocks get
                           // room for all their streams decode (8 per stream byte), zd_plan_decompress
  int32_t huf_src;         // comp index whose LUT the literals use (-1: none)
  int32_t tab_src[3];      // comp index whose LL/OF/ML table the sequences use (-1: none)
  uint8_t lit_type;
  uint8_t nstreams;        // streams actually decoded (the reference stops at a 0-size stream)
  uint8_t lit_rle;         // RLE literal byte
  uint8_t modes[3];        // raw LL/OF/ML modes of the mode byte
  uint8_t host_stage;      // GPU parse runs only parse stages < host_stage
  uint8_t prebuilt;        // 1: tables already present in the slots (context API); skip
  uint8_t seq_direct;      // 1: the sequence records are direct {ll, ml, offset_value} (zd_common.h)
};

// Results per compressed block (device).
struct CompState {
  uint32_t lit_count;      // literals actually produced
  uint32_t bs_off;         // rel offset of the sequence bitstream
  uint32_t bs_size;
  uint32_t stop;           // nonzero: literals/sequences stage failed or is out of domain
  uint8_t al[3];           // accuracy log of the LL/OF/ML table in this block's FSE slot
  uint8_t huf_bits;        // maxBits of this block's LUT
  uint8_t k1_bigh;         // K1: the Huffman table needs the large scratch (second pass)
  uint8_t k1_bigs;         // K1: a sequence table needs it
  uint8_t pad[2];
};

// Blocks of frames in order (all types).
struct BlockRec {
  uint64_t src;            // absolute offset of the block content
  uint32_t size;           // Block_Size (raw/RLE: bytes produced)
  int32_t comp;            // compressed block index or -1
  uint8_t type;            // 0 raw, 1 RLE, 2 compressed, 4 = skippable payload (raw copy)
  uint8_t last;
  uint8_t rle;
  uint8_t pad[5];
};

struct FrameDesc {
  uint64_t out;            // byte offset of the frame's output in the output buffer
  uint64_t out_cap;        // bytes available from `out`
  uint64_t out_len0;       // bytes already produced before this launch (context API)
  uint32_t first_block;    // into BlockRec[]
  uint32_t nblocks;        // blocks to execute (0 for frames skipped by parse errors)
  uint32_t lds;            // 1: executed by K4F (whole frame in LDS), 2: by K4J (block-parallel), 3: copied whole
                           // by K0 (every block raw / RLE), 0: by the streaming K4
  uint32_t skip;           // leading raw/RLE blocks copied by K0 (the streaming K4 starts after them)
  uint64_t skip_bytes;     // their output bytes
};

// K0: one piece (<= COPY_PIECE bytes) of a raw / RLE block whose output offset
// is known at plan time (every block before it in the frame is raw or RLE).
constexpr uint32_t COPY_PIECE = 32u << 10;
struct CopyDesc {
  uint64_t src;            // absolute offset of the bytes in d_src (raw)
  uint64_t dst;            // absolute offset in the output base
  uint32_t size;
  uint32_t fill;           // 0x100 | byte for RLE, 0 for raw
};

struct FrameState {
  uint64_t key;            // min error key
  uint64_t out_len;        // decoded length (frame-relative, includes out_len0)
  uint64_t rep[3];         // repeat offsets in/out (decoding_context.rs:20)
};

// ---------------------------------------------------------------------------
// K4J: frames of many blocks executed block-parallel (zd_kernels.hip K4J).
// A frame's bytes are laid out as one u32 state word each in its region
// [base, base + cap) of the state array: J_FINAL | byte for a byte whose
// value is known, else the distance back to the byte it copies (a pointer
// the pointer-jumping rounds follow, in place; every version of a word is
// true of the byte, so the rounds need no ordering between lanes).
// Distances keep frames past 2 GiB in reach: only a match source 2 GiB or
// more behind its byte is out of the domain.
// ---------------------------------------------------------------------------
constexpr uint32_t J_FINAL = 1u << 31;
constexpr int J_MAX_ROUNDS = 40;
// sequences per K4J scatter segment (one wave each; c3s: 1024 -> 512 took the
// scatter from 0.33 to 0.29 ms, the segment sums 9 -> 15 us; 256 no better)
#ifndef ZD_J_SEG
#define ZD_J_SEG 512
#endif
constexpr uint32_t J_SEG = ZD_J_SEG;
static_assert(J_SEG % 64 == 0, "a scatter segment is whole 64-sequence batches");
struct JFrame {
  uint64_t base;           // word index of the frame's region in the state array
  uint64_t cap;            // words of the region (>= the frame's capacity)
  uint64_t piece0;         // first 16-byte piece of the frame in the rounds' piece numbering
  uint32_t frame;          // plan frame index
  uint32_t jb0, njb;       // its blocks: JBlkDesc / JBlk [jb0, jb0 + njb)
  uint32_t pad;
};
struct JBlkDesc {          // static, from the host
  uint32_t block;          // BlockRec index
  uint32_t jframe;         // JFrame index
  uint32_t j;              // block index inside the frame
  uint32_t seg0;           // its scatter segments: JSeg [seg0, seg0 + max(1, ceil(nseq / J_SEG)))
};
struct JBlk {              // device: K4J pass results per block
  uint64_t out_start;      // frame position of the block's first output byte
  uint64_t size;           // output bytes (literals + match lengths)
  uint64_t rep_in[3];      // repeat offsets before the block (concrete)
  uint64_t map[3];         // the block's repeat-offset map (jr codes)
  uint32_t dead;           // 1: not executed (a failure before it, or past the capacity)
  uint32_t pad;
};
struct JSeg {              // device: where segment k of a block starts (KJ1 -> KJ3)
  uint64_t out_rel;        // output bytes of the block's sequences before the segment
  uint64_t map[3];         // repeat offsets there, as jr codes of the block's incoming ones
  uint32_t lit_rel;        // literals consumed before it
  uint32_t pad;
};
struct JSegDesc {          // static: the scatter's work list
  uint32_t jblk;           // JBlk index
  uint32_t k;              // segment of the block
};

// Workspace carve-up, all offsets in bytes from the workspace base.
struct Workspace {
  uint64_t comp, comp_state, blocks, frames, frame_state, frame_state0;
  uint64_t list_tables, list_huf, list_seq, list_k4f;   // u32 work lists
  uint64_t copies;                                      // CopyDesc[] for K0
  uint64_t lits, seqs, luts, fses;
  uint64_t jframes, jblkd, jblk, jseg, jsegd, jpend;    // K4J descriptors / state / round counters
  uint64_t jdone;                                       // K4J: one byte per piece, 1 once emitted
  uint64_t huge;                                        // K1: u32 count + the blocks whose trees have > 256 symbols
  uint64_t deep;                                        // K1's pool for deep trees of > 7,680 leaves: u32 used, then bytes
  uint64_t jst;                                         // K4J per-byte state words
  uint64_t redo, k2done;                                // zd_k_fused: frames for the redo pass, K2's finished workgroups
  uint64_t hframes;                                     // device-built plans: the walk's frame index (zd_walk.h HostFrame)
  uint64_t total;
};

}  // namespace zd
