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

// FSE decode entry: symbol | nbits << 8 | baseline << 16
ZD_HD inline uint32_t fse_entry(uint32_t sym, uint32_t nb, uint32_t base) { return sym | (nb << 8) | (base << 16); }

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
  int32_t huf_src;         // comp index whose LUT the literals use (-1: none)
  int32_t tab_src[3];      // comp index whose LL/OF/ML table the sequences use (-1: none)
  uint8_t lit_type;
  uint8_t nstreams;        // streams actually decoded (the reference stops at a 0-size stream)
  uint8_t lit_rle;         // RLE literal byte
  uint8_t modes[3];        // raw LL/OF/ML modes of the mode byte
  uint8_t host_stage;      // GPU parse runs only parse stages < host_stage
  uint8_t prebuilt;        // 1: tables already present in the slots (context API); skip
};

// Results per compressed block (device).
struct CompState {
  uint32_t lit_count;      // literals actually produced
  uint32_t bs_off;         // rel offset of the sequence bitstream
  uint32_t bs_size;
  uint32_t stop;           // nonzero: literals/sequences stage failed or is out of domain
  uint8_t al[3];           // accuracy log of the LL/OF/ML table in this block's FSE slot
  uint8_t huf_bits;        // maxBits of this block's LUT
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
};

struct FrameState {
  uint64_t key;            // min error key
  uint64_t out_len;        // decoded length (frame-relative, includes out_len0)
  uint64_t rep[3];         // repeat offsets in/out (decoding_context.rs:20)
};

// Workspace carve-up, all offsets in bytes from the workspace base.
struct Workspace {
  uint64_t comp, comp_state, blocks, frames, frame_state;
  uint64_t list_tables, list_huf, list_seq;   // u32 work lists
  uint64_t lits, seq_ll, seq_of, seq_ml, luts, fses;
  uint64_t total;
};

}  // namespace zd
