// zd_kernels.hip — gfx950 kernels of the ZSTD block-decode path.
//
//   K0 zd_k_rawcopy    raw / RLE blocks that lead a frame (block.rs:76-79)
//   K1 zd_k_tables     one compressed block per lane: Huffman tree description
//                      -> LUT, FSE table descriptions -> decode tables
//                      (huffman.rs:80-203, fse.rs:16-202, sequences.rs:91-187);
//                      zd_k_tables_seqw: the sequence tables one wave per block;
//                      zd_k_huf_pairs: each LUT of <= 11 bits -> K2's pair table
//   K2 zd_k_huffman    one stream per lane, 8 blocks per wave, pair tables in
//                      LDS (literals.rs:49-86 + huffman.rs:205-218)
//   K3 zd_k_sequences_q  the FSE state chain, four lanes per block, 16 blocks
//                      per wave, tables in LDS (sequences.rs:191-237)
//   K4 zd_k_execute    one wave per frame, 64 sequences per batch, a linear LDS
//                      window of recent output, aligned 16-B flushes to HBM
//                      (decoding_context.rs:50-106 + block.rs:74-99, with the
//                      value decode of decoders/sequence.rs:41-55); K4F / K4J /
//                      zd_k_fused: the executors for other plan shapes
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "../../include/zd.h"
#include "zd_common.h"
#include "zd_launch.h"
#include "zd_walk.h"

namespace zd {

const char* const kKernelNames[N_KERNELS] = {"zd_k_rawcopy", "zd_k_tables", "zd_k_huffman", "zd_k_sequences",
                                             "zd_k_execute", "zd_k_jexec"};
const char* const kDomNames[N_DOM] = {"zd_k_rawcopy", "zd_k_fused", "zd_k_execute", "zd_k_execute_lds",
                                      "zd_k_jsum+zd_k_jsum_blocks+zd_k_jprefix+zd_k_jscatter+zd_k_jround"};

// ---------------------------------------------------------------------------
// constants (decoders/sequence.rs:95-191, sequences.rs:29-39)
// ---------------------------------------------------------------------------
__constant__ uint32_t c_ml_base[53] = {
    3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29,
    30, 31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t c_ml_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                      0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t c_ll_base[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,   10,   11,   12,   13,   14,   15,   16,    18,
                                       20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t c_ll_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                      1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ int16_t c_ll_default[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                         2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t c_of_default[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
__constant__ int16_t c_ml_default[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                         1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
__device__ inline void key_min(FrameState* fs, uint32_t frame, uint64_t key) {
  atomicMin((unsigned long long*)&fs[frame].key, (unsigned long long)key);
}

__device__ inline int highbit32(uint32_t v) { return 31 - __clz(v); }

// 8 bytes at p; bytes outside [lo, hi) read as 0.
__device__ inline uint64_t load_u64(const uint8_t* p, const uint8_t* lo, const uint8_t* hi) {
  if (p >= lo && p + 8 <= hi) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
  }
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = p + i;
    if (q >= lo && q < hi) v |= (uint64_t)*q << (8 * i);
  }
  return v;
}

// ---------------------------------------------------------------------------
// BackwardBitParser (parsing.rs:191-259) as a cached reader.  Bits are numbered
// from the start of the stream (little-endian integer); the unread bits are
// [0, bitpos), read from the top.  `bitpos` equals the reference's `readable`.
// ---------------------------------------------------------------------------
struct BwBits {
  const uint8_t* base;
  const uint8_t* lo;
  const uint8_t* hi;
  int64_t bitpos;
  int64_t cache_lo;
  uint64_t cache;

  __device__ inline void refill() {
    int64_t byte_hi = (bitpos - 1) >> 3;
    int64_t byte_lo = byte_hi - 7;
    if (byte_lo < 0) byte_lo = 0;
    cache = load_u64(base + byte_lo, lo, hi);
    cache_lo = byte_lo * 8;
  }
  // parsing.rs:200-220: EmptyInputData, NullByte, skip padding + marker
  __device__ inline int init(const uint8_t* b, uint32_t n, const uint8_t* l, const uint8_t* h) {
    base = b; lo = l; hi = h;
    if (n == 0) return ZD_E_EMPTY_INPUT_DATA;
    uint8_t last = b[n - 1];
    if (last == 0) return ZD_E_NULL_BYTE;
    bitpos = 8ll * (n - 1) + highbit32(last);
    refill();
    return 0;
  }
  // k <= 32; zero-fills below bit 0
  __device__ inline uint32_t peek(int k) {
    if (bitpos - k < cache_lo && cache_lo > 0) refill();
    if (bitpos >= k) return (uint32_t)((cache >> (bitpos - k - cache_lo)) & ((1ull << k) - 1));
    return (uint32_t)((cache & ((1ull << bitpos) - 1)) << (k - bitpos));
  }
  // parsing.rs:228-254 (k <= 32)
  __device__ inline int take(int k, uint32_t* v) {
    if (k > bitpos) return ZD_E_NOT_ENOUGH_BITS;
    if (k == 0) { *v = 0; return 0; }
    *v = peek(k);
    bitpos -= k;
    return 0;
  }
};

// ForwardBitParser (parsing.rs:114-189), LSB-first (headers and table
// descriptions).  A 64-bit cache of the bytes from the last refill: one 8-byte
// load per ~40 bits read instead of two or three dependent byte loads per
// peek (K1's NCount parse, C3: the sequence-table half 298 us).
struct FwBits {
  const uint8_t* d;
  uint32_t nbytes;
  uint32_t pos;
  uint64_t cache = 0;
  int64_t cbit = -1;                               // bit of d that is cache bit 0 (-1: empty)
  __device__ inline uint32_t bits(uint32_t at, int len) {   // len <= 24, within range
    if (cbit < 0 || (int64_t)at < cbit || (int64_t)at + len > cbit + 64) {
      cache = load_u64(d + (at >> 3), d, d + nbytes);
      cbit = (int64_t)(at >> 3) * 8;
    }
    const uint32_t v = (uint32_t)(cache >> ((int64_t)at - cbit));
    return len >= 32 ? v : (v & ((1u << len) - 1));
  }
  __device__ inline int peek(int len, uint32_t* v) {
    if ((int64_t)nbytes * 8 - pos < len) return ZD_E_NOT_ENOUGH_BITS;
    *v = len ? bits(pos, len) : 0;
    return 0;
  }
  __device__ inline int take(int len, uint32_t* v) {
    if (int r = peek(len, v)) return r;
    pos += len;
    return 0;
  }
  __device__ inline void skip(int len) { pos += len; }
  __device__ inline uint32_t bytes_read() const { return pos / 8 + (pos % 8 > 0); }
};

// A table needs K1's large scratch (more than K1S_SYMS symbols, or a
// Huffman-weight table deeper than AL 6): the block goes to the second pass.
constexpr int K1_BIG = 1;
// A Huffman-weight stream past 255 weights (only in non-conforming input):
// the reference keeps every weight, its symbols wrapping as u8
// (huffman.rs:161-175); the block goes to the third pass (zd_k_tables_huge).
constexpr int K1_HUGE = 2;
constexpr uint32_t K1S_SYMS = 64;

// ForwardBitParser over a wave's registers (zd_k_fused's K4 waves): dword i
// from a 4-aligned base on lane i % 64 of r[i / 64]; FwBits' 64-bit cache
// refilled by two readlanes instead of a dependent memory load (past the
// 512 bytes held: memory).  The wave runs it on uniform values.
struct FwBitsW {
  const uint8_t* d;
  uint32_t nbytes;
  uint32_t pos;
  uint32_t r0, r1;
  uint32_t delta;                                  // bit of the register base where d starts
  uint64_t cache = 0;
  // (32-bit bookkeeping: a description lies within its block, < 2^24 bits
  // past the register base; 64-bit compares cost the serial walk SALU ops)
  int32_t cbit = -1;                               // register-base bit of cache bit 0 (-1: empty)
  __device__ inline uint32_t bits(uint32_t at, int len) {   // len <= 24, within range
    const int32_t a = (int32_t)(at + delta);
    if (cbit < 0 || a < cbit || a + len > cbit + 64) {
      const uint32_t w = a >> 5;
      if (w + 1 < 128) {
        const uint32_t lo = (uint32_t)(w < 64 ? __builtin_amdgcn_readlane((int)r0, (int)w)
                                              : __builtin_amdgcn_readlane((int)r1, (int)(w - 64)));
        const uint32_t hi = (uint32_t)(w + 1 < 64 ? __builtin_amdgcn_readlane((int)r0, (int)(w + 1))
                                                  : __builtin_amdgcn_readlane((int)r1, (int)(w - 63)));
        cache = ((uint64_t)hi << 32) | lo;
        cbit = (int64_t)w * 32;
      } else {
        cache = load_u64(d + (at >> 3), d, d + nbytes);
        cbit = (int32_t)delta + (int32_t)(at >> 3) * 8;
      }
    }
    return (uint32_t)(cache >> (a - cbit)) & ((1u << len) - 1);
  }
  __device__ inline int peek(int len, uint32_t* v) {
    if ((int32_t)(nbytes * 8) - (int32_t)pos < len) return ZD_E_NOT_ENOUGH_BITS;
    *v = len ? bits(pos, len) : 0;
    return 0;
  }
  __device__ inline int take(int len, uint32_t* v) {
    if (int r = peek(len, v)) return r;
    pos += len;
    return 0;
  }
  __device__ inline void skip(int len) { pos += len; }
  __device__ inline uint32_t bytes_read() const { return pos / 8 + (pos % 8 > 0); }
};

// parse_fse_table (fse.rs:16-69); dist holds max_sym entries (256: all)
template <typename BR>
__device__ int parse_ncount(BR& in, uint8_t* al_out, int16_t* dist, uint32_t* nsym_out, uint32_t max_sym) {
  uint32_t v;
  if (int r = in.take(4, &v)) return r;
  int al = (int)v + 5;
  if (al > FSE_MAX_AL) return ZD_E_LARGE_ACCURACY_LOG;
  int32_t remaining = 1 << al;
  uint32_t n_sym = 0;
  while (remaining > 0 && n_sym < 256) {
    int bits = highbit32((uint32_t)remaining + 1) + 1;
    uint32_t pk;
    if (int r = in.peek(bits, &pk)) return r;
    const uint32_t lower_mask = (1u << (bits - 1)) - 1;
    const uint32_t threshold = (1u << bits) - 1 - ((uint32_t)remaining + 1);
    // the reference's take(bits - 1) reads pk's low bits, take(bits) pk: one
    // read (the peek's bound covers both)
    const uint32_t low = pk & lower_mask;
    const bool short_code = low < threshold;
    const int32_t decoded = short_code ? (int32_t)low
                                       : (pk > lower_mask ? (int32_t)pk - (int32_t)threshold : (int32_t)pk);
    in.skip(short_code ? bits - 1 : bits);
    int32_t proba = decoded - 1;
    remaining -= proba < 0 ? -proba : proba;
    if (n_sym < max_sym) dist[n_sym] = (int16_t)proba;
    else if (max_sym < 256) return K1_BIG;
    n_sym++;
    if (proba == 0) {
      for (;;) {
        if (int r = in.take(2, &v)) return r;
        for (uint32_t z = 0; z < v; z++) {
          if (n_sym < max_sym) dist[n_sym] = 0;
          else if (max_sym < 256) return K1_BIG;
          n_sym++;
        }
        if (v != 3) break;
      }
    }
  }
  if (remaining != 0 || n_sym >= 256) return ZD_E_CORRUPTED_TABLE;
  *al_out = (uint8_t)al;
  *nsym_out = n_sym;
  return 0;
}

// FseTable::from_distribution (fse.rs:110-202), serial.  State u of symbol s
// (in position order) gets nextState = count(s) + u, stored with the symbol as
// a 16-bit entry (zd_common.h fse_entry); nbits/baseline follow from it and
// equal the reference's parts/base_width construction (fse.rs:169-189).
// `-1` symbols count as 1.  sym/next are LDS scratch (T and 256 entries).
#ifdef ZD_FZ_TRACE
// zd_k_fused timeline (scripts/fztrace.py): per frame s_memrealtime at the
// kernel's start, tables ready, chain end, K4's waits over, K4 end; K2's end
__device__ uint64_t fz_tr[1024][16];
__device__ uint64_t fz_k2end;
#define FZT(f, i) do { if ((f) < 1024) fz_tr[f][i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define FZT_ON 1
#else
#define FZT(f, i) do { } while (0)
#endif
#ifdef ZD_K1_PROF
__device__ uint64_t k1_prof[8];
#define K1T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define K1ADD(i, a, b) atomicAdd((unsigned long long*)&k1_prof[i], (unsigned long long)((b) - (a)))
#else
#define K1T(v) do { } while (0)
#define K1ADD(i, a, b) do { } while (0)
#endif
__device__ int build_fse(int al, const int16_t* dist, uint32_t nsym, uint16_t* __restrict__ table, uint8_t* sym,
                         uint16_t* next) {
  if (al > FSE_MAX_AL) return ZD_E_LARGE_ACCURACY_LOG;
  K1T(t0);
  uint32_t T = 1u << al;
  uint32_t zero_pos = T;
  for (uint32_t s = 0; s < nsym; s++) {
    if (dist[s] == -1) {
      if (zero_pos == 0) return ZD_E_REF_PANIC;
      sym[--zero_pos] = (uint8_t)s;
    }
  }
  uint32_t pos = 0, step = (T >> 1) + (T >> 3) + 3, mask = T - 1, placed = 0;
  for (uint32_t s = 0; s < nsym; s++) {
    // the count in a register: sym (bytes) may alias dist for the compiler,
    // which would reload it from LDS on every placement
    const int c = dist[s];
    if (c > 0 && zero_pos == 0) return ZD_E_REF_PANIC;   // the reference loops forever
    for (int k = 0; k < c; k++) {
      sym[pos] = (uint8_t)s;
      pos = (pos + step) & mask;
      while (pos >= zero_pos) pos = (pos + step) & mask;
    }
    placed += c > 0 ? (uint32_t)c : 0u;
  }
  if (placed != zero_pos) return ZD_E_CORRUPTED_TABLE;
  K1T(t1);
  K1ADD(0, t0, t1);
  for (uint32_t s = 0; s < nsym; s++) next[s] = dist[s] > 0 ? (uint16_t)dist[s] : (dist[s] == -1 ? 1 : 0);
  // next[s]++ in state order, four states a step (T >= 32): one LDS round
  // trip for the four counters instead of one per state; a symbol met again
  // inside the step continues from its earlier value there, and the
  // write-backs in state order leave each counter at its last value + 1
  for (uint32_t i = 0; i < T; i += 4) {
    const uint32_t w = *(const uint32_t*)(sym + i);
    const uint32_t s0 = w & 255, s1 = (w >> 8) & 255, s2 = (w >> 16) & 255, s3 = w >> 24;
    const uint32_t n0 = next[s0], n1 = next[s1], n2 = next[s2], n3 = next[s3];
    const uint32_t t0 = n0;
    const uint32_t t1 = s1 == s0 ? t0 + 1 : n1;
    const uint32_t t2 = s2 == s1 ? t1 + 1 : (s2 == s0 ? t0 + 1 : n2);
    const uint32_t t3 = s3 == s2 ? t2 + 1 : (s3 == s1 ? t1 + 1 : (s3 == s0 ? t0 + 1 : n3));
    next[s0] = (uint16_t)(t0 + 1);
    next[s1] = (uint16_t)(t1 + 1);
    next[s2] = (uint16_t)(t2 + 1);
    next[s3] = (uint16_t)(t3 + 1);
    table[i] = fse_entry(s0, t0);
    table[i + 1] = fse_entry(s1, t1);
    table[i + 2] = fse_entry(s2, t2);
    table[i + 3] = fse_entry(s3, t3);
  }
  K1T(t2);
  K1ADD(1, t1, t2);
  return 0;
}

// ---------------------------------------------------------------------------
// K1: tables, one compressed block per LANE (huffman.rs:80-203, fse.rs:16-202,
// sequences.rs:91-187).  Every table build is serial code; running blocks on
// lanes (instead of one block per wave with one lane busy) makes the whole
// chip build tables at once.  Each lane keeps its scratch in LDS and writes
// its Huffman LUT and compact FSE tables straight to the block's HBM slots.
// ---------------------------------------------------------------------------
#ifndef ZD_K1_LANES
#define ZD_K1_LANES 16
#endif
constexpr int K1_LANES = ZD_K1_LANES;
constexpr int K1_MAX_WEIGHTS = 255;               // a Huffman tree of 256 symbols (RFC 8878 4.2.1)
struct K1Lane {
  static constexpr uint32_t SYMS = 256, WFSE = FSE_TAB;
  uint16_t fse[FSE_TAB];                          // Huffman-weight FSE table
  uint8_t sym[FSE_TAB];                           // spread scratch
  uint16_t next[256];
  int16_t dist[256];
  uint8_t weights[K1_MAX_WEIGHTS + 1];
  uint16_t cnt[16], start[16], placed[16];        // per code width (<= 12)
};
// The first pass's scratch (1.2 KiB instead of 2.9: eight workgroups per CU
// instead of three, so table builds hide each other's LDS latency): up to 64
// symbols per table and Huffman-weight tables of AL <= 6 (zstd's limit).
struct K1LaneS {
  static constexpr uint32_t SYMS = K1S_SYMS, WFSE = 64;
  uint16_t fse[64];
  uint8_t sym[FSE_TAB];
  uint16_t next[K1S_SYMS];
  int16_t dist[K1S_SYMS];
  uint8_t weights[K1_MAX_WEIGHTS + 1];
  uint16_t cnt[16], start[16], placed[16];
};

// A LUT entry's bits 8-14: the code width (or an absent node's depth) f.
// Trees K2 decodes from LDS (p <= K2 LUT bits, 11) store (32 - f) & 31
// instead: K2's fast loop shifts its 64-bit bit window as two 32-bit halves,
// hi = alignbit(hi, lo, 32 - f), one 32-bit op on the symbol chain.
constexpr int K2_LUT_BITS = 11;
__device__ inline uint32_t lut_field(uint32_t f, int p) { return p <= K2_LUT_BITS ? (32 - f) & 31 : f; }
__device__ inline uint32_t lut_width(uint32_t e, bool s32) {
  const uint32_t f = (e >> 8) & 0x7F;
  return s32 ? (32 - f) & 31 : f;
}

// Entries [a, b) that no code reaches: the tree node there is Absent.  Its
// depth is that of the largest aligned block around the entry inside [a, b)
// (the entries just outside hold codes or lie past the table), which is the
// number of bits HuffmanDecoder::decode (huffman.rs:205-218) reads before
// it hits the node and panics.
__device__ void lut_holes(uint16_t* __restrict__ lut, int p, uint32_t a, uint32_t b) {
  for (uint32_t e = a; e < b; e++) {
    int k = p;
    for (; k > 0; k--) {
      const uint32_t lo = e & ~((1u << k) - 1);
      if (lo >= a && lo + (1u << k) <= b) break;
    }
    lut[e] = (uint16_t)(LUT_ABSENT | (lut_field((uint32_t)(p - k), p) << 8));
  }
}

// Trees deeper than the LUT (maxBits p in 13..31, non-conforming input:
// zstd encoders stop at 11) keep their codes as intervals of the p-bit code
// space instead, in the LUT slot: dword 0 the group count G, then per code
// width (longest first) {first code, end, width, offset of its symbols}, the
// symbol bytes from byte DEEP_SYMS_AT.  The same insertion as the LUT fill
// (from_number_of_bits + insert, huffman.rs:132-175): longest codes first,
// each width's symbols ascending from the next aligned slot, a code that no
// longer fits is dropped.  count(w) = symbols of width w, emit(w, k, dst)
// writes the first k of them.  K2 decodes these blocks with huf_stream_deep.
constexpr uint32_t DEEP_SYMS_AT = 512;
constexpr uint32_t DEEP_SYM_CAP = LUT_ENTRIES * 2 - DEEP_SYMS_AT;
constexpr uint32_t DEEP_IN_POOL = 1u << 31;      // tab[0]: the symbols are in the pool, at tab[DEEP_POOL_AT]
constexpr uint32_t DEEP_POOL_AT = DEEP_SYMS_AT / 4 - 1;   // (past 31 groups of 4 words)
// A tree with more placed leaves than the slot's DEEP_SYM_CAP bytes keeps its
// symbols in the plan's deep pool (pool_used: the pool's u32 fill counter,
// the bytes follow it 16 bytes on); past the pool it is out of the domain.
template <typename COUNT, typename EMIT>
__device__ int deep_build(uint32_t* tab, int p, COUNT count, EMIT emit, uint32_t* pool_used = nullptr) {
  const uint64_t T = 1ull << p;
  uint64_t pos = 0;
  uint32_t G = 0, off = 0, flag = 0;
  uint8_t* syms = (uint8_t*)tab + DEEP_SYMS_AT;
  {
    uint64_t q = 0, total = 0;                    // the leaves the insertion places
    for (int w = p; w >= 1; w--) {
      const uint32_t c = count(w);
      if (!c) continue;
      const uint64_t S = 1ull << (p - w);
      const uint64_t al = (q + S - 1) & ~(S - 1);
      const uint64_t fit = (T - al) / S;
      const uint64_t k = c < fit ? c : fit;
      q = al + k * S;
      total += k;
    }
    if (total > DEEP_SYM_CAP) {
      if (!pool_used) return ZD_E_OUT_OF_DOMAIN;
      const uint32_t at = atomicAdd(pool_used, (uint32_t)total);
      if ((uint64_t)at + total > DEEP_POOL_BYTES) return ZD_E_OUT_OF_DOMAIN;
      syms = (uint8_t*)pool_used + 16 + at;
      tab[DEEP_POOL_AT] = at;
      flag = DEEP_IN_POOL;
    }
  }
  for (int w = p; w >= 1; w--) {
    const uint32_t c = count(w);
    if (!c) continue;
    const uint64_t S = 1ull << (p - w);
    const uint64_t al = (pos + S - 1) & ~(S - 1);
    const uint64_t fit = (T - al) / S;
    const uint32_t k = (uint32_t)(c < fit ? c : fit);
    pos = al + k * S;
    if (!k) continue;
    tab[1 + 4 * G] = (uint32_t)al;
    tab[2 + 4 * G] = (uint32_t)pos;
    tab[3 + 4 * G] = (uint32_t)w;
    tab[4 + 4 * G] = off;
    emit(w, k, syms + off);
    off += k;
    G++;
  }
  tab[0] = G | flag;
  return 0;
}

// parse_fse (huffman.rs:108-130): the weights of an FSE-compressed tree
// description, two alternating FSE states sharing one table, each weight
// handed to put(i, w) (put returns false: K1_HUGE, the weights do not fit the
// pass's scratch).  The reference loops forever when every state left reads
// 0 bits (huffman.rs:121-124); the oracle (zd_oracle.c h_parse_fse) calls
// that a panic after guard_max weights, and so does this.
template <typename LN, typename PUT>
__device__ int k1_weight_stream(const uint8_t* desc, const uint8_t* src, const uint8_t* src_end, LN& L, PUT put,
                                uint32_t* nw_out) {
  const uint8_t h = desc[0];
  FwBits fw{desc + 1, h, 0};
  uint8_t al;
  uint32_t nsym;
  int st = parse_ncount(fw, &al, L.dist, &nsym, LN::SYMS);
  if (!st && (1u << al) > LN::WFSE) st = K1_BIG;
  if (!st) st = build_fse(al, L.dist, nsym, L.fse, L.sym, L.next);
  BwBits bs;
  if (!st) st = bs.init(desc + 1 + fw.bytes_read(), h - fw.bytes_read(), src, src_end);
  uint32_t nw = 0;
  if (!st) {
    const uint64_t guard_max = (8 * (uint64_t)h + 2) * ((1u << al) + 2) * 2;
    uint32_t sa = 0, sb = 0, v;
    st = bs.take(al, &sa);
    if (!st) st = bs.take(al, &sb);
    bool last_updated_is_first = false, last_read_is_first = false;
    bool has_a = true, has_b = true;
    while (!st) {
      const uint32_t cur = last_updated_is_first ? sb : sa;
      const uint32_t nb = fse_nb(L.fse[cur], al);
      if ((int64_t)nb > bs.bitpos) break;
      if (nw >= guard_max) { st = ZD_E_REF_PANIC; break; }
      uint32_t w;
      if (last_read_is_first) { last_read_is_first = false; if (!has_b) { st = ZD_E_REF_PANIC; break; } w = fse_sym(L.fse[sb]); has_b = false; }
      else { last_read_is_first = true; if (!has_a) { st = ZD_E_REF_PANIC; break; } w = fse_sym(L.fse[sa]); has_a = false; }
      if (!put(nw, w)) { st = K1_HUGE; break; }
      nw++;
      uint32_t& sx = last_updated_is_first ? sb : sa;
      bool& has = last_updated_is_first ? has_b : has_a;
      if (has) { st = ZD_E_REF_PANIC; break; }
      st = bs.take((int)nb, &v);
      if (st) break;
      sx = fse_base(L.fse[sx], al) + v;
      has = true;
      last_updated_is_first = !last_updated_is_first;
    }
    for (int k = 0; k < 2 && !st; k++) {
      uint32_t w;
      if (last_read_is_first) { last_read_is_first = false; if (!has_b) { st = ZD_E_REF_PANIC; break; } w = fse_sym(L.fse[sb]); has_b = false; }
      else { last_read_is_first = true; if (!has_a) { st = ZD_E_REF_PANIC; break; } w = fse_sym(L.fse[sa]); has_a = false; }
      if (!put(nw, w)) { st = K1_HUGE; break; }
      nw++;
    }
  }
  *nw_out = nw;
  return st;
}

// HuffmanDecoder::parse + from_weights + from_number_of_bits (huffman.rs:
// 80-203) -> LUT of 2^p u16 entries {symbol | width << 8}; entries no code
// reaches get LUT_ABSENT | depth of the absent tree node.  Returns status;
// *p_out = maxBits.  A weight stream longer than the scratch (255 weights,
// a tree of 256 symbols) returns K1_HUGE: the third pass takes the block.
template <typename LN>
__device__ int k1_huffman_lane(const uint8_t* desc, const uint8_t* src, const uint8_t* src_end, LN& L,
                               uint16_t* __restrict__ lut, int* p_out) {
  int st = 0;
  uint32_t nw = 0;
  const uint8_t h = desc[0];
  K1T(h0);
  if (h < 128) {
    st = k1_weight_stream(desc, src, src_end, L, [&](uint32_t i, uint32_t w) {
      if (i >= K1_MAX_WEIGHTS) return false;
      L.weights[i] = (uint8_t)w;
      return true;
    }, &nw);
  } else {
    // parse_direct (huffman.rs:92-106): high nibble first
    nw = (uint32_t)h - 127;
    for (uint32_t i = 0; i < nw; i++) {
      const uint8_t b = desc[1 + i / 2];
      L.weights[i] = (i & 1) ? (b & 15) : (b >> 4);
    }
  }
  if (st) return st;
  K1T(h1);
  K1ADD(3, h0, h1);
  // from_weights (huffman.rs:177-203)
  uint32_t sum = 0;
  for (uint32_t i = 0; i < nw; i++) {
    const uint32_t w = L.weights[i];
    if (!w) continue;
    if (w - 1 >= 32) return ZD_E_REF_PANIC;
    const uint32_t add = 1u << (w - 1);
    if (sum > 0xFFFFFFFFu - add) return ZD_E_REF_PANIC;
    sum += add;
  }
  if (sum == 0) return ZD_E_REF_PANIC;
  int p = highbit32(sum);
  if ((1ull << p) < sum) p++;
  if (p >= 32) return ZD_E_REF_PANIC;
  const uint8_t rest = (uint8_t)((1u << p) - sum);
  if (rest == 0) return ZD_E_REF_PANIC;           // D3
  const uint32_t manquant = (uint32_t)highbit32(rest) + 1;
  for (uint32_t i = 0; i < nw; i++)
    if (L.weights[i] > (uint32_t)p + 1) return ZD_E_REF_PANIC;
  if (manquant > (uint32_t)p + 1) return ZD_E_REF_PANIC;
  L.weights[nw] = (uint8_t)manquant;          // the implied last symbol: width p + 1 - manquant
  const uint32_t n = nw + 1;
  if (p > LUT_MAX_BITS) {
    *p_out = p;
    return deep_build((uint32_t*)lut, p,
                      [&](int w) {
                        uint32_t c = 0;
                        for (uint32_t i = 0; i < n; i++) c += L.weights[i] && (int)(p + 1 - L.weights[i]) == w;
                        return c;
                      },
                      [&](int w, uint32_t k, uint8_t* dst) {
                        uint32_t r = 0;
                        for (uint32_t i = 0; i < n && r < k; i++)
                          if (L.weights[i] && (int)(p + 1 - L.weights[i]) == w) dst[r++] = (uint8_t)i;
                      });
  }
  // width(i) = weight ? p + 1 - weight : 0 (never inserted, huffman.rs:163-165)
  // from_number_of_bits + insert (huffman.rs:132-175): longest codes first,
  // ascending symbol, each at the leftmost free aligned slot; a code that no
  // longer fits is not inserted.  Counting sort by width.
  for (int w = 0; w <= p; w++) { L.cnt[w] = 0; L.placed[w] = 0; }
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t wt = L.weights[i];
    if (wt) L.cnt[p + 1 - wt]++;
  }
  const uint32_t T = 1u << p;
  uint32_t pos = 0;
  for (int w = p; w >= 1; w--) {
    if (!L.cnt[w]) continue;
    const uint32_t S = 1u << (p - w);
    const uint32_t al = (pos + S - 1) & ~(S - 1);
    lut_holes(lut, p, pos, al);               // alignment gap: absent tree nodes
    const uint32_t fit = (T - al) / S;
    const uint32_t k = L.cnt[w] < fit ? L.cnt[w] : fit;
    L.start[w] = (uint16_t)al;
    L.placed[w] = (uint16_t)k;                // the first k symbols of this width get slots
    pos = al + k * S;
  }
  lut_holes(lut, p, pos, T);
  K1T(h2);
  K1ADD(4, h1, h2);
  for (int w = 0; w <= p; w++) L.cnt[w] = 0;  // reused as rank counters
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t wt = L.weights[i];
    if (!wt) continue;
    const int w = p + 1 - (int)wt;
    const uint32_t r = L.cnt[w]++;
    if (r >= L.placed[w]) continue;
    const uint32_t S = 1u << (p - w);
    const uint32_t at = L.start[w] + r * S;
    const uint16_t ent = (uint16_t)((i & 0xFF) | (lut_field((uint32_t)w, p) << 8));
    if (S >= 4) {
      const uint64_t e4 = (uint64_t)ent * 0x0001000100010001ull;
      for (uint32_t e = 0; e < S; e += 4) *(uint64_t*)(lut + at + e) = e4;
    } else {
      for (uint32_t e = 0; e < S; e++) lut[at + e] = ent;
    }
  }
  K1T(h3);
  K1ADD(5, h2, h3);
  *p_out = p;
  return 0;
}
// Sequence tables (sequences.rs:91-187) of one block: RLE bytes, FSE
// descriptions and predefined distributions, in LL, OF, ML order, each
// written as compact entries to the block's slot.  Returns status; *stage_sub
// = table index of a failure (3: the empty-bitstream check).
template <typename LN>
__device__ int k1_sequences_lane(const uint8_t* blk, const CompBlock& C, LN& L, uint16_t* slot, uint8_t al_out[3],
                                 uint32_t* bs_off, uint32_t* bs_size, int* sub) {
  uint32_t pos = C.seq_tables;
  for (int k = 0; k < 3; k++) {
    *sub = k;
    const int mode = C.modes[k];
    uint16_t* tab = slot + k * FSE_TAB;
    int st = 0, al = 0;
    if (mode == M_RLE) {
      if (pos >= C.size) st = ZD_E_NOT_ENOUGH_BYTES;
      else { tab[0] = fse_entry(blk[pos], 1); pos++; }   // AL 0: nb 0, baseline 0
    } else if (mode == M_FSE) {
      if (pos >= C.size) st = ZD_E_EMPTY_SLICE;
      else {
        FwBits fw{blk + pos, C.size - pos, 0};
        uint8_t a;
        uint32_t nsym;
        K1T(p0);
        st = parse_ncount(fw, &a, L.dist, &nsym, LN::SYMS);
        K1T(p1);
        K1ADD(2, p0, p1);
        if (!st) st = build_fse(a, L.dist, nsym, tab, L.sym, L.next);
        al = a;
        pos += fw.bytes_read();
      }
    } else if (mode == M_PREDEFINED) {
      const int16_t* d = k == 0 ? c_ll_default : (k == 1 ? c_of_default : c_ml_default);
      const uint32_t nsym = k == 0 ? 36 : (k == 1 ? 29 : 53);
      al = k == 1 ? 5 : 6;
      for (uint32_t x = 0; x < nsym; x++) L.dist[x] = d[x];
      st = build_fse(al, L.dist, nsym, tab, L.sym, L.next);
    }
    if (st) return st;
    if (mode != M_REPEAT) al_out[k] = (uint8_t)al;
  }
  *sub = 3;
  *bs_off = pos;                                  // seq.bitstream = input.slice(input.len()) (sequences.rs:72)
  *bs_size = pos < C.size ? C.size - pos : 0;
  return pos >= C.size ? ZD_E_EMPTY_SLICE : 0;
}

// Two passes: every block with the small scratch (K1LaneS), then the blocks
// that flagged k1_bigh / k1_bigs with the large one (the same code; the first
// pass records nothing for them).  PART: 1 the Huffman table (for K2), 2 the
// sequence tables (for K3), 3 both.  With the K2 | K3 fork the two parts run
// on the two streams: each writes its own CompState bytes, and a Huffman
// parse error still decides the frame's error (key_min: its stage sorts
// before the sequence tables' within a block).
template <bool BIG, int PART>
__global__ __launch_bounds__(K1_LANES) void zd_k_tables(const uint8_t* __restrict__ src, uint64_t src_size,
                                                        const CompBlock* __restrict__ comp, CompState* cstate,
                                                        FrameState* fstate, const uint32_t* __restrict__ list,
                                                        uint32_t n_list, uint16_t* luts, uint16_t* fses,
                                                        uint32_t* huge) {
  typedef typename std::conditional<BIG, K1Lane, K1LaneS>::type LN;
  __shared__ LN lanes[K1_LANES];
  const uint32_t li = blockIdx.x * K1_LANES + threadIdx.x;
  if (li >= n_list) return;
  K1T(k0);
#ifdef ZD_K1_PROF
  struct Done { uint64_t t; __device__ ~Done() { K1T(k1); K1ADD(6, t, k1); atomicAdd((unsigned long long*)&k1_prof[7], 1ull); } } done_{k0};
#endif
  LN& L = lanes[threadIdx.x];
  const uint32_t ci = list[li];
  if (BIG && !(((PART & 1) && cstate[ci].k1_bigh) || ((PART & 2) && cstate[ci].k1_bigs))) return;
  const CompBlock C = comp[ci];
  if (C.prebuilt) return;
  const uint8_t* blk = src + C.src;
  if ((PART & 1) && C.lit_type == LIT_COMPRESSED && C.host_stage > PS_HUF_DESC) {
    int p = 0;
    const int st = k1_huffman_lane(blk + C.lit_data, src, src + src_size, L, luts + (uint64_t)C.lut_slot * LUT_ENTRIES, &p);
    if (!BIG && st == K1_BIG) {
      cstate[ci].k1_bigh = 1;
      return;
    }
    if (st == K1_HUGE) {
      // the third pass builds this tree (its error, if any, sorts before the
      // sequence tables' in key_min); Block::parse goes on to the sequences
      huge[1 + atomicAdd(&huge[0], 1u)] = ci;
    } else if (st == ZD_E_OUT_OF_DOMAIN) {
      // the tree parsed (the reference's Block::parse goes on to the
      // sequences section) but no GPU LUT holds it: out of domain where the
      // reference would decode these literals, after every parse error of
      // the frame and every decode error of the blocks before
      key_min(fstate, C.frame, make_key(PH_DECODE, C.block_in_frame, DS_LITERALS, 0, ZD_E_OUT_OF_DOMAIN));
    } else if (st) {
      key_min(fstate, C.frame, make_key(PH_PARSE, C.block_in_frame, PS_HUF_DESC, 0, st));
      return;                                     // Block::parse stops at the literals section
    } else {
      cstate[ci].huf_bits = (uint8_t)p;
    }
  }
  if ((PART & 2) && C.nseq > 0 && C.host_stage > PS_SEQ_TABLES) {
    uint8_t al[3] = {0, 0, 0};
    uint32_t bo = 0, bsz = 0;
    int sub = 0;
    const int st = k1_sequences_lane(blk, C, L, fses + (uint64_t)C.fse_slot * FSE_SLOT, al, &bo, &bsz, &sub);
    if (!BIG && st == K1_BIG) {
      cstate[ci].k1_bigs = 1;
      return;
    }
    for (int k = 0; k < 3; k++)
      if (C.modes[k] != M_REPEAT && (sub > k || !st)) cstate[ci].al[k] = al[k];
    cstate[ci].bs_off = bo;
    cstate[ci].bs_size = bsz;
    if (st) key_min(fstate, C.frame, make_key(PH_PARSE, C.block_in_frame, PS_SEQ_TABLES, (uint32_t)sub, st));
  }
}

// Trees whose weight stream runs past 255 weights (non-conforming input):
// one block per lane, four lanes per workgroup, a grid that walks the list
// the first two passes appended to (huge[0] blocks).  The reference keeps
// every weight: symbol i is `i as u8`, and from_number_of_bits sorts by
// (width, symbol byte), so the tree depends only on how many weights of each
// width each byte value has -- counted, not stored: one run of the weight
// stream for from_weights' sum (huffman.rs:177-203), a second for the counts,
// then the same LUT fill as k1_huffman_lane in (width desc, byte asc) order
// (equal (width, byte) leaves are interchangeable).
constexpr int K1H_LANES = 1, K1H_GRID = 64;
struct K1LaneH {
  static constexpr uint32_t SYMS = 256, WFSE = FSE_TAB;
  uint16_t fse[FSE_TAB];
  uint8_t sym[FSE_TAB];
  uint16_t next[256];
  int16_t dist[256];
  uint32_t cnt[32][256];                          // weights per (code width, symbol byte)
  uint32_t tot[32], start[32], placed[32];
};

__device__ int k1_huffman_huge(const uint8_t* desc, const uint8_t* src, const uint8_t* src_end, K1LaneH& L,
                               uint16_t* lut, int* p_out, uint32_t* deep) {
  uint32_t sum = 0, maxw = 0, nw = 0;
  bool panic = false;
  int st = k1_weight_stream(desc, src, src_end, L, [&](uint32_t, uint32_t w) {
    if (w) {
      if (w - 1 >= 32 || sum > 0xFFFFFFFFu - (1u << (w - 1))) panic = true;
      else sum += 1u << (w - 1);
      maxw = w > maxw ? w : maxw;
    }
    return true;
  }, &nw);
  if (st) return st;
  if (panic || sum == 0) return ZD_E_REF_PANIC;
  int p = highbit32(sum);
  if ((1ull << p) < sum) p++;
  if (p >= 32) return ZD_E_REF_PANIC;
  const uint8_t rest = (uint8_t)((1u << p) - sum);
  if (rest == 0) return ZD_E_REF_PANIC;           // D3
  const uint32_t manquant = (uint32_t)highbit32(rest) + 1;
  if (maxw > (uint32_t)p + 1 || manquant > (uint32_t)p + 1) return ZD_E_REF_PANIC;
  for (int w = 0; w <= p; w++)
    for (int b = 0; b < 256; b++) L.cnt[w][b] = 0;
  uint32_t nw2 = 0;
  st = k1_weight_stream(desc, src, src_end, L, [&](uint32_t i, uint32_t w) {
    if (w) L.cnt[p + 1 - w][i & 0xFF]++;
    return true;
  }, &nw2);
  if (st) return st;
  L.cnt[p + 1 - manquant][nw & 0xFF]++;          // the implied last symbol
  if (p > LUT_MAX_BITS) {
    *p_out = p;
    return deep_build((uint32_t*)lut, p,
                      [&](int w) {
                        uint32_t t = 0;
                        for (int b = 0; b < 256; b++) t += L.cnt[w][b];
                        return t;
                      },
                      [&](int w, uint32_t k, uint8_t* dst) {
                        uint32_t r = 0;
                        for (int b = 0; b < 256 && r < k; b++)
                          for (uint32_t c = L.cnt[w][b]; c > 0 && r < k; c--) dst[r++] = (uint8_t)b;
                      },
                      deep);
  }
  const uint32_t T = 1u << p;
  uint32_t pos = 0;
  for (int w = p; w >= 1; w--) {
    uint32_t t = 0;
    for (int b = 0; b < 256; b++) t += L.cnt[w][b];
    L.tot[w] = t;
    if (!t) continue;
    const uint32_t S = 1u << (p - w);
    const uint32_t al = (pos + S - 1) & ~(S - 1);
    lut_holes(lut, p, pos, al);
    const uint32_t fit = (T - al) / S;
    const uint32_t k = t < fit ? t : fit;
    L.start[w] = al;
    L.placed[w] = k;
    pos = al + k * S;
  }
  lut_holes(lut, p, pos, T);
  for (int w = p; w >= 1; w--) {
    if (!L.tot[w]) continue;
    const uint32_t S = 1u << (p - w);
    uint32_t r = 0;
    for (int b = 0; b < 256 && r < L.placed[w]; b++) {
      const uint16_t ent = (uint16_t)(b | (lut_field((uint32_t)w, p) << 8));
      for (uint32_t c = L.cnt[w][b]; c > 0 && r < L.placed[w]; c--, r++)
        for (uint32_t e = 0; e < S; e++) lut[L.start[w] + r * S + e] = ent;
    }
  }
  *p_out = p;
  return 0;
}

__global__ __launch_bounds__(K1H_LANES) void zd_k_tables_huge(const uint8_t* __restrict__ src, uint64_t src_size,
                                                              const CompBlock* __restrict__ comp, CompState* cstate,
                                                              FrameState* fstate, const uint32_t* __restrict__ huge,
                                                              uint16_t* luts, uint32_t* deep) {
  __shared__ K1LaneH lanes[K1H_LANES];
  K1LaneH& L = lanes[threadIdx.x];
  const uint32_t n = huge[0];
  for (uint32_t k = blockIdx.x * K1H_LANES + threadIdx.x; k < n; k += gridDim.x * K1H_LANES) {
    const uint32_t ci = huge[1 + k];
    const CompBlock C = comp[ci];
    int p = 0;
    const int st = k1_huffman_huge(src + C.src + C.lit_data, src, src + src_size, L,
                                   luts + (uint64_t)C.lut_slot * LUT_ENTRIES, &p, deep);
    if (st == ZD_E_OUT_OF_DOMAIN)
      key_min(fstate, C.frame, make_key(PH_DECODE, C.block_in_frame, DS_LITERALS, 0, ZD_E_OUT_OF_DOMAIN));
    else if (st)
      key_min(fstate, C.frame, make_key(PH_PARSE, C.block_in_frame, PS_HUF_DESC, 0, st));
    else
      cstate[ci].huf_bits = (uint8_t)p;
  }
}

// ---------------------------------------------------------------------------
// Per-lane backward bitstream windows (K2, K3)
// ---------------------------------------------------------------------------
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef __attribute__((address_space(1))) const u32x4a4 g_u32x4a4;   // global (HBM) window loads
typedef __attribute__((address_space(3))) uint16_t lds_u16;          // LDS tables
typedef __attribute__((address_space(1))) const uint16_t g_u16;      // HBM tables
typedef uint32_t u32x4g __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4g g_u32x4g;            // record pairs (16-byte aligned)
typedef __attribute__((address_space(1))) uint32_t g_u32;

// MSB-first field of k bits from the top of t, k in [0, 63], no selects:
// (t >> 1) >> (63 - k) is 0 for k = 0.
__device__ inline uint32_t take_top(uint64_t& t, uint32_t k) {
  const uint32_t v = (uint32_t)((t >> 1) >> (63 - k));
  t <<= k;
  return v;
}

// Byte-aligned window: 16 bytes loaded at an unaligned address ending at
// the byte that holds bit pos-1 (gfx950 runs HSA queues in unaligned access
// mode, so global_load_dwordx4 takes any byte address), clamped at the input
// base.  sh = 128 - (pos - window start) is then in [0, 31] (0..7 unless
// clamped), so the top 64 bits below pos are one funnel with no edge cases.
struct WinU {
  uint64_t w0, w1;
  uint32_t sh;
};
typedef uint64_t u64x2a1 __attribute__((ext_vector_type(2), aligned(1)));
typedef __attribute__((address_space(1))) const u64x2a1 g_u64x2a1;
__device__ inline WinU winu_load(const uint8_t* s, uintptr_t base, int32_t pos) {
  const int32_t tb = (pos + 7) >> 3;
  uintptr_t a = (uintptr_t)((intptr_t)s + tb - 16);
  a = a < base ? base : a;
  const u64x2a1 v = *(g_u64x2a1*)a;
  WinU w;
  w.w0 = v.x;
  w.w1 = v.y;
  w.sh = (uint32_t)((int32_t)(((intptr_t)a + 16 - (intptr_t)s) * 8) - pos);
  return w;
}
// top 64 bits below pos - d (d + sh <= 94)
__device__ inline uint64_t winu_top(const WinU& w, uint32_t d) {
  const uint32_t k = w.sh + d;
  const uint64_t f = (w.w1 << (k & 63)) | ((w.w0 >> 1) >> ((63 - k) & 63));
  return k < 64 ? f : (w.w0 << (k & 63));
}

typedef uint32_t u32x4ua __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const u32x4ua g_u32x4ua;

// A backward bitstream window of 24 bytes: bits [wb, wb + 192) of the stream
// (bit 0 = LSB of byte 0), loaded unaligned as the 24 bytes ending at the
// byte that holds bit pos - 1, clamped at m = base - s (<= 0), the lowest
// byte offset a window may start at.  Loaded at pos_{i+1}, it covers every
// bit K3's steps i+1 and i+2 read (each step reads at most 63 extra + 27
// state bits), so a window load has a whole step more to land.
struct Win6 {
  uint32_t w0, w1, w2, w3, w4, w5;
  int32_t wb;
};
typedef uint32_t u32x2ua __attribute__((ext_vector_type(2), aligned(1)));
typedef __attribute__((address_space(1))) const u32x2ua g_u32x2ua;
__device__ inline Win6 win6_load(const uint8_t* s, int32_t m, int32_t pos) {
  const int32_t tb = (pos + 7) >> 3;
  const int32_t o = max(tb - 24, m);
  const u32x4ua v = *(g_u32x4ua*)(s + o);
  const u32x2ua u = *(g_u32x2ua*)(s + o + 16);
  Win6 w;
  w.w0 = v.x; w.w1 = v.y; w.w2 = v.z; w.w3 = v.w; w.w4 = u.x; w.w5 = u.y;
  w.wb = o * 8;
  return w;
}
__device__ inline uint32_t win6_bits(const Win6& w, int32_t p, uint32_t S) {
  const uint32_t y = (uint32_t)(p - (int32_t)S - w.wb);
  const uint32_t k = y >> 5;
  uint32_t lo = k == 0 ? w.w0 : w.w1;
  uint32_t hi = k == 0 ? w.w1 : w.w2;
  lo = k >= 2 ? w.w2 : lo;
  hi = k >= 2 ? w.w3 : hi;
  lo = k >= 3 ? w.w3 : lo;
  hi = k >= 3 ? w.w4 : hi;
  lo = k >= 4 ? w.w4 : lo;
  hi = k >= 4 ? w.w5 : hi;
  lo = k >= 5 ? w.w5 : lo;
  hi = k >= 5 ? 0u : hi;
  return __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit(hi, lo, y & 31), 0, S);
}


// The 64 bits below q of a 24-byte window, MSB-first (q - 32 >= wb, q <= wb + 192;
// bits below the window read as zero: K2 looks at the top 44 only).
__device__ inline uint64_t win6_top64(const Win6& w, int32_t q) {
  const uint32_t y = (uint32_t)(q - 32 - w.wb);          // bit offset of the top dword's low end
  const uint32_t k = y >> 5, sh = y & 31;                // k in [0, 5]
  // w[k-1], w[k], w[k+1] by the three bits of k: three selects deep
  // (a 5-deep chain of k >= i selects: K2 on C4 4 GiB 2.21 ms, this 2.18-2.20)
  const bool b0 = (k & 1) != 0, b1 = (k & 2) != 0, b2 = k >= 4;
  const uint32_t a01 = b0 ? w.w0 : 0u, a23 = b0 ? w.w2 : w.w1, a45 = b0 ? w.w4 : w.w3;
  const uint32_t b01 = b0 ? w.w1 : w.w0, b23 = b0 ? w.w3 : w.w2, b45 = b0 ? w.w5 : w.w4;
  const uint32_t c01 = b0 ? w.w2 : w.w1, c23 = b0 ? w.w4 : w.w3, c45 = b0 ? 0u : w.w5;
  const uint32_t a = b2 ? a45 : (b1 ? a23 : a01);
  const uint32_t b = b2 ? b45 : (b1 ? b23 : b01);
  const uint32_t c = b2 ? c45 : (b1 ? c23 : c01);
  const uint32_t hi = __builtin_amdgcn_alignbit(c, b, sh), lo = __builtin_amdgcn_alignbit(b, a, sh);
  return ((uint64_t)hi << 32) | lo;
}

// ---------------------------------------------------------------------------
// K2: Huffman literals (literals.rs:49-86 + huffman.rs:205-218), one STREAM
// per lane: a workgroup (one wave) takes K2_BLOCKS blocks, 4 lanes each, the
// blocks' LUTs in LDS.  Each lane walks its stream through a 16-byte register
// window, K2_GROUP symbols per window (<= 88 bits of a >= 97-bit window), and
// stores the group's bytes with one 8-byte store.  Stream k decodes to
// k * ceil(R/4) (RFC 8878 3.1.1.3.1.6); the reference concatenates streams
// decoded until empty (literals.rs:68-81), which is the same bytes whenever
// each stream holds its RFC share.  A block whose tree is deeper than 11 bits
// makes its workgroup read LUTs from HBM.
// ---------------------------------------------------------------------------
#ifndef ZD_K2_BLOCKS
#define ZD_K2_BLOCKS 8
#endif
constexpr int K2_BLOCKS = ZD_K2_BLOCKS;
constexpr int K2_LANES = 4 * K2_BLOCKS;
constexpr int K2_GROUP = 8;
static_assert(K2_LANES <= 64, "K2 workgroup must be a single wave");
static_assert(K2_GROUP * LUT_MAX_BITS <= 97, "a group must fit one window");
static_assert((K2_GROUP / 2) * LUT_MAX_BITS <= 64, "half a group must fit 64 bits");
typedef __attribute__((address_space(1))) uint64_t g_u64a1 __attribute__((aligned(1)));
typedef __attribute__((address_space(1))) u64x2a1 gw_u64x2a1;

// ---------------------------------------------------------------------------
// K2's pair table.  Trees of maxBits p <= 11 are decoded through a table of
// u32 entries, each giving the symbols a bit prefix starts with -- two when
// both codes fit the prefix -- so K2's serial chain (LDS lookup, shift) runs
// once per 1.6-1.8 symbols on zstd's literals instead of once per symbol.
// zd_k_huf_pairs converts a block's u16 LUT (K1) into it, in place in the LUT
// slot.  Prefixes are 10 bits, except that the lowest L 10-bit prefixes --
// those whose first code is 11 bits: insert places the longest codes first
// (huffman.rs:132-175), so they are the leading ones -- are split into their
// two 11-bit prefixes.  With x the top 11 bits of the window the entry is
//   j = min(x, (x >> 1) + L)
// (x for x >> 1 < L, the 10-bit prefix + L past them), 1024 + L entries.
//   bits 0-4   (32 - bits consumed) & 31      (v_alignbit takes it as is)
//   bits 5-7   0      bit 8  PR_TWO: a second symbol      bits 9-10  0
//              (K2 sums a half's four entries: bits 0-7 give its bits,
//              bits 8-10 its second symbols)
//   bits 11-14 width of the first code (PR_BAD: the absent node's depth;
//              0 with PR_BAD: PR_LONG, below)
//   bit 15     PR_BAD: K2's fast loop stops (absent node, or PR_LONG)
//   bits 16-23 first symbol             bits 24-31 second symbol (or 0)
// A deep 10-bit prefix past the leading run (only a malformed tree's last
// gap) is PR_LONG: the symbols of its 11-bit prefixes 0 / 1 in bits 16-23 /
// 24-31, bit 5 / 6 set when that node is absent (the exact path decodes it).
// ---------------------------------------------------------------------------
constexpr uint32_t PR_TWO = 1u << 8, PR_BAD = 1u << 15, PR_BAD0 = 1u << 5, PR_BAD1 = 1u << 6;
constexpr int PR_BITS = 10;
constexpr uint32_t PR_LMAX = 128;                  // split prefixes: n11 <= 256 codes of 11 bits, + a hole
constexpr uint32_t PR_ENTRIES = (1u << PR_BITS) + PR_LMAX;
constexpr uint32_t PR_L_AT = PR_ENTRIES;           // u32 index of L in the slot
static_assert((PR_L_AT + 1) * 4 <= LUT_ENTRIES * 2, "a pair table fits its LUT slot");
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(1))) const uint32_t gc_u32;

__device__ inline uint32_t pr_index(uint32_t x, uint32_t L) { return min(x, (x >> 1) + L); }

// The entry of the nb-bit prefix x (nb 10 or 11, p <= 11, the first code no
// longer than nb) from the u16 LUT (decode entries of the p-bit prefix,
// lut_field's (32 - f) form).
__device__ inline uint32_t pr_entry(const lds_u16* u, int p, uint32_t x, int nb) {
  auto at = [&](uint32_t y) { return p >= nb ? y << (p - nb) : y >> (nb - p); };
  const uint32_t e1 = u[at(x)];
  const uint32_t w1 = lut_width(e1, true);
  if (e1 & LUT_ABSENT) return PR_BAD | w1 << 11;
  uint32_t total = w1, two = 0, s2 = 0;
  if (w1 < (uint32_t)nb) {
    const uint32_t e2 = u[at((x << w1) & ((1u << nb) - 1))];
    const uint32_t w2 = lut_width(e2, true);
    if (!(e2 & LUT_ABSENT) && w2 <= nb - w1) {
      total += w2;
      two = PR_TWO;
      s2 = e2 & 0xFF;
    }
  }
  return ((32u - total) & 31) | two | w1 << 11 | (e1 & 0xFF) << 16 | s2 << 24;
}

// One symbol of the p-bit prefix idx (p <= 11) from a pair table, as the u16
// LUT gives it: the symbol, *nb its width (an absent node: its depth, *absent).
template <typename TP>
__device__ inline uint32_t pr_one(TP dl, uint32_t L, int p, uint32_t idx, int32_t* nb, bool* absent) {
  const uint32_t x = idx << (11 - p);
  const uint32_t e = dl[pr_index(x, L)];
  const uint32_t w = (e >> 11) & 15;
  if ((e & PR_BAD) && w == 0) {                   // PR_LONG
    const uint32_t b = x & 1;
    *nb = 11;
    *absent = (e & (b ? PR_BAD1 : PR_BAD0)) != 0;
    return (e >> (16 + 8 * b)) & 0xFF;
  }
  *nb = (int32_t)w;
  *absent = (e & PR_BAD) != 0;
  return (e >> 16) & 0xFF;
}

// zd_k_huf_pairs: one wave per block of K1's list that built a LUT of maxBits
// <= 11: the LUT is staged in LDS, L found by a wave reduction, then the
// slot is overwritten with the pair table and L.
constexpr int PR_WAVES = 4;
__global__ __launch_bounds__(64 * PR_WAVES) void zd_k_huf_pairs(const CompBlock* __restrict__ comp,
                                                                 const CompState* __restrict__ cstate,
                                                                 const uint32_t* __restrict__ list, uint32_t n_list,
                                                                 uint16_t* luts) {
  __shared__ __attribute__((aligned(16))) uint16_t u[PR_WAVES][1 << K2_LUT_BITS];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t li = blockIdx.x * PR_WAVES + wv;
  if (li >= n_list) return;                        // whole waves: no workgroup barrier below
  const uint32_t ci = list[li];
  const CompBlock& C = comp[ci];
  if (C.lit_type != LIT_COMPRESSED || C.host_stage <= PS_HUF_DESC || C.prebuilt) return;
  const int p = cstate[ci].huf_bits;
  if (p == 0 || p > K2_LUT_BITS) return;
  uint16_t* slot = luts + (uint64_t)C.lut_slot * LUT_ENTRIES;
  const lds_u16* U = (const lds_u16*)u[wv];
  {                                                // 16 bytes per lane and step
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const int n16 = (1 << p) / 8;
    if (n16 == 0) { if (lane < (1 << p)) u[wv][lane] = slot[lane]; }
    else for (int e = lane; e < n16; e += 64) ((u32x4*)u[wv])[e] = ((const u32x4*)slot)[e];
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // deep(i): the 10-bit prefix i starts with an 11-bit code or absent node
  auto deep = [&](uint32_t i) {
    return p > PR_BITS && (lut_width(U[2 * i], true) > PR_BITS || lut_width(U[2 * i + 1], true) > PR_BITS);
  };
  uint32_t first = 1u << PR_BITS;                  // the lowest prefix that is not deep
  for (uint32_t i = lane; i < (1u << PR_BITS); i += 64)
    if (!deep(i)) { first = i; break; }
  for (int o = 32; o > 0; o >>= 1) first = min(first, (uint32_t)__shfl_xor((int)first, o));
  const uint32_t L = min(first, PR_LMAX);
  uint32_t* dl = (uint32_t*)slot;
  for (uint32_t j = lane; j < (1u << PR_BITS) + L; j += 64) {
    uint32_t ent;
    if (j < 2 * L) {
      ent = pr_entry(U, p, j, 11);
    } else {
      const uint32_t i = j - L;
      if (deep(i)) {                               // PR_LONG
        const uint32_t e0 = U[2 * i], e1 = U[2 * i + 1];
        ent = PR_BAD | (e0 & 0xFF) << 16 | (e1 & 0xFF) << 24 | ((e0 & LUT_ABSENT) ? PR_BAD0 : 0u) |
              ((e1 & LUT_ABSENT) ? PR_BAD1 : 0u);
      } else {
        ent = pr_entry(U, p, i, PR_BITS);
      }
    }
    dl[j] = ent;
  }
  if (lane == 0) dl[PR_L_AT] = L;
}

// One Huffman stream of a tree of maxBits p <= 11 from its pair table (LDS,
// or HBM for a workgroup with a deeper tree; huffman.rs:205-218 on a
// BackwardBitParser, parsing.rs:191-259).  Fast path while at least
// K2_GROUP * 12 bits remain: 24-byte windows two groups ahead (the window
// loaded when group g ends, ending at the byte of pos_{g+1}, covers groups
// g+1 and g+2, so a load has a whole group more to land); a group is two
// halves of 4 lookups (<= 44 bits each, 4-8 symbols), one 8-byte store per
// half at the half's first byte (its bytes past the half's symbols are
// overwritten by what follows).  Both groups of a trip run on every lane; a
// lane that stops keeps its position and stores into the slack.  The tail
// (and any group that meets PR_BAD) goes symbol by symbol with the
// reference's checks.
template <typename TP>
__device__ int huf_stream_pr(const uint8_t* bs, uint32_t size, uintptr_t base, TP dl, uint32_t L, int p,
                             uint8_t* out, uint32_t cap, uint32_t* count_out, uint8_t* dummy) {
  uint32_t count = 0;
  *count_out = 0;
  if (size == 0) return ZD_E_EMPTY_INPUT_DATA;
  const uint8_t lastb = bs[size - 1];
  if (lastb == 0) return ZD_E_NULL_BYTE;
  int32_t pos = (int32_t)(8 * (size - 1)) + highbit32(lastb);
  constexpr uint32_t ROOM = 2 * K2_GROUP;          // the bytes a group's two stores may touch
  const int32_t m = (int32_t)max((intptr_t)base - (intptr_t)bs, (intptr_t)-24);
  Win6 wa = win6_load(bs, m, pos);
  asm volatile("" ::: "memory");
  *(g_u64a1*)dummy = 0;
  Win6 wb = win6_load(bs, m, pos);
  asm volatile("" ::: "memory");
  *(g_u64a1*)dummy = 0;
  bool live = pos >= K2_GROUP * LUT_MAX_BITS && count + ROOM <= cap;
  auto group = [&](Win6& w) {
    uint64_t acc[2];
    uint32_t n[2], used = 0, bad = 0;
    // the group's 96 bits below pos, MSB first in (hi, lo, x), taken from the
    // window once: sp = pos - wb - 96 in 0..96 (the window covers >= 97 bits
    // below pos; bits under it read as 0 and a group consumes <= 88)
    const uint32_t sp = (uint32_t)(pos - w.wb - 96);
    const bool b0 = (sp & 32) != 0, b1 = (sp & 64) != 0;
    const uint32_t a0 = b0 ? w.w1 : w.w0, a1 = b0 ? w.w2 : w.w1, a2 = b0 ? w.w3 : w.w2;
    const uint32_t a3 = b0 ? w.w4 : w.w3, a4 = b0 ? w.w5 : w.w4, a5 = b0 ? 0u : w.w5;
    const uint32_t c0 = b1 ? a2 : a0, c1 = b1 ? a3 : a1, c2 = b1 ? a4 : a2, c3 = b1 ? a5 : a3;
    uint32_t hi = __builtin_amdgcn_alignbit(c3, c2, sp), lo = __builtin_amdgcn_alignbit(c2, c1, sp);
    uint32_t x = __builtin_amdgcn_alignbit(c1, c0, sp);
#pragma unroll
    for (int h = 0; h < 2; h++) {
      // half 1 peeks at most 3 * 11 + 11 bits past its start: hi:lo hold them
      uint32_t S = 0;
      uint64_t a = 0;
#pragma unroll
      for (int j = 0; j < K2_GROUP / 2; j++) {
        const uint32_t e = dl[pr_index(hi >> 21, L)];
        hi = __builtin_amdgcn_alignbit(hi, lo, e);
        lo = __builtin_amdgcn_alignbit(lo, h == 0 ? x : 0u, e);
        if (h == 0) x = __builtin_amdgcn_alignbit(x, 0u, e);
        const uint32_t c8 = 8 * j + 8 * ((S >> 8) & 7);          // bytes before this lookup's
        a |= (uint64_t)(e >> 16) << c8;
        S += e;
        bad |= e;
      }
      used += 32 * (K2_GROUP / 2) - (S & 0xFF);
      acc[h] = a;
      n[h] = K2_GROUP / 2 + ((S >> 8) & 7);
    }
    const bool ok = live && !(bad & PR_BAD);
    pos = ok ? pos - (int32_t)used : pos;
    w = win6_load(bs, m, pos);
    asm volatile("" ::: "memory");
    // the group's bytes as one 16-byte store: half 1's after half 0's n[0]
    // (4..8); bytes past a half's symbols are 0
    const uint32_t s0 = 8 * n[0] - 32;                      // 0..32
    const uint64_t v0 = acc[0] | ((acc[1] << s0) << 32);
    const uint64_t v1 = s0 == 32 ? acc[1] : acc[1] >> (32 - s0);
    *(gw_u64x2a1*)(ok ? out + count : dummy) = (u64x2a1){v0, v1};
    count += ok ? n[0] + n[1] : 0;
    live = ok && pos >= K2_GROUP * LUT_MAX_BITS && count + ROOM <= cap;
  };
  while (live) {
    group(wa);
    group(wb);
  }
  // symbol by symbol with the reference's checks (huf_stream's tail)
  int st = 0;
  WinU w = winu_load(bs, base, pos);
  int32_t p0 = pos;
  const uint32_t sh = 64 - p;
  while (pos > 0 && !st) {
    if ((p0 - pos) + (int32_t)w.sh > 100) {
      w = winu_load(bs, base, pos);
      p0 = pos;
    }
    uint32_t idx = (uint32_t)(winu_top(w, (uint32_t)(p0 - pos)) >> sh);
    if (pos < p) idx &= ~((1u << (p - pos)) - 1);     // zero-fill below the stream (parsing.rs peek)
    int32_t nb;
    bool absent;
    const uint32_t sym = pr_one(dl, L, p, idx, &nb, &absent);
    if (absent) st = nb <= pos ? ZD_E_REF_PANIC : ZD_E_NOT_ENOUGH_BITS;
    else if (nb > pos) st = ZD_E_NOT_ENOUGH_BITS;
    else {
      pos -= nb;
      if (count < cap) out[count] = (uint8_t)sym;
      count++;
    }
  }
  *count_out = count;
  return st;
}

// One Huffman stream, backward (huffman.rs:205-218 on a BackwardBitParser,
// parsing.rs:191-259), LUT in HBM: a workgroup with a tree deeper than K2's
// LDS tables (maxBits 12).  Fast path while at least K2_GROUP * 12 bits remain:
// a byte-aligned 16-byte window per group of 8 symbols, the top 64 bits
// taken twice (4 symbols each, <= 48 bits), one lookup and one shift per
// symbol, one 8-byte store per group.  The tail (and any group that meets an
// absent tree node) goes symbol by symbol with the reference's checks.
__device__ int huf_stream(const uint8_t* bs, uint32_t size, uintptr_t base, g_u16* lut, int p, uint8_t* out,
                          uint32_t cap, uint32_t* count_out, uint8_t* dummy) {
  uint32_t count = 0;
  *count_out = 0;
  if (size == 0) return ZD_E_EMPTY_INPUT_DATA;
  const uint8_t lastb = bs[size - 1];
  if (lastb == 0) return ZD_E_NULL_BYTE;
  int32_t pos = (int32_t)(8 * (size - 1)) + highbit32(lastb);
  const uint32_t sh = 64 - p;
  // The next group's window is loaded before this group's store: vmcnt
  // drains in issue order, so a group waits for its window, not the store.
  // The loop entry repeats that order (a store into the block's literal
  // slack, never read) so the wait at the loop head stays vmcnt(1).
  {
  WinU w = winu_load(bs, base, pos);
  asm volatile("" ::: "memory");
  *(g_u64a1*)dummy = 0;
  while (pos >= K2_GROUP * LUT_MAX_BITS && count + K2_GROUP <= cap) {
    uint64_t acc = 0;
    uint32_t used = 0, bad = 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint64_t t = winu_top(w, used);
#pragma unroll
      for (int j = 0; j < K2_GROUP / 2; j++) {
        const uint32_t e = lut[(uint32_t)(t >> sh)];
        const uint32_t nb = lut_width(e, p <= K2_LUT_BITS);
        bad |= e & LUT_ABSENT;
        t <<= nb;
        used += nb;
        acc |= (uint64_t)(e & 0xFF) << (8 * (h * (K2_GROUP / 2) + j));
      }
    }
    if (bad) break;                            // redo this group with the exact checks
    pos -= (int32_t)used;
    w = winu_load(bs, base, pos);
    asm volatile("" ::: "memory");
    *(g_u64a1*)(out + count) = acc;
    count += K2_GROUP;
  }
  }
  // symbol by symbol with the reference's checks; one window serves while
  // its top p bits stay inside it (the tail from the fast loop: < 88 bits)
  int st = 0;
  WinU w = winu_load(bs, base, pos);
  int32_t p0 = pos;
  while (pos > 0 && !st) {
    if ((p0 - pos) + (int32_t)w.sh > 100) {
      w = winu_load(bs, base, pos);
      p0 = pos;
    }
    uint32_t idx = (uint32_t)(winu_top(w, (uint32_t)(p0 - pos)) >> sh);
    if (pos < p) idx &= ~((1u << (p - pos)) - 1);     // zero-fill below the stream (parsing.rs peek)
    const uint32_t e = lut[idx];
    const int32_t nb = (int32_t)lut_width(e, p <= K2_LUT_BITS);
    if (e & LUT_ABSENT) st = nb <= pos ? ZD_E_REF_PANIC : ZD_E_NOT_ENOUGH_BITS;
    else if (nb > pos) st = ZD_E_NOT_ENOUGH_BITS;
    else {
      pos -= nb;
      if (count < cap) out[count] = (uint8_t)e;
      count++;
    }
  }
  *count_out = count;
  return st;
}

// One stream of a deep tree (deep_build): symbol by symbol, the top p bits
// (p <= 31) looked up in the slot's code intervals; a code that falls between
// intervals is an absent tree node at the depth of the largest aligned block
// of the gap around it (as lut_holes).  The reference's checks as in
// huf_stream's tail.
__device__ int huf_stream_deep(const uint8_t* bs, uint32_t size, uintptr_t base, const uint32_t* tab, int p,
                               uint8_t* out, uint32_t cap, uint32_t* count_out, const uint8_t* pool) {
  uint32_t count = 0;
  *count_out = 0;
  if (size == 0) return ZD_E_EMPTY_INPUT_DATA;
  const uint8_t lastb = bs[size - 1];
  if (lastb == 0) return ZD_E_NULL_BYTE;
  int32_t pos = (int32_t)(8 * (size - 1)) + highbit32(lastb);
  const uint32_t G = tab[0] & ~DEEP_IN_POOL;
  const uint8_t* syms = (tab[0] & DEEP_IN_POOL) ? pool + tab[DEEP_POOL_AT] : (const uint8_t*)tab + DEEP_SYMS_AT;
  const uint64_t T = 1ull << p;
  int st = 0;
  while (pos > 0 && !st) {
    const WinU w = winu_load(bs, base, pos);
    uint32_t idx = (uint32_t)(winu_top(w, 0) >> (64 - p));
    if (pos < p) idx &= ~((1u << (p - pos)) - 1);     // zero-fill below the stream (parsing.rs peek)
    uint64_t a = 0, b = T;
    int32_t nb = -1;
    uint8_t sym = 0;
    for (uint32_t g = 0; g < G; g++) {
      const uint32_t lo = tab[1 + 4 * g], hi = tab[2 + 4 * g];
      if (idx < lo) { b = lo; break; }
      if (idx < hi) {
        nb = (int32_t)tab[3 + 4 * g];
        sym = syms[tab[4 + 4 * g] + ((idx - lo) >> (p - nb))];
        break;
      }
      a = hi;
    }
    if (nb < 0) {
      int k = p;
      for (; k > 0; k--) {
        const uint64_t lo = (uint64_t)idx & ~((1ull << k) - 1);
        if (lo >= a && lo + (1ull << k) <= b) break;
      }
      st = p - k <= pos ? ZD_E_REF_PANIC : ZD_E_NOT_ENOUGH_BITS;
    } else if (nb > pos) {
      st = ZD_E_NOT_ENOUGH_BITS;
    } else {
      pos -= nb;
      if (count < cap) out[count] = sym;
      count++;
    }
  }
  *count_out = count;
  return st;
}

__global__ __launch_bounds__(K2_LANES) void zd_k_huffman(const uint8_t* __restrict__ src,
                                                         const CompBlock* __restrict__ comp, CompState* cstate,
                                                         FrameState* fstate, const uint32_t* __restrict__ list,
                                                         uint32_t n_list, const uint16_t* __restrict__ luts,
                                                         uint8_t* lits, uint32_t* k2done,
                                                         const uint8_t* __restrict__ deep_pool) {
#ifndef ZD_K2_LDS_PAD
#define ZD_K2_LDS_PAD 0
#endif
  __shared__ __attribute__((aligned(16))) uint32_t dl[K2_BLOCKS][PR_ENTRIES + ZD_K2_LDS_PAD];
  __shared__ uint32_t counts[K2_BLOCKS][4];
  __shared__ int errs[K2_BLOCKS][4];
  const int lane = threadIdx.x, b = lane >> 2, k = lane & 3;
  const uint32_t li = blockIdx.x * K2_BLOCKS + b;
  bool act = li < n_list;
  const uint32_t ci = act ? list[li] : 0;
  CompBlock C;
  if (act) C = comp[ci];
  if (act) {
    const uint64_t key0 = fstate[C.frame].key;
    if (key0 != KEY_NONE && key_phase(key0) == PH_PARSE) act = false;
  }
  int p = 0;
  const uint16_t* g = nullptr;
  if (act) {
    const uint32_t hs = (uint32_t)C.huf_src;
    p = cstate[hs].huf_bits;
    g = luts + (uint64_t)comp[hs].lut_slot * LUT_ENTRIES;
    if (p == 0) {            // LUT not built (K1 stopped: parse error or out of domain)
      if (k == 0) cstate[ci].stop = 1;
      act = false;
    }
  }
  const bool use_lds = __ballot(act && p > K2_LUT_BITS) == 0;
  if (use_lds && act) {      // the block's 4 lanes copy its pair table, 16 bytes at a time
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const u32x4 g_u4;
    typedef __attribute__((address_space(3))) u32x4 l_u4;
#pragma unroll 4
    for (int e = k; e < (int)PR_ENTRIES / 4; e += 4) ((l_u4*)dl[b])[e] = ((g_u4*)g)[e];
  }
  const uint32_t L = act && p <= K2_LUT_BITS ? ((const uint32_t*)g)[PR_L_AT] : 0;
  __syncthreads();
  const int m = act ? C.nstreams : 0;
  const uint32_t R = act ? C.lit_regen : 0;
  const uint32_t seg = (R + 3) / 4;
  if (act && k < m) {
    uint32_t off = C.streams;
    for (int j = 0; j < k; j++) off += C.stream_size[j];
    const uint32_t start = (uint32_t)k * seg;
    const uint32_t cap = k < m - 1 ? seg : (R > start ? R - start : 0);
    const uint8_t* blk = src + C.src;
    const uintptr_t lo = (uintptr_t)src;
    // the block's literal slot: R + 16 + lit_extra bytes of literals (the
    // streams laid back-to-back may run past R), then 16 bytes of slack that
    // the fast loops' placeholder stores hit (never read)
    uint8_t* slack = lits + C.lit_out + R + 16 + C.lit_extra;
    uint32_t count;
    int st;
    if (p > LUT_MAX_BITS)
      st = huf_stream_deep(blk + off, C.stream_size[k], lo, (const uint32_t*)g, p, lits + C.lit_out + start, cap,
                           &count, deep_pool);
    else if (use_lds)
      st = huf_stream_pr<const lds_u32*>(blk + off, C.stream_size[k], lo, (const lds_u32*)dl[b], L, p,
                                         lits + C.lit_out + start, cap, &count, slack);
    else if (p <= K2_LUT_BITS)
      st = huf_stream_pr<gc_u32*>(blk + off, C.stream_size[k], lo, (gc_u32*)g, L, p, lits + C.lit_out + start, cap,
                                 &count, slack);
    else
      st = huf_stream(blk + off, C.stream_size[k], lo, (g_u16*)g, p, lits + C.lit_out + start, cap, &count,
                              slack);
    counts[b][k] = count;
    errs[b][k] = st;
    if (st) key_min(fstate, C.frame, make_key(PH_DECODE, C.block_in_frame, DS_LITERALS, k, st));
  }
  __syncthreads();
  // The reference concatenates what each stream decodes until it runs out of
  // bits (literals.rs:68-81).  When a block's streams do not hold their RFC
  // shares (only in non-conforming input), lane 0 lays the streams out
  // back-to-back and the block's lanes decode again into that layout.
  __shared__ uint32_t redo_at[K2_BLOCKS][4];
  __shared__ int redo[K2_BLOCKS];
  if (act && k == 0) {
    bool err = false, rfc = true;
    for (int j = 0; j < m; j++) err |= errs[b][j] != 0;
    uint32_t total = 0;
    for (int j = 0; j < m && !err; j++) {
      const uint32_t cap = j < m - 1 ? seg : (R > (uint32_t)j * seg ? R - (uint32_t)j * seg : 0);
      if (j < m - 1 ? counts[b][j] != seg : counts[b][j] > cap) rfc = false;
      redo_at[b][j] = total;
      total += counts[b][j];
    }
    const bool fits = total <= R + 16 + C.lit_extra;   // the block's literal slot
    if (!rfc && !err && !fits)
      key_min(fstate, C.frame,
              make_key(PH_DECODE, C.block_in_frame, DS_LITERALS, DS_LIT_OVERFLOW_SUB, ZD_E_OUT_OF_DOMAIN));
    redo[b] = !rfc && !err && fits;
    cstate[ci].lit_count = total;
    if (err || (!rfc && !fits)) cstate[ci].stop = 1;
  }
  __syncthreads();
  if (act && k < m && redo[b]) {
    uint32_t off = C.streams;
    for (int j = 0; j < k; j++) off += C.stream_size[j];
    const uint8_t* blk = src + C.src;
    uint32_t count;
    const uint32_t at = redo_at[b][k];
    if (p > LUT_MAX_BITS)
      (void)huf_stream_deep(blk + off, C.stream_size[k], (uintptr_t)src, (const uint32_t*)g, p, lits + C.lit_out + at,
                            counts[b][k], &count, deep_pool);
    else if (use_lds)
      (void)huf_stream_pr<const lds_u32*>(blk + off, C.stream_size[k], (uintptr_t)src, (const lds_u32*)dl[b], L, p,
                                          lits + C.lit_out + at, counts[b][k], &count,
                                          lits + C.lit_out + R + 16 + C.lit_extra);
    else if (p <= K2_LUT_BITS)
      (void)huf_stream_pr<gc_u32*>(blk + off, C.stream_size[k], (uintptr_t)src, (gc_u32*)g, L, p, lits + C.lit_out + at,
                                  counts[b][k], &count, lits + C.lit_out + R + 16 + C.lit_extra);
    else
      (void)huf_stream(blk + off, C.stream_size[k], (uintptr_t)src, (g_u16*)g, p,
                               lits + C.lit_out + at, counts[b][k], &count, lits + C.lit_out + R + 16 + C.lit_extra);
  }
  // zd_k_fused's K4 waves wait for every K2 workgroup: the workgroup (one
  // wave) releases its literals and CompState bytes at agent scope, then counts
  if (k2done) {
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(k2done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
#ifdef ZD_FZ_TRACE
    if (threadIdx.x == 0) atomicMax((unsigned long long*)&fz_k2end, (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
  }
}

// ---------------------------------------------------------------------------
// K3: sequences (sequences.rs:191-237, decoders/sequence.rs:30-93) — the FSE
// state chain only, one block per LANE.  The chain of a block is strictly
// serial (each state update reads bits whose position depends on the
// previous step), so K3 does the least per step that the chain needs: three
// LDS table lookups, the bit position, the three state updates.  It records
// per sequence {bit position before its extra bits, LL/ML/OF states}; the
// values (codes -> baselines, extra bits, repeat offsets) are independent
// per sequence once those are known and are decoded in parallel by K4.
//
// Tables live in LDS, re-encoded on load for the chain (zd_common.h
// k3_entry: nextState | extra-bit count of the symbol << 10 | code-max flag),
// LL 512 | ML 512 | OF 256 entries per lane.  A lane whose OF table is deeper
// than 256 states (AL 9; zstd's offset tables are AL <= 8) makes its
// workgroup use HBM tables in the sym format instead (slow path).
// ---------------------------------------------------------------------------
#ifndef ZD_K3_LANES
#define ZD_K3_LANES 16
#endif
constexpr int K3_LANES = ZD_K3_LANES;
#define K3_CHAIN seq_chain2      // the exact chain (windows two steps ahead)
#ifndef ZD_K3_LA
#define ZD_K3_LA 4                   // windows L steps ahead (C4: L2 17.3 ms, L3 14.5, L4 13.8)
#endif
#ifndef ZD_K3_WN
#define ZD_K3_WN 6                   // window dwords
#endif
#define K3_FAST seq_chainfl<ZD_K3_LA, ZD_K3_WN>
#define K3_ENTRY(e, k, al) k3f_entry(e, k, al)  // default: seq_chainfl, exact chain from HBM on a reject
constexpr int K3_TL = 512, K3_TM = 512, K3_TO = 256;
constexpr int K3_TAB = K3_TL + K3_TM + K3_TO;
static_assert(K3_LANES <= 64, "K3 workgroup must be a single wave");

// records (posA, stA), (posB, stB) as a pair (zd_common.h rec_pack) at p
__device__ inline void k3_store_pair(uint64_t* p, uint32_t posA, uint32_t stA, uint32_t posB, uint32_t stB) {
  uint32_t v[4];
  rec_pack(posA, stA, posB, stB, v);
  *(g_u32x4g*)p = u32x4g{v[0], v[1], v[2], v[3]};
}
// record i of a block (K3's pairs, zd_common.h, or a direct word)
__device__ inline uint64_t rec_get(const uint64_t* SQ, uint32_t i, bool direct) {
  if (direct) return SQ[i];
  const u32x4g v = *(const g_u32x4g*)(SQ + (i & ~1u));
  return rec_unpack(v.x, v.y, v.z, v.w, i & 1);
}
// record j of the block's pairs, read back after the chain stored it
__device__ inline uint64_t k3_reread(const uint64_t* out, uint32_t j) {
  const u32x4g v = *(volatile g_u32x4g*)(out + (j & ~1u));
  return rec_unpack(v.x, v.y, v.z, v.w, j & 1);
}

template <typename TP, bool K3_SYM>
__device__ int seq_chain2(const uint8_t* bs, uint32_t bs_size, uintptr_t base, TP tll, TP tml, TP tof, int all,
                          int alo, int alm, uint32_t n, uint64_t* __restrict__ out) {
  if (bs_size == 0) return ZD_E_EMPTY_INPUT_DATA;
  const uint8_t lastb = bs[bs_size - 1];
  if (lastb == 0) return ZD_E_NULL_BYTE;
  int32_t pos = (int32_t)(8 * (bs_size - 1)) + highbit32(lastb);
  const int32_t A = all + alo + alm;
  if (A > pos) return ZD_E_NOT_ENOUGH_BITS;
  const int32_t m = (int32_t)max((intptr_t)base - (intptr_t)bs, (intptr_t)-24);
  const int32_t pos0 = pos;
  const Win6 wi = win6_load(bs, m, pos);         // the init read
  const uint32_t v0 = win6_bits(wi, pos, (uint32_t)A);
  uint32_t sLL = v0 >> (alo + alm), sOF = __builtin_amdgcn_ubfe(v0, alm, alo), sML = __builtin_amdgcn_ubfe(v0, 0, alm);
  pos -= A;
  const uint32_t aL = all - 31, aM = alm - 31, aO = alo - 31;
  const uint32_t TL = 1u << all, TM = 1u << alm, TO = 1u << alo;
  // The loop entry sees the same memory-op order as its back edge (window,
  // store, window), so the wait for a window two steps old is not a drain:
  // step 0's window is loaded again for that.  Records are stored in pairs
  // (zd_common.h): the even step of an iteration stores (record i, record
  // i + 1), the odd one keeps its record for the next pair.
  Win6 wa = win6_load(bs, m, pos0);              // step 0 (covers pos0 - A - 90)
  asm volatile("" ::: "memory");
  uint32_t pPos = (uint32_t)pos, pSt = sLL | (sML << 10) | (sOF << 20);   // record 0
  k3_store_pair(out, pPos, pSt, pPos, pSt);
  Win6 wb = win6_load(bs, m, pos);               // step 1
  int st = 0;
  uint32_t i = 0;
  // one step reading window `use`, loading the window two steps ahead into
  // `use`.  Both steps of an iteration run on every lane (no branch between
  // them, so the loop entry keeps one memory-op order): a lane that finished
  // in the first keeps its status and leaves the pair it stored alone.
  auto step = [&](Win6& use, bool live, bool even) -> bool {
    uint32_t eLL = tll[sLL], eOF = tof[sOF], eML = tml[sML];
    if (K3_SYM) {
      eLL = k3_entry(eLL, 0);
      eOF = k3_entry(eOF, 1);
      eML = k3_entry(eML, 2);
    }
    const uint32_t nsL = eLL & 1023, nsM = eML & 1023, nsO = eOF & 1023;
    const uint32_t nbL = __builtin_clz(nsL) + aL, nbM = __builtin_clz(nsM) + aM, nbO = __builtin_clz(nsO) + aO;
    const uint32_t E = ((eLL >> 10) & 31) + ((eML >> 10) & 31) + ((eOF >> 10) & 31);
    const bool codemax = ((eLL | eML | eOF) & K3_BAD) != 0;
    const bool last = i + 1 >= n;
    const uint32_t S = last ? 0 : nbL + nbM + nbO;
    const int sst = codemax ? ZD_E_SEQUENCE_CODE_MAX_EXCEEDED : ((int32_t)(E + S) > pos ? ZD_E_NOT_ENOUGH_BITS : 0);
    st = live ? sst : st;
    const int32_t p2 = pos - (int32_t)E;
    const uint32_t v = win6_bits(use, p2, S);
    pos = p2 - (int32_t)S;
    use = win6_load(bs, m, pos);                   // for step i + 2
    const uint32_t vO = __builtin_amdgcn_ubfe(v, 0, nbO), vM = __builtin_amdgcn_ubfe(v, nbO, nbM);
    const uint32_t vL = v >> (nbO + nbM);
    sLL = (nsL << nbL) + vL - TL;
    sML = (nsM << nbM) + vM - TM;
    sOF = (nsO << nbO) + vO - TO;
    const uint32_t stw = sLL | (sML << 10) | (sOF << 20);   // record i + 1
    asm volatile("" ::: "memory");
    if (even) {
      k3_store_pair(out + i, pPos, pSt, (uint32_t)pos, stw);
    } else {
      pPos = (uint32_t)pos;
      pSt = stw;
    }
    i++;
    return !live || sst != 0 || last;
  };
  for (;;) {
    const bool d1 = step(wa, true, true);
    const bool d2 = step(wb, !d1, false);
    if (d2) break;
  }
  return st;
}

// N-dword bitstream window ending at the byte of pos (clamped to start at m).
template <int N>
struct WinN {
  uint32_t w[N];
  int32_t wb;
};
template <int N>
__device__ inline WinN<N> winn_load(const uint8_t* s, int32_t m, int32_t pos) {
  const int32_t o = max((pos + (7 - 32 * N)) >> 3, m);
  WinN<N> w;
#pragma unroll
  for (int k = 0; k + 4 <= N; k += 4) {
    const u32x4ua v = *(g_u32x4ua*)(s + o + 4 * k);
    w.w[k] = v.x; w.w[k + 1] = v.y; w.w[k + 2] = v.z; w.w[k + 3] = v.w;
  }
  if (N % 4 == 2) {
    const u32x2ua u = *(g_u32x2ua*)(s + o + 4 * (N - 2));
    w.w[N - 2] = u.x; w.w[N - 1] = u.y;
  }
  w.wb = o * 8;
  return w;
}
// 32 bits from bit y up (0 <= y <= 32 N; bits past the window read as zero)
template <int N>
__device__ inline uint32_t winn_at(const WinN<N>& w, uint32_t y) {
  // (a qword-then-dword select takes fewer instructions but a longer
  // dependent chain: 14.8 vs 13.8 ms for K3 on C4; a threshold tree, the
  // same 5 compares and 10 selects but 3 deep instead of 5: 5.63 -> 5.99 ms
  // on 4 GiB)
  uint32_t lo = w.w[0], hi = w.w[1];
#pragma unroll
  for (int i = 1; i < N; i++) {
    lo = y >= 32u * i ? w.w[i] : lo;
    hi = y >= 32u * i ? (i + 1 < N ? w.w[i + 1] : 0u) : hi;
  }
  return __builtin_amdgcn_alignbit(hi, lo, y & 31);
}

// winn_at by the three bits of the dword index (N = 6): three selects deep
// instead of five (few-chains regime: the step is the chain's latency)
template <int N>
__device__ inline uint32_t winn_at_tree(const WinN<N>& w, uint32_t y) {
  static_assert(N == 6 || N == 8, "tree select for 6- or 8-dword windows");
  const bool b0 = (y & 32) != 0, b1 = (y & 64) != 0, b2 = y >= 128;
  const uint32_t l01 = b0 ? w.w[1] : w.w[0], l23 = b0 ? w.w[3] : w.w[2], l45 = b0 ? w.w[5] : w.w[4];
  const uint32_t h01 = b0 ? w.w[2] : w.w[1], h23 = b0 ? w.w[4] : w.w[3];
  uint32_t lo, hi;
  if constexpr (N == 6) {
    const uint32_t h45 = b0 ? 0u : w.w[5];
    lo = b2 ? l45 : (b1 ? l23 : l01);
    hi = b2 ? h45 : (b1 ? h23 : h01);
  } else {
    const uint32_t l67 = b0 ? w.w[7] : w.w[6];
    const uint32_t h45 = b0 ? w.w[6] : w.w[5], h67 = b0 ? 0u : w.w[7];
    lo = b2 ? (b1 ? l67 : l45) : (b1 ? l23 : l01);
    hi = b2 ? (b1 ? h67 : h45) : (b1 ? h23 : h01);
  }
  return __builtin_amdgcn_alignbit(hi, lo, y & 31);
}

// The fast chain: no checks inside the loop.  Each table gives nextState and
// the step's total bit count for that table (k3f_entry), so a step is
// pos -= tLL + tML + tOF, then the LL | ML | OF state bits are the low bits
// at the new position.  Steps 0 .. n-2 update the states (a lane whose count
// runs past n-1 stores into the spare slots); the epilogue re-reads record
// n-1 and checks the last step (extra bits only, sequences.rs:223-229).
// Windows are loaded L steps ahead (a ring of L): a 4N-byte window ending at
// the byte of pos_{i+1} covers steps i+1..i+L when they read <= 32 N - 7
// bits together (text: ~35 bits a step).  Anything the reference would
// reject -- a code above the maximum anywhere (K3F_BAD), the position going
// negative before the last step, the last step's extra bits running out --
// or a window that did not cover its step (ymin < 0), and the block is
// decoded again by the exact chain, which finds the reference's error.  U
// steps per trip, records stored in pairs; a pair past the block's last
// record goes to its two spare slots (host: seq_out).  Returns 1 when the
// block needs the exact chain, else 0.
template <int L, int N>
__device__ int seq_chainfl(const uint8_t* bs, uint32_t bs_size, uintptr_t base, const lds_u16* tll,
                           const lds_u16* tml, const lds_u16* tof, int all, int alo, int alm, uint32_t n,
                           uint64_t* __restrict__ out) {
  constexpr int U = (L % 2 == 0) ? L : 2 * L;
  static_assert(N % 4 == 0 || N % 4 == 2, "window: dwordx4 pieces and one dwordx2");
  if (bs_size == 0) return 1;
  const uint8_t lastb = bs[bs_size - 1];
  if (lastb == 0) return 1;
  int32_t pos = (int32_t)(8 * (bs_size - 1)) + highbit32(lastb);
  const int32_t A = all + alo + alm;
  if (A > pos) return 1;
  // windows never start below the input nor end past the stream's block
  if ((intptr_t)bs - (intptr_t)base + (intptr_t)bs_size < 4 * N) return 1;
  const int32_t m = (int32_t)max((intptr_t)base - (intptr_t)bs, (intptr_t)(-4 * N));
  const int32_t pos0 = pos;
  const Win6 wi = win6_load(bs, m, pos);
  const uint32_t v0 = win6_bits(wi, pos, (uint32_t)A);
  uint32_t sLL = v0 >> (alo + alm), sOF = __builtin_amdgcn_ubfe(v0, alm, alo), sML = __builtin_amdgcn_ubfe(v0, 0, alm);
  pos -= A;
  const uint32_t aL = all - 31, aM = alm - 31, aO = alo - 31;
  const uint32_t TL = 1u << all, TM = 1u << alm, TO = 1u << alo;
  // record 0, then the pairs: an even step stores (record i, record i + 1),
  // an odd step keeps its record for the next pair.  Loop entry: the trip's
  // memory-op order (window, store, window, window, store, ...)
  uint32_t pPos = (uint32_t)pos, pSt = sLL | (sML << 10) | (sOF << 20);
  const uint32_t n_even = (n + 1) & ~1u;              // the spare pair
  WinN<N> w[L];
#pragma unroll
  for (int k = 0; k < L; k++) {
    w[k] = winn_load<N>(bs, m, k == 0 ? pos0 : pos);
    if (!(k & 1)) {
      asm volatile("" ::: "memory");
      k3_store_pair(out, pPos, pSt, pPos, pSt);
    }
  }
  uint32_t mx = 0;
  int32_t ymin = 0;
  // (forming the next LDS addresses as (ns << nb + 1) + const + 2 v, one add
  // nearer the state bits, measured slower: 14.9 vs 13.8 ms)
  auto step = [&](WinN<N>& use) -> uint32_t {
    const uint32_t eLL = tll[sLL], eOF = tof[sOF], eML = tml[sML];
    mx = max(mx, max(eLL, max(eML, eOF)));
    const uint32_t nsL = eLL & 1023, nsM = eML & 1023, nsO = eOF & 1023;
    const uint32_t nbL = __builtin_clz(nsL) + aL, nbM = __builtin_clz(nsM) + aM, nbO = __builtin_clz(nsO) + aO;
    pos -= (int32_t)((eLL >> 10) + (eML >> 10) + (eOF >> 10));
    const int32_t y = pos - use.wb;
    ymin = min(ymin, y);
    const uint32_t r = winn_at<N>(use, (uint32_t)y);
    use = winn_load<N>(bs, m, pos);                // for the step L on
    const uint32_t vO = __builtin_amdgcn_ubfe(r, 0, nbO), vM = __builtin_amdgcn_ubfe(r, nbO, nbM);
    const uint32_t vL = __builtin_amdgcn_ubfe(r, nbO + nbM, nbL);
    sLL = (nsL << nbL) + vL - TL;
    sML = (nsM << nbM) + vM - TM;
    sOF = (nsO << nbO) + vO - TO;
    return sLL | (sML << 10) | (sOF << 20);
  };
  uint32_t i = 0;
  for (; i + 1 < n; i += U) {
#pragma unroll
    for (int k = 0; k < U; k += 2) {
      const uint32_t sa = step(w[k % L]);
      asm volatile("" ::: "memory");
      const uint32_t slot = i + k;                  // pair (i + k, i + k + 1)
      k3_store_pair(out + (slot < n ? slot : n_even), pPos, pSt, (uint32_t)pos, sa);
      pSt = step(w[(k + 1) % L]);
      pPos = (uint32_t)pos;
    }
  }
  // the record the last trip kept (record i): the block's last when n - 1 == i
  k3_store_pair(out + (i < n ? i : n_even), pPos, pSt, pPos, pSt);
  const uint64_t rl = k3_reread(out, n - 1);
  const int32_t pl = (int32_t)(uint32_t)rl;
  const uint32_t st = (uint32_t)(rl >> 32);
  const uint32_t eLL = tll[st & 1023], eML = tml[(st >> 10) & 1023], eOF = tof[(st >> 20) & 1023];
  mx = max(mx, max(eLL, max(eML, eOF)));
  const uint32_t S = (__builtin_clz(eLL & 1023) + aL) + (__builtin_clz(eML & 1023) + aM) + (__builtin_clz(eOF & 1023) + aO);
  const int32_t E = (int32_t)((eLL >> 10) + (eML >> 10) + (eOF >> 10) - S);
  return (mx >= K3F_BAD || ymin < 0 || pl < 0 || E > pl) ? 1 : 0;
}

__device__ inline void k3_fail(const CompBlock& C, uint32_t ci, CompState* cstate, FrameState* fstate, int st) {
  key_min(fstate, C.frame, make_key(PH_DECODE, C.block_in_frame, DS_SEQUENCES, 0, st));
  cstate[ci].stop = 1;
}

__global__ __launch_bounds__(K3_LANES) void zd_k_sequences(const uint8_t* __restrict__ src,
                                                           const CompBlock* __restrict__ comp, CompState* cstate,
                                                           FrameState* fstate, const uint32_t* __restrict__ list,
                                                           uint32_t n_list, const uint16_t* __restrict__ fses,
                                                           uint64_t* __restrict__ recs) {
  __shared__ __attribute__((aligned(16))) uint16_t tabs[K3_LANES * K3_TAB];
  const int lane = threadIdx.x;
  const uint32_t li = blockIdx.x * K3_LANES + lane;
  bool act = li < n_list;
  const uint32_t ci = act ? list[li] : 0;
  CompBlock C;
  if (act) C = comp[ci];
  if (act) {
    const uint64_t key0 = fstate[C.frame].key;
    if (key0 != KEY_NONE && key_phase(key0) == PH_PARSE) act = false;
  }
  int al[3] = {0, 0, 0};
  const uint16_t* g[3] = {nullptr, nullptr, nullptr};
  if (act) {
    for (int k = 0; k < 3; k++) {
      const uint32_t s = (uint32_t)C.tab_src[k];
      al[k] = cstate[s].al[k];
      g[k] = fses + (uint64_t)comp[s].fse_slot * FSE_SLOT + k * FSE_TAB;
    }
  }
  // tables -> LDS in the chain format (every lane its own three), unless
  // some lane needs AL 9 offsets
  const bool deep = act && al[1] > 8;
  const bool use_lds = __ballot(deep) == 0;      // the workgroup is one wave
  lds_u16* mine = (lds_u16*)tabs + lane * K3_TAB;
  if (use_lds && act) {
    const int dst[3] = {0, K3_TL + K3_TM, K3_TL};     // LL | ML | OF in LDS
    for (int k = 0; k < 3; k++) {
      const int cnt = 1 << al[k];
      if (cnt >= 8) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) const u32x4 g_u4;
        typedef __attribute__((address_space(3))) u32x4 l_u4;
        g_u4* s4 = (g_u4*)g[k];
        l_u4* d4 = (l_u4*)(mine + dst[k]);
        for (int e = 0; e < cnt / 8; e++) {
          u32x4 v = s4[e];
          v.x = K3_ENTRY(v.x & 0xFFFF, k, al[k]) | (K3_ENTRY(v.x >> 16, k, al[k]) << 16);
          v.y = K3_ENTRY(v.y & 0xFFFF, k, al[k]) | (K3_ENTRY(v.y >> 16, k, al[k]) << 16);
          v.z = K3_ENTRY(v.z & 0xFFFF, k, al[k]) | (K3_ENTRY(v.z >> 16, k, al[k]) << 16);
          v.w = K3_ENTRY(v.w & 0xFFFF, k, al[k]) | (K3_ENTRY(v.w >> 16, k, al[k]) << 16);
          d4[e] = v;
        }
      } else {
        for (int e = 0; e < cnt; e++) mine[dst[k] + e] = (uint16_t)K3_ENTRY(((g_u16*)g[k])[e], k, al[k]);
      }
    }
  }
  __syncthreads();
  if (!act) return;
  const CompState cs = cstate[ci];
  const uint8_t* blk = src + C.src;
  const uintptr_t lo = (uintptr_t)src;
  int st = 0;
  bool exact = !use_lds;
  if (use_lds)
    exact = K3_FAST(blk + cs.bs_off, cs.bs_size, lo, mine, mine + K3_TL, mine + K3_TL + K3_TM, al[0], al[1],
                       al[2], C.nseq, recs + C.seq_out) != 0;
  if (exact)
    st = K3_CHAIN<g_u16*, true>(blk + cs.bs_off, cs.bs_size, lo, (g_u16*)g[0], (g_u16*)g[2], (g_u16*)g[1], al[0],
                                 al[1], al[2], C.nseq, recs + C.seq_out);
  if (st) k3_fail(C, ci, cstate, fstate, st);
}
// ---------------------------------------------------------------------------
// K3Q: the fast chain with four lanes per block (a quad): lane roles OF, ML,
// LL and a dummy, each with its own table, state and bit count, so a step is
// one table lookup per lane instead of three per lane; the three counts are
// summed and the state bits split with quad DPP moves, the window select is
// the same in all four lanes.  Records, checks and the exact-chain fallback
// are seq_chainfl's (same records bit for bit).  The fourth lane shadows the
// LL lane (its table, its states stay valid indices) and is masked out of
// the sums, the bit split and the record (LDS is full: no room for a dummy
// table next to four workgroups' 40 KiB of tables).
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ inline uint32_t qdpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
}
constexpr int QP_SWAP1 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int QP_SWAP2 = 0x4E;   // quad_perm [2,3,0,1]
__device__ inline uint32_t quad_sum(uint32_t x) {
  x += qdpp<QP_SWAP1>(x);
  return x + qdpp<QP_SWAP2>(x);
}
__device__ inline uint32_t quad_or(uint32_t x) {
  x |= qdpp<QP_SWAP1>(x);
  return x | qdpp<QP_SWAP2>(x);
}
__device__ inline uint32_t quad_max(uint32_t x) {
  x = max(x, qdpp<QP_SWAP1>(x));
  return max(x, qdpp<QP_SWAP2>(x));
}
// PUB (zd_k_fused): every 16 records the chain publishes to *prog the
// 16-record lines of `out` whose stores have completed (a line eight pairs
// back: vmcnt(32) leaves the newer window loads and stores in flight), for
// the K4 wave of its workgroup.
template <int L, int N, bool PUB = false>
__device__ int seq_chainq(const uint8_t* bs, uint32_t bs_size, uintptr_t base, const lds_u16* tab, int role,
                          int all, int alo, int alm, uint32_t n, uint64_t* __restrict__ out,
                          volatile __attribute__((address_space(3))) uint32_t* prog = nullptr) {
  constexpr int U = (L % 2 == 0) ? L : 2 * L;
  if (bs_size == 0) return 1;
  const uint8_t lastb = bs[bs_size - 1];
  if (lastb == 0) return 1;
  int32_t pos = (int32_t)(8 * (bs_size - 1)) + highbit32(lastb);
  const int32_t A = all + alo + alm;
  if (A > pos) return 1;
  if ((intptr_t)bs - (intptr_t)base + (intptr_t)bs_size < 4 * N) return 1;
  const int32_t m = (int32_t)max((intptr_t)base - (intptr_t)bs, (intptr_t)(-4 * N));
  const int32_t pos0 = pos;
  const Win6 wi = win6_load(bs, m, pos);
  const uint32_t v0 = win6_bits(wi, pos, (uint32_t)A);
  // this lane's role: OF (0) | ML (1) | LL (2) | LL's shadow (3: the LL
  // table and the LL lane's bit offsets, so it tracks the LL state exactly;
  // masked out of the count sums by m3)
  const int alr = role == 0 ? alo : role == 1 ? alm : all;
  const uint32_t m3 = role == 3 ? 0u : ~0u, m0 = role == 0 ? 0u : ~0u;
  const uint32_t ar = (uint32_t)(alr - 31), Tr = 1u << alr;
  uint32_t s = role == 0 ? __builtin_amdgcn_ubfe(v0, alm, alo)
             : role == 1 ? __builtin_amdgcn_ubfe(v0, 0, alm)
             : v0 >> (alo + alm);
  pos -= A;
  // Records in pairs (zd_common.h), one dword per lane and no cross-lane
  // moves: OF lane x (its two states and the position step), ML lane y, LL
  // lane z, shadow w (the pair's first position).  An even step stores the
  // pair (record i, record i + 1), an odd one keeps its record.
  uint32_t pS = s, pPos = (uint32_t)pos;
  auto pair_word = [&](uint32_t sB, uint32_t posB) -> uint32_t {
    const uint32_t d = pS | (sB << 10);
    const uint32_t x = d | ((pPos - posB) << 20);
    return role == 3 ? pPos : (role == 0 ? x : d);
  };
  g_u32* const outw = (g_u32*)out + role;
  const uint32_t n_even = (n + 1) & ~1u;              // the spare pair
  // loop entry: the trip's memory-op order (window, store, window, window, store, ...)
  WinN<N> w[L];
#pragma unroll
  for (int k = 0; k < L; k++) {
    w[k] = winn_load<N>(bs, m, k == 0 ? pos0 : pos);
    if (!(k & 1)) {
      asm volatile("" ::: "memory");
      outw[0] = pair_word(s, (uint32_t)pos);
    }
  }
  uint32_t mx = 0;
  int32_t ymin = 0;
  auto step = [&](WinN<N>& use) {
    const uint32_t e = tab[s];
    mx = max(mx, e);                                // (the shadow lane's e is the LL lane's)
    const uint32_t ns = e & 1023, nb = __builtin_clz(ns) + ar;
    // the three roles' counts by three quad broadcasts and one add3 (the
    // shadow lane's count never enters), y from the position before the step
    // (C3 K3 2.31 -> 2.22 ms)
    const uint32_t c = e >> 10;
    const uint32_t csum = qdpp<0x00>(c) + qdpp<0x55>(c) + qdpp<0xAA>(c);
    const int32_t y = (pos - use.wb) - (int32_t)csum;
    pos -= (int32_t)csum;
    ymin = min(ymin, y);
    const uint32_t r = winn_at_tree<N>(use, (uint32_t)y);   // (linear select: C3 K3 2.21 ms, tree 2.06)
    use = winn_load<N>(bs, m, pos);
    // the state bits sit OF | ML | LL upwards from y: offsets 0, nbO, nbO +
    // nbM (the shadow takes the LL lane's), by quad_perm [0,0,1,1] twice
    const uint32_t t = qdpp<0x50>(nb) & m0;
    const uint32_t v = __builtin_amdgcn_ubfe(r, t + qdpp<0x50>(t), nb);
    s = (ns << nb) + v - Tr;   // (the next address formed from v in one op: 2.07 -> 2.11 ms on C3)
  };
  uint32_t i = 0;
  // a trip runs while i + 1 < n, so with U = 4 its pairs i, i + 2 are <= n,
  // and a pair at n (n even) is the spare pair: the pair stores walk a pointer
  g_u32* wp = outw;
  for (; i + 1 < n; i += U) {
#pragma unroll
    for (int k = 0; k < U; k += 2) {
      step(w[k % L]);
      asm volatile("" ::: "memory");
      const uint32_t slot = i + k;                  // pair (i + k, i + k + 1)
      if constexpr (U == 4) {
        *wp = pair_word(s, (uint32_t)pos);
        wp += 4;
      } else {
        outw[2 * (slot < n ? slot : n_even)] = pair_word(s, (uint32_t)pos);
      }
      if constexpr (PUB) {
        // The line published here ends with pair slot - 14, seven pairs back;
        // each pair since issued K3_PAIR_VMEM vector-memory ops (two window
        // loads of N / 4 dwordx4 (+ one dwordx2) each, one store), so
        // vmcnt(32) has drained that store only when 7 pairs issue more than
        // 32 ops (N = 6 or 8: 35; N = 4 would leave it in flight)
        constexpr int K3_PAIR_VMEM = 2 * (N / 4 + (N % 4 == 2 ? 1 : 0)) + 1;
        static_assert(7 * K3_PAIR_VMEM > 32, "seq_chainq PUB: vmcnt(32) would not cover the published line's stores");
        if (((slot + 2) & 15) == 0 && slot + 2 >= 32) {
          asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
          if (role == 0) *prog = (slot + 2 - 16) >> 4;
        }
      }
      step(w[(k + 1) % L]);
      pS = s;
      pPos = (uint32_t)pos;
    }
  }
  // the record the last trip kept (record i): the block's last when n - 1 == i
  outw[2 * (i < n ? i : n_even)] = pair_word(pS, pPos);
  const uint64_t rl = k3_reread(out, n - 1);
  const int32_t pl = (int32_t)(uint32_t)rl;
  const uint32_t st = (uint32_t)(rl >> 32);
  const uint32_t shr = role == 0 ? 20 : role == 1 ? 10 : 0;
  const uint32_t el = tab[(st >> shr) & 1023] & m3;
  mx = quad_max(max(mx, el));
  const uint32_t S = quad_sum((__builtin_clz(el & 1023) + ar) & m3);
  const int32_t E = (int32_t)(quad_sum(el >> 10) - S);
  return (mx >= K3F_BAD || ymin < 0 || pl < 0 || E > pl) ? 1 : 0;
}

#ifndef ZD_K3Q_CHAINS
#define ZD_K3Q_CHAINS 16
#endif
constexpr int K3Q_CHAINS = ZD_K3Q_CHAINS;   // blocks per workgroup (one wave, four lanes each)
static_assert(K3Q_CHAINS == 8 || K3Q_CHAINS == 16, "K3Q: 8 or 16 chains per wave");
__global__ __launch_bounds__(64) void zd_k_sequences_q(const uint8_t* __restrict__ src,
                                                       const CompBlock* __restrict__ comp, CompState* cstate,
                                                       FrameState* fstate, const uint32_t* __restrict__ list,
                                                       uint32_t n_list, const uint16_t* __restrict__ fses,
                                                       uint64_t* __restrict__ recs, const uint8_t* __restrict__ redo) {
  __shared__ __attribute__((aligned(16))) uint16_t tabs[K3Q_CHAINS * K3_TAB];
  const int lane = threadIdx.x;
  const int role = lane & 3, q = lane >> 2;
  const uint32_t li = blockIdx.x * K3Q_CHAINS + q;
  bool act = q < K3Q_CHAINS && li < n_list;
  const uint32_t ci = act ? list[li] : 0;
  CompBlock C;
  if (act) C = comp[ci];
  if (act && redo && !redo[C.frame]) act = false;   // the redo pass after zd_k_fused: flagged frames only
  if (act) {
    const uint64_t key0 = fstate[C.frame].key;
    if (key0 != KEY_NONE && key_phase(key0) == PH_PARSE) act = false;
  }
  int al[3] = {0, 0, 0};
  const uint16_t* g[3] = {nullptr, nullptr, nullptr};
  if (act) {
    for (int k = 0; k < 3; k++) {
      const uint32_t sidx = (uint32_t)C.tab_src[k];
      al[k] = cstate[sidx].al[k];
      g[k] = fses + (uint64_t)comp[sidx].fse_slot * FSE_SLOT + k * FSE_TAB;
    }
  }
  const bool deep = act && al[1] > 8;
  const bool use_lds = __ballot(deep) == 0;
  lds_u16* mine = (lds_u16*)tabs + q * K3_TAB;
  if (use_lds && act) {
    // the quad's lanes fill the three tables (lane k < 3: table k)
    const int dst[3] = {0, K3_TL + K3_TM, K3_TL};     // LL | ML | OF in LDS
    if (role < 3) {
      const int k = role;
      const int cnt = 1 << al[k];
      if (cnt >= 8) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) const u32x4 g_u4;
        typedef __attribute__((address_space(3))) u32x4 l_u4;
        g_u4* s4 = (g_u4*)g[k];
        l_u4* d4 = (l_u4*)(mine + dst[k]);
        for (int e = 0; e < cnt / 8; e++) {
          u32x4 v = s4[e];
          v.x = K3_ENTRY(v.x & 0xFFFF, k, al[k]) | (K3_ENTRY(v.x >> 16, k, al[k]) << 16);
          v.y = K3_ENTRY(v.y & 0xFFFF, k, al[k]) | (K3_ENTRY(v.y >> 16, k, al[k]) << 16);
          v.z = K3_ENTRY(v.z & 0xFFFF, k, al[k]) | (K3_ENTRY(v.z >> 16, k, al[k]) << 16);
          v.w = K3_ENTRY(v.w & 0xFFFF, k, al[k]) | (K3_ENTRY(v.w >> 16, k, al[k]) << 16);
          d4[e] = v;
        }
      } else {
        for (int e = 0; e < cnt; e++) mine[dst[k] + e] = (uint16_t)K3_ENTRY(((g_u16*)g[k])[e], k, al[k]);
      }
    }
  }
  __syncthreads();
  if (!act) return;
  const CompState cs = cstate[ci];
  const uint8_t* blk = src + C.src;
  const uintptr_t lo = (uintptr_t)src;
  int st = 0;
  bool exact = !use_lds;
  if (use_lds) {
    const lds_u16* tab = role == 0 ? mine + K3_TL + K3_TM : role == 1 ? mine + K3_TL : mine;
    exact = seq_chainq<ZD_K3_LA, ZD_K3_WN>(blk + cs.bs_off, cs.bs_size, lo, tab, role, al[0], al[1], al[2], C.nseq,
                                          recs + C.seq_out) != 0;
  }
  if (exact && role == 0)
    st = K3_CHAIN<g_u16*, true>(blk + cs.bs_off, cs.bs_size, lo, (g_u16*)g[0], (g_u16*)g[2], (g_u16*)g[1], al[0],
                                 al[1], al[2], C.nseq, recs + C.seq_out);
  if (st) k3_fail(C, ci, cstate, fstate, st);
}
// ---------------------------------------------------------------------------
// K3L: the latency-first FSE chain, for plans of few blocks (C3, the single
// 100 MB frame), where a K3Q wave's 16 chains all run alone on their SIMD and
// a step costs what one wave issues for it (~54 instructions at 4 cycles).
// One block per wave, every lane running the same chain (wave-uniform): the
// bit position lives in an SGPR, the bitstream window is spread over the
// wave's lanes (lane L holds dword D + L of the stream; the 64 bits under the
// position come by two v_readlane, no select tree and no per-step load), and
// each LDS table entry is 64 bits: lo = nb | (extra + nb) << 8 | bad << 16
// (nb in the low 5 bits, so it is the bfe width as it stands, and the sum of
// the OF and ML entries is the LL state bits' offset), hi = the LDS address
// of the next state's baseline (table + 8 x baseline), so a new state is one
// shift-add.  The three lookups go out together, one wait.  Records are K3Q's
// pairs, bit for bit (zd_common.h rec_pack): the states come back from the
// addresses (LL at byte 0, ML at 4096, OF at 8192 of a 4 KiB-aligned table
// block: state = address >> 3 & 511).  Rejects as seq_chainq: a code above
// the maximum anywhere, the position going negative, the last step's extra
// bits running out -- the block then goes to the exact chain.
// ---------------------------------------------------------------------------
constexpr uint32_t K3L_ML = 4096, K3L_OF = 8192, K3L_BYTES = 10240;   // LL at 0
#ifndef ZD_K3L_ASM
#define ZD_K3L_ASM 1                    // the step's count sum and 64-bit funnel as one op each
#endif
#ifndef ZD_K3L_SHADOW
#define ZD_K3L_SHADOW 1                 // pair formatting behind the next step's table reads
#endif
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ inline uint64_t k3l_entry(uint32_t e, int k, int al, uint32_t tab) {
  const uint32_t c = e & 63, ns = (e >> 6) & 1023;
  uint32_t base, eb;
  bool bad;
  if (k == 0) { ll_code(c, &base, &eb); bad = c > 35; }
  else if (k == 2) { ml_code(c, &base, &eb); bad = c > 52; }
  else { eb = c; bad = c > 31; }
  bad = bad || ns == 0 || hb32(ns) > al;
  const uint32_t nb = bad ? 0u : (uint32_t)(al - hb32(ns));
  const uint32_t bl = bad ? 0u : (ns << nb) - (1u << al);
  const uint32_t lo = bad ? (1u << 16) : (nb | ((eb + nb) << 8));     // a bad entry moves nothing
  return (uint64_t)lo | ((uint64_t)(tab + 8 * bl) << 32);
}
// The block's three tables (fses slots, k = 0 LL, 1 OF, 2 ML) as K3L entries
// at LDS byte address tb (4 KiB-aligned), all 64 lanes.
__device__ inline void k3l_tables(const uint16_t* __restrict__ fses, const CompBlock& C, const CompBlock* __restrict__ comp,
                                  const CompState* __restrict__ cstate, uint32_t tb, int al[3], int lane) {
  for (int k = 0; k < 3; k++) {
    const uint32_t s = (uint32_t)C.tab_src[k];
    al[k] = cstate[s].al[k];
    const uint16_t* g = fses + (uint64_t)comp[s].fse_slot * FSE_SLOT + k * FSE_TAB;
    const uint32_t t = tb + (k == 0 ? 0u : k == 2 ? K3L_ML : K3L_OF);
    const int cnt = 1 << min(al[k], k == 1 ? 8 : 9);
    for (int e = lane; e < cnt; e += 64) *(lds_u64*)(uintptr_t)(t + 8 * e) = k3l_entry(g[e], k, al[k], t);
  }
}
// PUB (zd_k_fused): after every 16 records the chain publishes to *prog the
// 16-record lines whose stores have completed (the line eight pairs back).
template <bool PUB = false>
__device__ int seq_chainl(const uint8_t* bs, uint32_t bs_size, uintptr_t base, uint32_t tb, int all, int alo, int alm,
                          uint32_t n, uint64_t* __restrict__ out, volatile lds_u32* prog = nullptr) {
  const int lane = threadIdx.x & 63;
  if (bs_size == 0 || (tb & 4095) || alo > 8) return 1;
  const uint8_t lastb = bs[bs_size - 1];
  if (lastb == 0) return 1;
  int32_t pos = (int32_t)(8 * (bs_size - 1)) + highbit32(lastb);   // bits above bs
  const int32_t A = all + alo + alm;
  if (A > pos) return 1;
  // positions and window dwords relative to the dword-aligned address at or below bs
  const uint8_t* bsa = (const uint8_t*)((uintptr_t)bs & ~(uintptr_t)3);
  const int32_t boff = (int32_t)(((uintptr_t)bs & 3) * 8);
  const uint64_t below = ((uintptr_t)bsa - (base & ~(uintptr_t)3)) >> 2;   // dwords of input below bsa
  const int32_t dmin = below > (1u << 30) ? -(1 << 30) : -(int32_t)below;
  auto wload = [&](int32_t D) -> uint32_t {
    const int32_t d = max(D + lane, dmin);
    return *(const g_u32*)(bsa + 4 * (int64_t)d);
  };
  // the window: dwords [D, D + 64) of the stream, one per lane; Q = the
  // position relative to dword D (the chain's one running number: the step
  // subtracts its bit count from it, its dword is lane Q >> 5), pos = Q + qb
  int32_t D = ((pos + boff) >> 5) - 62;
  int32_t Q = pos + boff - 32 * D;
  int32_t qb = 32 * D - boff;
  // win1: the window moved down one lane (lane L holds dword D + L + 1), so
  // both dwords under a position come by readlane at one lane index
  auto shl1 = [](uint32_t w) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w, 0x130, 0xf, 0xf, false); };
  uint32_t win = wload(D);
  uint32_t win1 = shl1(win);
  uint32_t nxt;
  // (Q stays in a VGPR: an SGPR that the VALU writes (v_readfirstlane,
  // v_readlane) costs ~20 cycles when the SALU reads it, ~0 when the VALU
  // does, profiles/r6_salu_bench.txt -- so the lane index is the only
  // crossing, and the 64-bit funnel shift is one VALU op on the SGPR pair)
  auto bits32 = [&](int32_t q) -> uint32_t {  // 32 bits from window bit q up
    // (the shift stays on the VALU: left to the compiler it moved it past the
    // v_readfirstlane onto the SALU, one crossing more on the chain)
    int32_t qd;
    asm("v_ashrrev_i32 %0, 5, %1" : "=v"(qd) : "v"(q));
    const int idx = __builtin_amdgcn_readfirstlane(qd);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)win, idx);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)win1, idx);
#if ZD_K3L_ASM
    // one 64-bit shift of the SGPR pair (the shift count, q & 31, is off the
    // path), where the compiler moved lo to a VGPR and used v_alignbit
    uint64_t r;
    asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "v"((uint32_t)q & 31u), "s"(((uint64_t)hi << 32) | lo));
    return (uint32_t)r;
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (q & 31));
#endif
  };
  const uint32_t v0 = bits32(Q - A) & (uint32_t)((1ull << A) - 1);
  uint32_t aL = tb + 8 * (v0 >> (alo + alm));
  uint32_t aO = tb + K3L_OF + 8 * __builtin_amdgcn_ubfe(v0, alm, alo);
  uint32_t aM = tb + K3L_ML + 8 * __builtin_amdgcn_ubfe(v0, 0, alm);
  Q -= A;
  uint32_t bad = 0;
#ifdef ZD_K3L_PROF
  const uint64_t tp0 = __builtin_amdgcn_s_memtime();
  const uint64_t rp0 = __builtin_amdgcn_s_memrealtime();
#endif
  auto lshl3_add = [](uint32_t v, uint32_t b) -> uint32_t {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(r) : "v"(v), "v"(b));
    return r;
  };
  uint64_t eL, eM, eO;
  auto issue = [&]() {                         // the step's three table reads
    eL = *(const lds_u64*)(uintptr_t)aL;
    eM = *(const lds_u64*)(uintptr_t)aM;
    eO = *(const lds_u64*)(uintptr_t)aO;
  };
  auto finish = [&]() {
    const uint32_t lL = (uint32_t)eL, lM = (uint32_t)eM, lO = (uint32_t)eO;
    const uint32_t lOM = lO + lM;              // (its low 5 bits: the LL state bits' offset)
#if ZD_K3L_ASM
    uint32_t ls;                               // one add on the path, not two
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(ls) : "v"(lO), "v"(lM), "v"(lL));
#else
    const uint32_t ls = lOM + lL;
#endif
    bad |= ls;
    Q -= (ls >> 8) & 255;
    const uint32_t r = bits32(Q);
    const uint32_t vO = __builtin_amdgcn_ubfe(r, 0, lO), vM = __builtin_amdgcn_ubfe(r, lO, lM);
    const uint32_t vL = __builtin_amdgcn_ubfe(r, lOM, lL);
    aO = lshl3_add(vO, (uint32_t)(eO >> 32));
    aM = lshl3_add(vM, (uint32_t)(eM >> 32));
    aL = lshl3_add(vL, (uint32_t)(eL >> 32));
  };
  auto step = [&]() { issue(); finish(); };
  // a record's state field: the address's index bits (tables 4 KiB-aligned)
  auto sx = [](uint32_t a) { return __builtin_amdgcn_ubfe(a, 3, 9); };
  // pair (record A, record B) in K3Q's words
  auto put = [&](uint64_t* p, uint32_t pA, uint32_t lA, uint32_t mA, uint32_t oA, uint32_t pB, uint32_t lB, uint32_t mB,
                 uint32_t oB) {
#ifdef ZD_EXP_K3L_RAWPUT
    // timing only (with ZD_K3L_PROF): each record stored as it stands, no
    // formatting (both into the pair's slot); the chain then rejects, and the
    // exact chain writes the records
    *(g_u32x4g*)p = u32x4g{oA, mA, lA, pA};
    asm volatile("" ::: "memory");
    *(g_u32x4g*)p = u32x4g{oB, mB, lB, pB};
#else
    const u32x4g v{sx(oA) | (sx(oB) << 10) | ((pA - pB) << 20), sx(mA) | (sx(mB) << 10), sx(lA) | (sx(lB) << 10), pA};
    *(g_u32x4g*)p = v;
#endif
  };
  const uint32_t n_even = (n + 1) & ~1u;       // the spare pair
  uint32_t pP = (uint32_t)(Q + qb), pL = aL, pM = aM, pO = aO;   // record i, kept for its pair
  uint32_t i = 0;
  // a trip runs while i + 1 < n, so its pairs i, i + 2 are <= n, and a pair
  // at n (n even) is the spare pair: the pair stores walk a pointer
  uint64_t* wp = out;
  // per window: the next one loads while this one's trips run (a trip's four
  // steps read <= 4 x 89 bits below the position: 12 dwords), and becomes
  // the window when fewer than 13 dwords are left below the position
  while (i + 1 < n) {
  if (__builtin_amdgcn_readfirstlane(Q >> 5) < 13) {
    D -= 48;
    Q += 48 * 32;
    qb -= 48 * 32;
    win = nxt;
    win1 = shl1(win);
  }
  nxt = wload(D - 48);
  do {
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
      step();
#if ZD_K3L_SHADOW
      // the pair (i + k, i + k + 1) is formatted and stored while the next
      // step's table reads are in flight: the asm keeps its operands (and so
      // the formatting) behind those reads, where the compiler otherwise put
      // up to eight of its VALU ops ahead of them, on the chain's path
      uint32_t cP = (uint32_t)(Q + qb), cL = aL, cM = aM, cO = aO;
      issue();
      asm volatile("" : "+v"(pP), "+v"(pL), "+v"(pM), "+v"(pO), "+v"(cP), "+v"(cL), "+v"(cM), "+v"(cO) :: "memory");
      put(wp, pP, pL, pM, pO, cP, cL, cM, cO);
      wp += 2;
      finish();
#else
      put(wp, pP, pL, pM, pO, (uint32_t)(Q + qb), aL, aM, aO);   // pair (i + k, i + k + 1)
      wp += 2;
      step();
#endif
      pP = (uint32_t)(Q + qb); pL = aL; pM = aM; pO = aO;
    }
    i += 4;
    if constexpr (PUB) {
      // every 16 records: the lines up to the one that ended 16 records ago,
      // whose stores are older than the newest eight vector-memory ops (the
      // eight pair stores since, and at most one window load)
      if ((i & 15) == 0 && i >= 32) {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        if (lane == 0) *prog = (i - 16) >> 4;
      }
    }
  } while (i + 1 < n && __builtin_amdgcn_readfirstlane(Q >> 5) >= 13);
  }
  // the record the last trip kept (record i): the block's last when n - 1 == i
  put(out + (i < n ? i : n_even), pP, pL, pM, pO, pP, pL, pM, pO);
#ifdef ZD_K3L_PROF
  {
    const uint64_t tp1 = __builtin_amdgcn_s_memtime(), rp1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && blockIdx.x < 4)
      printf("K3L block %u: %u steps, %.1f memtime ticks a step, %.1f ns a step (memrealtime 100 MHz)\n", blockIdx.x, i,
             (double)(tp1 - tp0) / (double)max(i, 1u), 10.0 * (double)(rp1 - rp0) / (double)max(i, 1u));
  }
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t rl = k3_reread(out, n - 1);
  const int32_t pl = (int32_t)(uint32_t)rl;
  const uint32_t st = (uint32_t)(rl >> 32);
  const uint32_t lL = *(const lds_u32*)(uintptr_t)(tb + 8 * (st & 1023));
  const uint32_t lM = *(const lds_u32*)(uintptr_t)(tb + K3L_ML + 8 * ((st >> 10) & 1023));
  const uint32_t lO = *(const lds_u32*)(uintptr_t)(tb + K3L_OF + 8 * ((st >> 20) & 255));
  const uint32_t ls = lL + lM + lO;
  // the last sequence's extra bits: its count sum less its state bits
  const int32_t E = (int32_t)(((ls >> 8) & 255) - ((lL & 31) + (lM & 31) + (lO & 31)));
#ifdef ZD_EXP_K3L_RAWPUT
  return 1;
#endif
  return ((bad | ls) >> 16 || pl < 0 || E > pl) ? 1 : 0;
}

__global__ __launch_bounds__(64) void zd_k_sequences_l(const uint8_t* __restrict__ src,
                                                       const CompBlock* __restrict__ comp, CompState* cstate,
                                                       FrameState* fstate, const uint32_t* __restrict__ list,
                                                       uint32_t n_list, const uint16_t* __restrict__ fses,
                                                       uint64_t* __restrict__ recs, const uint8_t* __restrict__ redo) {
  __shared__ __attribute__((aligned(4096))) uint64_t tabs[K3L_BYTES / 8];
  const int lane = threadIdx.x;
  const uint32_t li = blockIdx.x;
  if (li >= n_list) return;
  const uint32_t ci = list[li];
  const CompBlock C = comp[ci];
  if (redo && !redo[C.frame]) return;          // the redo pass after zd_k_fused: flagged frames only
  const uint64_t key0 = fstate[C.frame].key;
  if (key0 != KEY_NONE && key_phase(key0) == PH_PARSE) return;
  const uint32_t tb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint64_t*)tabs;
  int al[3];
  k3l_tables(fses, C, comp, cstate, tb, al, lane);
  __syncthreads();
  const CompState cs = cstate[ci];
  const uint8_t* blk = src + C.src;
  int st = 0;
  if (seq_chainl(blk + cs.bs_off, cs.bs_size, (uintptr_t)src, tb, al[0], al[1], al[2], C.nseq, recs + C.seq_out) &&
      lane == 0) {
    const uint16_t* g[3];
    for (int k = 0; k < 3; k++) {
      const uint32_t s = (uint32_t)C.tab_src[k];
      g[k] = fses + (uint64_t)comp[s].fse_slot * FSE_SLOT + k * FSE_TAB;
    }
    st = K3_CHAIN<g_u16*, true>(blk + cs.bs_off, cs.bs_size, (uintptr_t)src, (g_u16*)g[0], (g_u16*)g[2], (g_u16*)g[1],
                                al[0], al[1], al[2], C.nseq, recs + C.seq_out);
  }
  if (st) k3_fail(C, ci, cstate, fstate, st);
}

// A K3 record pair read as 8-byte halves, record i's slot on lane i (a batch
// starting at an even record): the halves are exchanged with the partner lane
// and the lane's record unpacked (zd_common.h).  All 64 lanes active.
__device__ inline uint64_t rec_lane(uint64_t raw, int lane) {
  const uint32_t lo = (uint32_t)raw, hi = (uint32_t)(raw >> 32);
  const uint32_t plo = qdpp<QP_SWAP1>(lo), phi = qdpp<QP_SWAP1>(hi);
  const uint32_t h = lane & 1;
  return rec_unpack(h ? plo : lo, h ? phi : hi, h ? lo : plo, h ? hi : phi, h);
}

// ---------------------------------------------------------------------------
// K4: execute (decoding_context.rs:50-106 + block.rs:74-99), one frame per
// wave, one sequence per lane, 64 sequences per batch.  A frame that decodes
// past the capacity its plan reserved (its Frame_Content_Size, or 128 KiB per
// block without one; the reference checks neither) is out of the GPU path's
// domain (ZD_E_OUT_OF_DOMAIN).
//
// The wave keeps a linear LDS window: frame bytes [hs, pos) with hs aligned
// so that LDS offsets and HBM addresses share 16-byte alignment.  A batch
// writes its literals and matches into the window with 16-byte unaligned LDS
// copies (gfx950 runs in unaligned mode; tools/unaligned_check.hip), then the
// completed aligned chunks are flushed to HBM with 16-byte stores, and every
// K4_B bytes the last K4_W bytes slide to the front.  Match sources before
// hs are read from the frame's output in HBM (L1-bypassing loads, after the
// flush stores have drained).  Matches may depend on earlier sequences of
// the same batch: a lane copies once its source lies entirely below the
// first unfinished sequence's match (the batch frontier); a match copies its
// source period by period, byte q+j = byte q-off+(j mod off), which is the
// reference's byte-by-byte push (decoding_context.rs:95-98).
// ---------------------------------------------------------------------------
// History and room of the 7,200-byte window (round 5, C4 10 GiB on one box:
// history 1 / 2 / 3 / 4 / 4.5 / 5 / 5.25 KiB -> K4 18.70 / 18.23 / 17.98 /
// 17.66 / 17.73 / 18.74 / 18.71 ms -- more matches find their source in LDS
// until the slides come every batch; room 1792 / 1536 / 1280 at 4 KiB:
// 17.72 / 17.69 / 17.62, within noise)
#ifndef ZD_K4_W
#define ZD_K4_W 4096
#endif
#ifndef ZD_K4_B
#define ZD_K4_B 1536
#endif
constexpr int K4_W = ZD_K4_W;                 // history kept after a slide
constexpr int K4_B = ZD_K4_B;                 // room kept for a batch (a slide when less is left)
#ifndef ZD_K4_C
#define ZD_K4_C 7200
#endif
constexpr int K4_C = ZD_K4_C;                 // window bytes
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(3))) uint8_t l_u8;
typedef __attribute__((address_space(3))) u32x4a1 l_u32x4a1;
typedef __attribute__((address_space(3))) uint64_t l_u64a1 __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) uint32_t l_u32a1 __attribute__((aligned(1)));
typedef __attribute__((address_space(3))) uint16_t l_u16a1 __attribute__((aligned(1)));
typedef __attribute__((address_space(1))) const u32x4a1 g_cu32x4a1;
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
typedef __attribute__((address_space(3))) u32x4 l_u32x4;

__device__ inline u32x4 ldg16(const uint8_t* p) { return *(g_cu32x4a1*)p; }
// Match sources in HBM are read through the caches: the frame's own recent
// output, re-read by later matches (plain loads: the nontemporal form took
// 28.3 ms against 23.4 in round 1)
// (timing-only variants that change the output live in tools/exp_variants.patch)
__device__ inline u32x4 ldg16_src(const uint8_t* p) { return *(g_cu32x4a1*)p; }
// streams read once (records, literals): plain loads (nontemporal loads of
// the records, windows and literal stage measured slower: 1 GiB K4 2.06 ->
// 2.11 ms)
__device__ inline u32x4 ldg16_once(const uint8_t* p) {
  return *(g_cu32x4a1*)p;
}
__device__ inline u32x4 lds16(const l_u8* p) { return *(const l_u32x4a1*)p; }
// stores the first n (0..16) bytes of v at p
__device__ inline void sts_n(l_u8* p, u32x4 v, uint32_t n) {
  if (n >= 16) { *(l_u32x4a1*)p = v; return; }
  if (n & 8) { *(l_u64a1*)p = (uint64_t)v.x | ((uint64_t)v.y << 32); v.x = v.z; v.y = v.w; p += 8; }
  if (n & 4) { *(l_u32a1*)p = v.x; v.x = v.y; p += 4; }
  if (n & 2) { *(l_u16a1*)p = (uint16_t)v.x; v.x >>= 16; p += 2; }
  if (n & 1) { *p = (uint8_t)v.x; }
}
__device__ inline void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// The smallest multiple of the period off (1..15) that is >= 16, without a
// division (the compiler hoisted the division out of the rounds loop, ~25
// VALU ops per batch): 2 off from 8 on, else 5-bit entries of a constant.
__device__ inline uint32_t period16(uint32_t off) {
  constexpr uint64_t T = 16ull | 16ull << 5 | 18ull << 10 | 16ull << 15 | 20ull << 20 | 18ull << 25 | 21ull << 30;
  return off >= 8 ? 2 * off : (uint32_t)(T >> (5 * ((off - 1) & 7))) & 31;
}
__device__ inline int64_t readlane_i64(int64_t x, int l) {
  int lo = __shfl((int)(uint32_t)x, l, 64);
  int hi = __shfl((int)(uint32_t)((uint64_t)x >> 32), l, 64);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// Inclusive prefix sum over the 64 lanes (all active) with DPP moves:
// row_shr 1/2/4/8 inside 16-lane rows, then row_bcast 15 and 31 across rows.

// per-lane source lane (ds_bpermute)
__device__ inline uint64_t readlane_any_u64(uint64_t x, int l) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)x, l, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(x >> 32), l, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint64_t readlane_u64(uint64_t x, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
// Repeat offsets after `cnt` fresh lanes ending at lane end - 1 pushed their
// values on top of (r0, r1, r2) (decoding_context.rs:67-71 applied cnt times).
__device__ inline void rep_push(uint64_t val, int cnt, int end, uint64_t r0, uint64_t r1, uint64_t r2, uint64_t* a0,
                                uint64_t* a1, uint64_t* a2) {
  uint64_t b0 = r0, b1 = r1, b2 = r2;
  if (cnt >= 1) { b0 = readlane_u64(val, end - 1); b1 = r0; b2 = r1; }
  if (cnt >= 2) { b1 = readlane_u64(val, end - 2); b2 = r0; }
  if (cnt >= 3) b2 = readlane_u64(val, end - 3);
  *a0 = b0; *a1 = b1; *a2 = b2;
}

// Frame positions are 32-bit: frames with sequences stay below MAX_FRAME_OUT
// (2^27) and the planner caps every frame the streaming K4 runs below 2^31.
// K4's workgroup is one wave: LDS operations of a wave execute in order, so
// ordering between its own LDS writes and reads needs no lgkmcnt drain or
// s_barrier, only that the compiler keeps program order.
__device__ inline void k4_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// The window geometry: C bytes, W of history kept by a slide, B of room
// kept for a batch.
template <int C_, int W_, int B_>
struct K4W {
  static constexpr int C = C_, W = W_, B = B_;
  l_u8* buf;
  uint8_t* out;            // frame output (frame position 0)
  int32_t a0;              // frame position of the first 16-byte aligned HBM address (0..15)
  int32_t hs;              // frame position of buf[0]; hs = a0 (mod 16), may be < 0
  int32_t pos;             // decoded length
  int32_t fl;              // HBM holds [0, fl)
  int32_t cap;
  int lane;
  __device__ inline l_u8* at(int32_t p) const { return buf + (p - hs); }
  __device__ inline int32_t space() const { return C - (pos - hs); }
  __device__ inline int32_t alignd(int32_t p) const { return ((p - a0) & ~15) + a0; }
  // 16 bytes of frame output at p (p >= 0): LDS when inside the window, else HBM
  __device__ inline u32x4 src16(int32_t p) const { return p >= hs ? lds16(at(p)) : ldg16_src(out + (uint32_t)p); }
};
typedef K4W<K4_C, K4_W, K4_B> K4;

// HBM <- window: the aligned 16-byte chunks of [fl, pos) (all of it if final)
template <typename WX>
__device__ __attribute__((always_inline)) inline void k4_flush(WX& X, bool final) {
  const int32_t A = X.alignd(X.fl), E = X.alignd(X.pos);
  for (int32_t c = A + 16 * X.lane; c < E; c += 1024) {
    const u32x4 v = lds16(X.at(c));
    if (c >= 0) {
      *(g_u32x4*)(X.out + c) = v;
    } else {                                   // the frame's head chunk: only its own bytes
      for (int32_t b = 0; b < c + 16; b++) X.out[b] = *X.at(b);
    }
  }
  if (final) {
    for (int32_t b = (E > X.fl ? E : X.fl) + X.lane; b < X.pos; b += 64) X.out[b] = *X.at(b);
    X.fl = X.pos;
  } else if (E > X.fl) {
    X.fl = E;
  }
}

// Slides the window so that at least K4_B bytes are free (keeps K4_W of
// history).  An ascending chunked copy: each 1 KiB step reads all its chunks
// before writing any, and later steps read above everything written so far.
template <typename WX>
__device__ __attribute__((always_inline)) inline void k4_room(WX& X) {
  if (X.space() >= WX::B) return;
  const int32_t nh = X.alignd(X.pos - WX::W);  // <= fl: pos - fl < 16
  const int32_t n = X.pos - nh;                // <= W + 15 bytes move down by nh - hs
  const l_u8* from = X.at(nh);
  for (int32_t x = 16 * X.lane; x - 16 * X.lane < n; x += 1024) {
    u32x4 v;
    if (x < n) v = lds16(from + x);
    __builtin_amdgcn_wave_barrier();
    if (x < n) *(l_u32x4a1*)(X.buf + x) = v;
    __builtin_amdgcn_wave_barrier();
  }
  k4_sync();
  X.hs = nh;
}

// Appends n literal bytes from s (HBM) or the fill byte (s == nullptr), the
// whole wave copying 16 bytes per lane.  false: past the frame capacity.
template <typename WX>
__device__ __attribute__((always_inline)) inline bool k4_emit_lits(WX& X, const uint8_t* s, uint32_t fill, uint32_t n) {
  const u32x4 f4 = (u32x4){fill * 0x01010101u, fill * 0x01010101u, fill * 0x01010101u, fill * 0x01010101u};
  while (n) {
    k4_room(X);
    const int32_t chunk = (int32_t)min(n, (uint32_t)(X.space() - 16));
    if ((int64_t)X.pos + chunk > X.cap) return false;
    for (int32_t x = 16 * X.lane; x < chunk; x += 1024) {
      const u32x4 v = s ? ldg16(s + x) : f4;
      sts_n(X.at(X.pos + x), v, (uint32_t)(chunk - x));
    }
    k4_sync();
    X.pos += chunk;
    if (s) s += chunk;
    n -= (uint32_t)chunk;
    k4_flush(X, false);
  }
  return true;
}

// Appends n bytes of a match at offset off (1 <= off <= pos), whole wave.
// Byte j = byte (q - off + j mod off): every source byte precedes the match
// start q, in the window or (once slid out) in HBM.  A period shorter than 16
// is first unrolled into `pat` (48 bytes of it), so every 16-byte piece is one
// LDS read.
template <typename WX>
__device__ __attribute__((always_inline)) inline bool k4_emit_match(WX& X, l_u8* pat, uint32_t off, uint32_t n) {
  const int32_t q = X.pos;                     // match start
  uint32_t j0 = 0;
  const bool small = off < 16;
  const bool need_hbm = !small && q - (int32_t)off < X.hs;
  if (small) {                                 // q - off >= hs here: the period is in the window
    if (X.lane < 48) pat[X.lane] = *X.at(q - (int32_t)off + (int32_t)((uint32_t)X.lane % off));
    k4_sync();
  }
  if (__ballot(need_hbm)) wait_vm();
  while (j0 < n) {
    k4_room(X);
    if (j0 && !small) wait_vm();              // the last chunk's flush, before reading it back
    const int32_t chunk = (int32_t)min(n - j0, (uint32_t)(X.space() - 16));
    if ((int64_t)X.pos + chunk > X.cap) return false;
    for (int32_t x = 16 * X.lane; x < chunk; x += 1024) {
      const uint32_t j = j0 + (uint32_t)x, r = j % off;
      const uint32_t m = (uint32_t)(chunk - x < 16 ? chunk - x : 16);
      if (small) {
        sts_n(X.at(X.pos + x), lds16(pat + r), m);
      } else if (r + m <= off) {
        sts_n(X.at(X.pos + x), X.src16(q - (int32_t)off + (int32_t)r), m);
      } else {                                 // the piece wraps at the period
        for (uint32_t b = 0; b < m; b++) {
          const int32_t p = q - (int32_t)off + (int32_t)((j + b) % off);
          *X.at(X.pos + x + b) = p >= X.hs ? *X.at(p) : __builtin_nontemporal_load(X.out + p);
        }
      }
    }
    k4_sync();
    X.pos += chunk;
    j0 += (uint32_t)chunk;
    k4_flush(X, false);
  }
  return true;
}

// Inclusive prefix sum over the 64 lanes (all active) with DPP moves:
// row_shr 1/2/4/8 inside 16-lane rows, then row_bcast 15 and 31 across rows.
#ifndef ZD_K4_DPPASM
#define ZD_K4_DPPASM 1
#endif
__device__ inline uint32_t wave_scan_incl(uint32_t x) {
#if ZD_K4_DPPASM
  // one v_add_u32_dpp per step (the builtin form compiles to v_mov_dpp +
  // v_add); in place, so lanes a row_mask or the row edge leaves out keep x.
  // s_nop 1: the 2 wait states a DPP read of a just-written VGPR needs.
  asm volatile(
      "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
      "s_nop 1"
      : "+v"(x));
  return x;
#endif
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x;
}

#ifndef ZD_K4_MINW
#define ZD_K4_MINW 4
#endif
#ifndef ZD_K4_CODELUT
#define ZD_K4_CODELUT 1
#endif
#ifndef ZD_K4_INWIN
#define ZD_K4_INWIN 1
#endif
#ifndef ZD_K4_OVS
#define ZD_K4_OVS 1                         // pass 0: merged 16-byte chunks written past their end (0: exact per-part stores)
#endif
constexpr int K4_WPAD = ZD_K4_OVS ? 16 : 0;  // LDS bytes below the window
#ifndef ZD_K4_OVS_TRIP
#define ZD_K4_OVS_TRIP 2                    // pass 0: chunks past the second, this many per trip, loads first
#endif
constexpr uint32_t K4_OVS_TRIP = ZD_K4_OVS_TRIP;
#ifndef ZD_K4_STG
#define ZD_K4_STG 512                       // C4, 4 GiB: 1024 8.36 ms, 512 8.25, 256 8.24
#endif
constexpr uint32_t K4_STG = ZD_K4_STG;      // literal bytes staged per batch (64 lanes x 16 at most)
typedef __attribute__((address_space(3))) uint32_t l_u32;
// One K4 wave's LDS: the window, the period pattern, the block's LL | OF | ML
// symbols, the batch's literal stage and the code tables.
struct K4Lds {
  l_u8* win;                 // K4_C bytes
  l_u8* pat;                 // 64
  l_u8* stab;                // 3 x FSE_TAB
  l_u8* stg;                 // K4_STG + 16
  l_u32* codelut;            // 2 x 64
};
// Fused mode (zd_k_fused): the frame's records arrive while K3 runs in the
// same workgroup.  prog counts the 16-record lines K3 has completed
// (K4F_PROG_FINAL: all, K4F_PROG_ABANDON: the chain was rejected); k2done /
// k2need: K2's finished workgroups (the literals) in HBM.
constexpr uint32_t K4F_PROG_FINAL = 0x7FFFFFFFu, K4F_PROG_ABANDON = 0xFFFFFFFFu;
struct K4Fuse {
  const volatile l_u32* prog;
  const volatile l_u32* trdy;                 // nonzero: the block's sequence tables are in HBM
  const uint32_t* k2done;
  uint32_t k2need;
  uint32_t frame;
};
#ifndef ZD_FZ_SLEEP
#define ZD_FZ_SLEEP 2
#endif
// The frame's sequence tables (wave 0 of zd_k_fused builds them, with their
// CompState bytes and any parse error key), then K2's literals.  Relaxed
// polls (an acquire per poll would invalidate the caches every time, under
// the chains running beside), one acquire fence at the end: it also drops
// the CU's copy of the frame's key line, which wave 0 read before its
// key_min (an L2 atomic).  false: a wait ran past its bound, the frame goes
// to the redo pass.
__device__ inline bool k4f_wait_k2(const K4Fuse& z) {
  bool ok = false;
  for (uint32_t it = 0; it < (1u << 22) && !ok; it++) {
    ok = *z.trdy != 0;
    if (!ok) __builtin_amdgcn_s_sleep(ZD_FZ_SLEEP);
  }
  if (ok && z.k2need) {
    // bounded near K2's own time (fused plans hold <= 4 frames per CU: K2
    // takes well under 1 ms there); a wait past ~30 ms sends the frame to the
    // redo pass, which zd_plan_info.fused_redo_frames reports
    ok = false;
    for (uint32_t it = 0; it < (1u << 15) && !ok; it++) {
      ok = __hip_atomic_load(z.k2done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= z.k2need;
      if (!ok) __builtin_amdgcn_s_sleep(32);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return ok;
}
// records [0, rec_end) complete (whole 16-record lines); false: abandon
__device__ inline bool k4f_wait_recs(const K4Fuse& z, uint32_t rec_end) {
  const uint32_t need = (rec_end + 15) >> 4;
  for (uint32_t it = 0; it < (1u << 22); it++) {
    const uint32_t v = *z.prog;
    if (v == K4F_PROG_ABANDON) return false;
    if (v >= need) return true;
    __builtin_amdgcn_s_sleep(ZD_FZ_SLEEP);
  }
  return false;
}

template <bool FZ>
__device__ __attribute__((always_inline)) inline void k4_body(const uint8_t* __restrict__ src, uint8_t* outbase,
                                                   const FrameDesc* __restrict__ frames, FrameState* fstate,
                                                   const BlockRec* __restrict__ blocks,
                                                   const CompBlock* __restrict__ comp,
                                                   const CompState* __restrict__ cstate,
                                                   const uint8_t* __restrict__ lits,
                                                   const uint64_t* __restrict__ seqs,
                                                   const uint16_t* __restrict__ fses, uint32_t f_begin,
                                                   uint32_t f_end, uint32_t f_step, const uint8_t* __restrict__ redo,
                                                   const K4Lds& M, const K4Fuse* fz, uint8_t* redo_out) {
  l_u8* const win = M.win;
  l_u8* const pat = M.pat;
  l_u8* const stg = M.stg;
  const int lane = threadIdx.x & 63;
#if ZD_K4_CODELUT
  // LL | ML code -> baseline | extra-bit count << 24 (ll_code / ml_code,
  // sequences.rs tables), one LDS read per code instead of ~20 VALU ops
  l_u32 (*codelut)[64] = (l_u32 (*)[64])M.codelut;
  l_u8 (*stab)[FSE_TAB] = (l_u8 (*)[FSE_TAB])M.stab;
  {
    uint32_t b, e;
    ll_code((uint32_t)lane, &b, &e);
    codelut[0][lane] = b | (e << 24);
    ml_code((uint32_t)lane, &b, &e);
    codelut[1][lane] = b | (e << 24);
    k4_sync();
  }
#endif
#if !ZD_K4_CODELUT
  l_u8 (*stab)[FSE_TAB] = (l_u8 (*)[FSE_TAB])M.stab;
#endif
  // persistent over frames when the grid is capped
  for (uint32_t f = f_begin; f < f_end; f += f_step) {
  if (redo && !redo[f]) continue;                // the redo pass after zd_k_fused: its flagged frames only
  const FrameDesc F = frames[f];
  if (F.lds) continue;                           // K4F / K4J execute this frame
  FrameState* S = &fstate[f];
  bool abandoned = false;                        // fused mode: the frame goes to the redo pass
  if constexpr (FZ) abandoned = !k4f_wait_k2(*fz);   // (K1 and K2 have run: keys final)
  if (FZ && lane == 0) FZT(f, 3);
  const uint64_t key0 = S->key;
  if (key0 != KEY_NONE && key_phase(key0) == PH_PARSE) continue;

  K4 X;
  X.buf = (l_u8*)win;
  X.out = outbase + F.out;
  X.a0 = (int32_t)((16 - ((uintptr_t)X.out & 15)) & 15);
  X.lane = lane;
  X.pos = (int32_t)(F.out_len0 + F.skip_bytes);    // K0 wrote the leading raw/RLE blocks
  X.fl = X.pos;
  X.cap = (int32_t)(F.out_cap < 0x7FFFFFF0ull ? F.out_cap : 0x7FFFFFF0ull);
  {
    // window start: aligned, at most K4_W bytes back (context API: the
    // existing output's tail comes back from HBM)
    X.hs = X.alignd(X.pos > K4_W ? X.pos - K4_W : 0);
    for (int32_t p = (X.hs > 0 ? X.hs : 0) + lane; p < X.pos; p += 64) *X.at(p) = X.out[p];
    k4_sync();
  }
  // repeat offsets in 32 bits: every offset a frame can use without an
  // ImpossibleValue is below 2^31 (a position), and a larger one stops the
  // frame at its sequence, so saturating at 2^32 - 1 keeps every outcome
  auto sat32 = [](uint64_t v) -> uint32_t { return v < 0xFFFFFFFFull ? (uint32_t)v : 0xFFFFFFFFu; };
  uint32_t rep[3] = {sat32(S->rep[0]), sat32(S->rep[1]), sat32(S->rep[2])};
  uint64_t err_key = abandoned ? 0 : KEY_NONE;
  // HBM holds [0, fl_safe) with every store completed (the bytes two batches
  // back); fl_last = the flush boundary after the previous batch
  int32_t fl_safe = X.fl;
#ifdef ZD_K4_PROF
  uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tq = __builtin_amdgcn_s_memtime(), nb = 0, nr = 0;
#define K4_PHASE(i) do { const uint64_t tn = __builtin_amdgcn_s_memtime(); ph[i] += tn - tq; tq = tn; } while (0)
#else
#define K4_PHASE(i) do { } while (0)
#endif
// ISA markers (tests/test_isa_pass0.py compiles with -DZD_ISA_MARKS=1 and
// checks the instructions between them): empty in the library
#if ZD_ISA_MARKS
#define ZD_ISA_MARK(txt) asm volatile(txt)
#else
#define ZD_ISA_MARK(txt) do { } while (0)
#endif

  for (uint32_t j = F.skip; j < F.nblocks && err_key == KEY_NONE; j++) {
    const BlockRec B = blocks[F.first_block + j];
    // a decode error found before (K2), or a limit the plan found (a frame
    // past the int32 positions: block 0), ends the frame at its block
    if (key0 != KEY_NONE && key_phase(key0) != PH_PARSE && key_block(key0) <= j) break;
    if (B.type == 5) continue;
    if (B.type == 0 || B.type == 4) {
      if (!k4_emit_lits(X, src + B.src, 0, B.size)) err_key = make_key(PH_LIMIT, j, LS_CAPACITY, 0, ZD_E_OUT_OF_DOMAIN);
      continue;
    }
    if (B.type == 1) {
      if (!k4_emit_lits(X, nullptr, B.rle, B.size)) err_key = make_key(PH_LIMIT, j, LS_CAPACITY, 0, ZD_E_OUT_OF_DOMAIN);
      continue;
    }
    const CompBlock C = comp[B.comp];
    const CompState CS = cstate[B.comp];
    if (CS.stop) break;
    const uint8_t* lsrc = nullptr;
    uint32_t lfill = 0;
    uint32_t nl;
    if (C.lit_type == LIT_RAW) { lsrc = src + C.src + C.lit_data; nl = C.lit_regen; }
    else if (C.lit_type == LIT_RLE) { lfill = C.lit_rle; nl = C.lit_regen; }
    else { lsrc = lits + C.lit_out; nl = CS.lit_count; }
    const u32x4 f4 = (u32x4){lfill * 0x01010101u, lfill * 0x01010101u, lfill * 0x01010101u, lfill * 0x01010101u};
    uint32_t lit_cursor = 0;
    const uint64_t* SQ = seqs + C.seq_out;
    const uint32_t n = C.nseq;
    const bool direct = C.seq_direct != 0;
    // the block's LL/OF/ML symbols (K1's sym entries, zd_common.h) -> LDS
    const uint8_t* bsp = src + C.src + CS.bs_off;
    if (n && !direct) {
      for (int k = 0; k < 3; k++) {
        const uint32_t s = (uint32_t)C.tab_src[k];
        const uint16_t* g = fses + (uint64_t)comp[s].fse_slot * FSE_SLOT + k * FSE_TAB;
        const int cnt = 1 << cstate[s].al[k];
        for (int e = lane; e < cnt; e += 64) stab[k][e] = (uint8_t)(g[e] & 63);
      }
      k4_sync();
    }
    // Software pipeline over batches of 64 sequences: the records two
    // batches ahead, the bitstream windows of the next batch and its literal
    // bytes (1 KiB from the literal cursor, staged through LDS) one ahead,
    // so a batch waits on nothing it issued itself.  A sequence too large
    // for the window's room leaves the batch loop; the whole wave copies it
    // and the pipeline restarts after it.
    const bool lit_stage = lsrc != nullptr;
    // K3 records come in pairs (zd_common.h), a block's first at an even
    // index: lane i loads record i's 8-byte slot, half of its pair, and the
    // halves are exchanged with the partner lane once the load has landed
    // (rec_lane, at the wait that is there anyway).  A pipeline restart at an
    // odd record runs that one sequence alone, so batches start even.  The
    // context API's direct records are one 8-byte word each.
    const uint32_t n_ld = direct ? n : (n + 1) & ~1u;
    auto rec_at = [&](uint32_t i) -> uint64_t { return i < n_ld ? SQ[i] : 0; };
    auto rec_of = [&](uint64_t raw) -> uint64_t { return direct ? raw : rec_lane(raw, lane); };
    auto win_of = [&](uint64_t r, bool v) -> WinU {
      return winu_load(bsp, (uintptr_t)src, (v && !direct) ? (int32_t)(uint32_t)r : 0);
    };
    auto lit_of = [&](uint32_t cur) -> u32x4 {
      return (lit_stage && 16 * (uint32_t)lane < K4_STG && cur + 16 * (uint32_t)lane < nl) ? ldg16_once(lsrc + cur + 16 * lane) : f4;
    };
    for (uint32_t s0 = 0; s0 < n && err_key == KEY_NONE;) {
      if constexpr (FZ) {
        if (!k4f_wait_recs(*fz, min(n_ld, s0 + 128))) { abandoned = true; err_key = 0; break; }
      }
      const bool odd0 = !direct && (s0 & 1);        // a restart at an odd record
      const uint32_t vlim = odd0 ? s0 + 1 : n;       // (that record alone)
      uint64_t recA = odd0 ? (lane == 0 ? rec_get(SQ, s0, false) : 0) : rec_of(rec_at(s0 + lane));
      uint64_t recB = rec_at(s0 + 64 + lane);
      WinU winA = win_of(recA, s0 + lane < vlim);
      u32x4 litA = lit_of(lit_cursor);
      bool big = false;                              // batch loop left for one large sequence
      uint32_t bll = 0, bml = 0;
      uint32_t boff = 0;
      // One batch: the current pipeline set (records, windows, literal bytes of
      // this batch, records of the next) in, the next set out.  The loop runs it
      // twice a trip with the two sets' roles swapped, so no register rotation
      // is left at the back edge (the compiler kept ~16 moves a batch there).
      // false: the batch loop ends (an error, a large sequence, a partial batch).
      auto batch = [&](uint64_t& recA, WinU& winA, u32x4& litA, uint64_t& recB, uint64_t& recBv_o, WinU& winB_o,
                       u32x4& litB_o, uint64_t& recC_o) __attribute__((always_inline)) -> bool {
        const uint32_t i = s0 + lane;
        const bool valid = i < vlim;
        K4_PHASE(7);
        // this batch's literal bytes from the cursor on; lanes past the stage
        // all store into its 16-byte tail (only ever read as overshoot):
        // unconditional, a branch here cost 4 % of K4
        *(l_u32x4*)(stg + min(16 * (uint32_t)lane, K4_STG)) = litA;
        // The previous batch's output goes to HBM here, after the wait for
        // this batch's prefetched loads: those stores then have a batch to
        // drain before the next wait (vmcnt counts stores too, in order).
        // (the wait below is the one the compiler places here anyway)
        wait_vm();
        fl_safe = X.fl;
        // the next batch's windows and the records after it, first thing
        recBv_o = rec_of(recB);
        const uint64_t recBv = recBv_o;
        winB_o = win_of(recBv, s0 + 64 + lane < n);
        if constexpr (FZ) {
          if (!k4f_wait_recs(*fz, min(n_ld, s0 + 192))) { abandoned = true; err_key = 0; return false; }
        }
        recC_o = rec_at(s0 + 128 + lane);
        k4_flush(X, false);
        // Sequence values (update_symbol_value, decoders/sequence.rs:41-55):
        // K3 recorded the bit position and the three states; OF, ML, LL
        // extra bits are read here, in that order, below the position.
        uint32_t ll = 0, ml = 0, ofv = 0;
        bool giant = false;
        if (valid) {
          if (direct) {
            seq_values(recA, C.seq_side, i, &ll, &ml, &ofv);
            giant = ofv == DIRECT_GIANT && !C.seq_side;
          } else {
            const uint32_t stt = (uint32_t)(recA >> 32);
            const uint32_t llc = stab[0][stt & 1023], mlc = stab[2][(stt >> 10) & 1023], ofc = stab[1][stt >> 20] & 31;
            uint32_t llbase, llb, mlbase, mlb;
#if ZD_K4_CODELUT
            const uint32_t cl = codelut[0][llc], cm = codelut[1][mlc];
            llbase = cl & 0xFFFFFF; llb = cl >> 24;
            mlbase = cm & 0xFFFFFF; mlb = cm >> 24;
#else
            ll_code(llc, &llbase, &llb);
            ml_code(mlc, &mlbase, &mlb);
#endif
            // the OF, ML, LL extra bits MSB-first below the position: from
            // the top 32 bits when the batch's fit them (three bit-field
            // extracts), else from the top 64
            const uint32_t S3 = ofc + mlb + llb;
            if (__ballot(S3 > 32 || winA.sh > 32) == 0) {
              const uint32_t t32 = (uint32_t)((winA.w1 << winA.sh) >> 32);
              ofv = (1u << ofc) + __builtin_amdgcn_ubfe(t32, 32 - ofc, ofc);
              ml = mlbase + __builtin_amdgcn_ubfe(t32, 32 - ofc - mlb, mlb);
              ll = llbase + __builtin_amdgcn_ubfe(t32, 32 - S3, llb);
            } else {
              uint64_t t = winu_top(winA, 0);
              const uint32_t ob = take_top(t, ofc), mb = take_top(t, mlb), lb = take_top(t, llb);
              ofv = (1u << ofc) + ob;
              ml = mlbase + mb;
              ll = llbase + lb;
            }
          }
        }
        K4_PHASE(0);
        // the next batch's literal bytes (used only when all 64 lanes
        // execute, so from the cursor after all of them)
        const uint32_t inc_ll = wave_scan_incl(ll);
        litB_o = lit_of(lit_cursor + (uint32_t)__builtin_amdgcn_readlane((int)inc_ll, 63));
        k4_room(X);
        const uint32_t tot = ll + ml;
        const uint32_t inc_tot = wave_scan_incl(tot);
        const uint32_t opos = inc_tot - tot, lpos = inc_ll - ll;
        const uint64_t fitm = __ballot(valid && (int32_t)inc_tot <= X.space() - 16);
        const uint32_t k = (uint32_t)__popcll(fitm);
        const int kk = k ? (int)k : 1;                 // lanes this batch executes
        // decode_offset (decoding_context.rs:50-75): fresh offsets (> 3)
        // are direct; the rare repeat codes walk the batch in order on the
        // scalar unit, each from the state the fresh offsets before it left.
        const bool fresh = ofv > 3;
        // off32: a fresh lane's offset (offset_value - 3; 2^32 - 1 for the
        // context API's giant values), a repeat lane's once the walk set it
        uint32_t off32 = giant ? 0xFFFFFFFFu : ofv - 3;
        int derr = 0;
        uint64_t rm = __ballot(valid && !fresh && lane < kk);
        // state after lane `prev` (uniform: readfirstlane keeps the walk on the scalar unit)
        uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)rep[0]);
        uint32_t r1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)rep[1]);
        uint32_t r2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)rep[2]);
        int prev = -1;
        // a repeat lane's code (offset_value 0..3) and whether its literals_length is 0
        const uint32_t rcode = (ofv & 3) | (ll != 0 ? 4u : 0u);
        while (rm) {
          const int ri = __ffsll((long long)rm) - 1;
          rm &= rm - 1;
          // the fresh lanes between prev and ri pushed their values (at most the last three count)
          const int cnt = ri - prev - 1;
          uint32_t a0 = r0, a1 = r1, a2 = r2;
          if (cnt >= 1) { a0 = (uint32_t)__builtin_amdgcn_readlane((int)off32, ri - 1); a1 = r0; a2 = r1; }
          if (cnt >= 2) { a1 = (uint32_t)__builtin_amdgcn_readlane((int)off32, ri - 2); a2 = r0; }
          if (cnt >= 3) a2 = (uint32_t)__builtin_amdgcn_readlane((int)off32, ri - 3);
          const uint32_t ci = (uint32_t)__builtin_amdgcn_readlane((int)rcode, ri);
          const uint32_t oi = ci & 3;
          uint32_t o = 0;
          int e = 0;
          if (oi == 0) {
            e = ZD_E_NULL_OFFSET;
          } else {
            const uint32_t idx = oi - ((ci & 4) ? 1u : 0u);
            if (idx == 0) { o = a0; }
            else if (idx == 1) { o = a1; a1 = a0; a0 = o; }
            else if (idx == 2) { o = a2; a2 = a1; a1 = a0; a0 = o; }
            else if (a0 == 0) { e = ZD_E_REF_PANIC; }     // usize underflow of offsets[0] -= 1
            else { o = a0 - 1; a2 = a1; a1 = a0; a0 = o; }
          }
          off32 = lane == ri ? o : off32;
          derr = lane == ri ? e : derr;
          r0 = a0; r1 = a1; r2 = a2;
          prev = ri;
          if (e) break;                                // the frame stops at this sequence
        }
        // the repeat state after lane end - 1, the lanes after prev fresh
        auto rep_after = [&](int end) {
          const int c = end - 1 - prev;
          uint32_t b0 = r0, b1 = r1, b2 = r2;
          if (c >= 1) { b0 = (uint32_t)__builtin_amdgcn_readlane((int)off32, end - 1); b1 = r0; b2 = r1; }
          if (c >= 2) { b1 = (uint32_t)__builtin_amdgcn_readlane((int)off32, end - 2); b2 = r0; }
          if (c >= 3) b2 = (uint32_t)__builtin_amdgcn_readlane((int)off32, end - 3);
          rep[0] = b0; rep[1] = b1; rep[2] = b2;
        };
        K4_PHASE(1);
        // matches whose source lies wholly in HBM, flushed two batches ago or
        // earlier (those stores completed before this batch's waits): their
        // first 32 source bytes are loaded now, to land during the checks
        // and the literal copies
        const int32_t q = X.pos + (int32_t)(opos + ll);
        const int32_t slo = q - (int32_t)off32;
        const int32_t shi = slo + (int32_t)(off32 < ml ? off32 : ml);
        const bool far = valid && lane < kk && ml && off32 >= 16 && off32 <= (uint32_t)q &&
                         shi <= (X.hs < fl_safe ? X.hs : fl_safe);
#if ZD_K4_OVS
        // pass 0 (below) writes each lane's sequence as 16-byte chunks that
        // merge its literal and match bytes; a far lane's first two chunks'
        // match bytes are loaded now (chunk b reads the source at slo + b - ll,
        // so the match bytes land at chunk offset ll - b; a chunk of literal
        // bytes only reads at slo)
        u32x4 fv0, fv1;
        const bool far0 = far && slo >= 16;
        const uint32_t n0f = ll + ml;
        const uint32_t bb1 = n0f >= 32 ? 16u : (n0f > 16 ? n0f - 16 : 0u);
        if (far0) {
          fv0 = ldg16_src(X.out + (uint32_t)(ll >= 16 ? slo : slo - (int32_t)ll));
          if (n0f > 16) fv1 = ldg16_src(X.out + (uint32_t)(ll >= bb1 + 16 ? slo : slo + (int32_t)bb1 - (int32_t)ll));
        }
#else
        u32x4 fv0, fv1;
        if (far) {
          fv0 = ldg16_src(X.out + (uint32_t)slo);
          if (ml > 16) fv1 = ldg16_src(X.out + (uint32_t)(slo + 16));
        }
#endif
        // matches whose source lies wholly in the window and before this
        // batch (written by earlier batches, so no order among the lanes):
        // copied from LDS in the same pass as the far ones, not in rounds.
        // Not overlapping (off >= ml): the pass reads four pieces before it
        // writes them (a lane at the batch start with ll = 0 and off < ml
        // has shi = q = the batch start)
        const bool inwin = ZD_K4_INWIN && valid && lane < kk && ml && !far && off32 >= 16 && off32 >= ml &&
                           off32 <= (uint32_t)q && slo >= X.hs && shi <= X.pos;
        // checks (decoding_context.rs:86-90, D9), in 32 bits: positions stay
        // below 2^31 + 2^25 and off32 saturates (an offset of 2^32 or more
        // is past any position)
        const uint32_t before = (uint32_t)X.pos + opos;
        const bool dbad = valid && derr != 0;
        const bool imp = valid && !dbad && (lit_cursor + lpos + ll > nl || off32 > before + ll);
        const bool panic = valid && !dbad && !imp && ml != 0 && off32 == 0;
        const uint64_t badm = __ballot(dbad || imp || panic);
        if (badm) {
          const int b = __ffsll((long long)badm) - 1;
          if (b < kk) {
            const int code = __builtin_amdgcn_readlane(dbad ? derr : (imp ? ZD_E_IMPOSSIBLE_VALUE : ZD_E_REF_PANIC), b);
            err_key = make_key(PH_DECODE, j, DS_EXECUTE, s0 + b, code);
            return false;
          }
        }
        if (k == 0) {                                  // lane 0 alone does not fit the room
          big = true;
          bll = (uint32_t)__builtin_amdgcn_readlane((int)ll, 0);
          bml = (uint32_t)__builtin_amdgcn_readlane((int)ml, 0);
          boff = (uint32_t)__builtin_amdgcn_readlane((int)off32, 0);
          rep_after(1);
          return false;
        }
        const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)inc_tot, (int)k - 1);
        const uint32_t L = (uint32_t)__builtin_amdgcn_readlane((int)inc_ll, (int)k - 1);
        if ((int64_t)X.pos + T > X.cap) { err_key = make_key(PH_LIMIT, j, LS_CAPACITY, s0, ZD_E_OUT_OF_DOMAIN); return false; }
        const bool act = (uint32_t)lane < k;
        k4_sync();                               // staged literals visible
#if ZD_K4_OVS
        // Pass 0: every executing lane writes its bytes as 16-byte chunks at
        // its output start: the whole sequence (literals then match) when
        // the match source lies before this batch (far: HBM, inwin: window)
        // or there is no match, else its literals only (the match follows in
        // the frontier rounds).  Chunks start every 16 bytes and the last one
        // ends exactly at the lane's end, so only a lane writing fewer than 16
        // bytes writes past its end: into later lanes' bytes, which this same
        // store rewrites (LDS: within one wave's ds_write, the highest lane
        // writing a byte wins -- tools/lds_order_check, test_lds_write_order)
        // or which the lanes' own later writes cover (a literals-only lane's
        // match, a lane with literals past the stage).  A chunk takes
        // ll - b literal bytes (from the stage) then match bytes read at
        // slo + b - ll: the bytes before slo are never used, and the window
        // keeps 16 bytes of padding below its start for them.
        const bool lslow = act && ll && lit_stage && lpos + ll > K4_STG;
        const bool full0 = act && !lslow && (ml == 0 || far0 || inwin);
        const uint32_t n0 = (act && !lslow) ? (full0 ? ll + ml : ll) : 0u;
        if (n0) {
          l_u8* d = X.at(X.pos + (int32_t)opos);
          const uint32_t last = n0 >= 16 ? n0 - 16 : 0u;
          const bool src_far = full0 && far0;
          const bool src_win = full0 && inwin;
          // the chunk at byte bb of the lane's run: ll - bb literal bytes from
          // the stage, then match bytes mv (read at msrc(bb))
          auto msrc = [&](uint32_t bb) -> int32_t {
            return ll >= bb + 16 ? slo : slo + (int32_t)bb - (int32_t)ll;
          };
          auto put = [&](uint32_t bb, u32x4 mv) {
            const uint32_t kl = ll > bb ? min(ll - bb, 16u) : 0u;   // literal bytes in the chunk
            u32x4 lv = f4;
            if (lit_stage) lv = lds16((const l_u8*)stg + min(lpos + bb, K4_STG));
            const uint64_t mlo = kl >= 8 ? ~0ull : ((1ull << (8 * kl)) - 1);
            const uint64_t mhi = kl >= 16 ? ~0ull : (kl <= 8 ? 0ull : ((1ull << (8 * (kl - 8))) - 1));
            u32x4 v;
            v.x = ((uint32_t)mlo & lv.x) | (~(uint32_t)mlo & mv.x);
            v.y = ((uint32_t)(mlo >> 32) & lv.y) | (~(uint32_t)(mlo >> 32) & mv.y);
            v.z = ((uint32_t)mhi & lv.z) | (~(uint32_t)mhi & mv.z);
            v.w = ((uint32_t)(mhi >> 32) & lv.w) | (~(uint32_t)(mhi >> 32) & mv.w);
            ZD_ISA_MARK("; ZDPUT<");
            *(l_u32x4a1*)(d + bb) = v;       // ONE ds_write_b128 (test_isa_pass0)
            ZD_ISA_MARK("; ZDPUT>");
          };
          auto mload = [&](uint32_t bb) -> u32x4 {
            return src_far ? ldg16_src(X.out + (uint32_t)msrc(bb)) : src_win ? lds16(X.at(msrc(bb))) : f4;
          };
          // chunks 0 and 1 (a far lane's match bytes were loaded above), then
          // four at a time, their loads first (no match here overlaps itself)
          put(0, src_far ? fv0 : mload(0));
          if (n0 > 16) put(min(16u, last), src_far ? fv1 : mload(min(16u, last)));   // (far: bb1 == min(16, last))
          for (uint32_t j0 = 2; 16 * j0 < n0; j0 += K4_OVS_TRIP) {
            u32x4 m[K4_OVS_TRIP];
#pragma unroll
            for (uint32_t q = 0; q < K4_OVS_TRIP; q++)
              if (16 * (j0 + q) < n0) m[q] = mload(min(16 * (j0 + q), last));
#pragma unroll
            for (uint32_t q = 0; q < K4_OVS_TRIP; q++)
              if (16 * (j0 + q) < n0) put(min(16 * (j0 + q), last), m[q]);
          }
        }
        if (__ballot(lslow)) {                         // literals past the stage: exact, from HBM
          if (lslow) {
            l_u8* d = X.at(X.pos + (int32_t)opos);
            for (uint32_t x = 0; x < ll; x += 16) sts_n(d + x, ldg16(lsrc + lit_cursor + lpos + x), ll - x);
          }
        }
        K4_PHASE(2);
        K4_PHASE(3);
        if (__ballot(act && ml && !full0 && slo < X.hs)) wait_vm();
        uint64_t done = __ballot(!act || full0);
#else
        // literals (every lane its own run; from the stage when it holds them)
        if (act && ll) {
          l_u8* d = X.at(X.pos + (int32_t)opos);
          if (!lit_stage || lpos + ll <= K4_STG) {
            const l_u8* sp = (const l_u8*)stg + lpos;
            for (uint32_t x = 0; x < ll; x += 16) sts_n(d + x, lit_stage ? lds16(sp + x) : f4, ll - x);
          } else {
            for (uint32_t x = 0; x < ll; x += 16) sts_n(d + x, ldg16(lsrc + lit_cursor + lpos + x), ll - x);
          }
        }
        K4_PHASE(2);
        // far matches from the bytes loaded above (ml < off: no overlap);
        // the rest in frontier rounds
        if (far || inwin) {
          l_u8* d = X.at(q);
          u32x4 a0 = fv0;
          if (inwin) a0 = lds16(X.at(slo));
          sts_n(d, a0, ml);
          if (ml > 16) {
            u32x4 a1 = fv1;
            if (inwin) a1 = lds16(X.at(slo + 16));
            sts_n(d + 16, a1, ml - 16);
          }
          // the rest four pieces at a time: one load latency per 64 bytes
          for (uint32_t x = 32; x < ml; x += 64) {
            u32x4 v0, v1 = fv0, v2 = fv0, v3 = fv0;
            if (inwin) {
              v0 = lds16(X.at(slo + (int32_t)x));
              if (x + 16 < ml) v1 = lds16(X.at(slo + (int32_t)x + 16));
              if (x + 32 < ml) v2 = lds16(X.at(slo + (int32_t)x + 32));
              if (x + 48 < ml) v3 = lds16(X.at(slo + (int32_t)x + 48));
            } else {
              const uint8_t* sp = X.out + (uint32_t)slo;
              v0 = ldg16_src(sp + x);
              if (x + 16 < ml) v1 = ldg16_src(sp + x + 16);
              if (x + 32 < ml) v2 = ldg16_src(sp + x + 32);
              if (x + 48 < ml) v3 = ldg16_src(sp + x + 48);
            }
            sts_n(d + x, v0, ml - x);
            if (x + 16 < ml) sts_n(d + x + 16, v1, ml - x - 16);
            if (x + 32 < ml) sts_n(d + x + 32, v2, ml - x - 32);
            if (x + 48 < ml) sts_n(d + x + 48, v3, ml - x - 48);
          }
        }
        if (__ballot(act && ml && !far && slo < X.hs)) wait_vm();
        uint64_t done = __ballot(!act || ml == 0 || far || inwin);
#endif
        k4_sync();
        K4_PHASE(3);
        while (done != ~0ull) {
          const int U = __ffsll((long long)~done) - 1;
          const int32_t qU = __builtin_amdgcn_readlane(q, U);
          const bool mine = !((done >> lane) & 1) && (lane == U || shi <= qU);
          if (mine) {
            l_u8* d = X.at(q);
            if (off32 >= 16) {
              for (uint32_t x = 0; x < ml; x += 16) sts_n(d + x, X.src16(slo + (int32_t)x), ml - x);
            } else {                             // small period: first 16 bytes bytewise, then 16-byte steps
              const uint32_t m16 = period16(off32);
              const uint32_t head = ml < 16 ? ml : 16;
              uint32_t r = 0;
              for (uint32_t x = 0; x < head; x++) {
                d[x] = *X.at(slo + (int32_t)r);
                r = r + 1 == off32 ? 0 : r + 1;
              }
              for (uint32_t x = 16; x < ml; x += 16) sts_n(d + x, lds16(d + x - m16), ml - x);
            }
          }
          done |= __ballot(mine);
          k4_sync();
#ifdef ZD_K4_PROF
          nr++;
#endif
        }
        K4_PHASE(4);
#ifdef ZD_K4_PROF
        nb++;
#endif
        rep_after((int)k);                             // state after lane k - 1
        lit_cursor += L;
        X.pos += (int32_t)T;
        s0 += k;
        K4_PHASE(5);
        return !(k < 64 || s0 >= n);                  // a partial batch: the pipeline restarts at s0
      };
      uint64_t recA2 = 0, recB2 = 0;
      WinU winA2 = winA;
      u32x4 litA2 = litA;
      for (;;) {
        if (!batch(recA, winA, litA, recB, recA2, winA2, litA2, recB2)) break;
        if (!batch(recA2, winA2, litA2, recB2, recA, winA, litA, recB)) break;
      }
      k4_flush(X, false);                            // k4_room and the large-sequence path expect it
      if (big && err_key == KEY_NONE) {
        // one sequence larger than the window's room: the whole wave copies it
        if (!k4_emit_lits(X, lsrc ? lsrc + lit_cursor : nullptr, lfill, bll) ||
            !k4_emit_match(X, (l_u8*)pat, boff, bml)) {
          err_key = make_key(PH_LIMIT, j, LS_CAPACITY, s0, ZD_E_OUT_OF_DOMAIN);
          break;
        }
        lit_cursor += bll;
        s0 += 1;
      }
    }
    if (err_key != KEY_NONE) break;
    // leftover literals (decoding_context.rs:101-103)
    if (lit_cursor < nl && !k4_emit_lits(X, lsrc ? lsrc + lit_cursor : nullptr, lfill, nl - lit_cursor))
      err_key = make_key(PH_LIMIT, j, LS_CAPACITY, n, ZD_E_OUT_OF_DOMAIN);
  }
  if (err_key != KEY_NONE) {
    if (lane == 0) {
      if (abandoned) redo_out[f] = 1;
      else key_min(fstate, f, err_key);
    }
    k4_sync();
    continue;
  }
  k4_flush(X, true);
  if (FZ && lane == 0) FZT(f, 4);
#ifdef ZD_K4_PROF
  if (lane == 0 && f < 3)
    printf("K4 frame %u batches %llu rounds %llu: rec/val %llu scan/rep %llu chk/lit %llu far %llu rounds %llu flush %llu top %llu\n", f,
           (unsigned long long)nb, (unsigned long long)nr, (unsigned long long)ph[0], (unsigned long long)ph[1],
           (unsigned long long)ph[2], (unsigned long long)ph[3], (unsigned long long)ph[4], (unsigned long long)ph[5],
           (unsigned long long)ph[7]);
#endif
  if (lane == 0) {
    S->out_len = (uint64_t)X.pos;
    S->rep[0] = rep[0];
    S->rep[1] = rep[1];
    S->rep[2] = rep[2];
  }
  k4_sync();                               // the window is reused by the next frame
  }
}

__global__ __launch_bounds__(64, ZD_K4_MINW) void zd_k_execute(const uint8_t* __restrict__ src, uint8_t* outbase,
                                                   const FrameDesc* __restrict__ frames, FrameState* fstate,
                                                   const BlockRec* __restrict__ blocks,
                                                   const CompBlock* __restrict__ comp,
                                                   const CompState* __restrict__ cstate,
                                                   const uint8_t* __restrict__ lits,
                                                   const uint64_t* __restrict__ seqs,
                                                   const uint16_t* __restrict__ fses, uint32_t f_begin,
                                                   uint32_t f_end, const uint8_t* __restrict__ redo) {
  // (16 bytes of padding below the window: pass 0 reads up to 15 bytes before a match source)
  __shared__ __attribute__((aligned(16))) uint8_t win[K4_WPAD + K4_C];
  __shared__ __attribute__((aligned(16))) uint8_t pat[64];
  __shared__ __attribute__((aligned(16))) uint8_t stab[3 * FSE_TAB];   // LL | OF | ML symbols of the block
  __shared__ __attribute__((aligned(16))) uint8_t stg[K4_STG + 16];    // a batch's literal bytes (K4_STG of them)
  __shared__ uint32_t codelut[2 * 64];
  const K4Lds M{(l_u8*)win + K4_WPAD, (l_u8*)pat, (l_u8*)stab, (l_u8*)stg, (l_u32*)codelut};
  k4_body<false>(src, outbase, frames, fstate, blocks, comp, cstate, lits, seqs, fses, f_begin + blockIdx.x, f_end,
                 gridDim.x, redo, M, nullptr, nullptr);
}

// ---------------------------------------------------------------------------
// zd_k_fused: K1's sequence half, K3 and K4 of FZ_FRAMES single-block frames
// in one workgroup, for plans of few such frames (C3), where K3 is one round
// of chains and a K4 launch after it would leave every frame waiting for the
// longest chain.  Wave 0 builds the blocks' FSE tables (quad q, lane k < 3:
// table k of frame q, straight into LDS; zd_k_tables PART 2 is not launched)
// and runs K3Q on them, publishing each chain's completed 16-record lines to
// LDS (seq_chainq PUB); wave 1 + q runs K4 for frame q (k4_body FZ), waiting
// for the tables (trdy), for K2's literals (zd_k_huffman counts its
// workgroups in k2done, released at agent scope) and for its records line by
// line, so K4 runs behind the chain instead of after all chains.  Records and
// literals never share a 128-byte line between blocks in such plans, and a
// K4 wave reads a line only once it is complete, so the wave's caches hold no
// stale record or literal.  A chain the fast path rejects (or a wait past its
// bound) flags its frame in `redo`: the K4 wave abandons the frame without
// writing its state, and the redo pass (K3Q + K4 over the flagged frames,
// after this kernel, on the tables this kernel left in HBM) decodes it as the
// unfused pipeline would.
// ---------------------------------------------------------------------------
// The K4 waves' build of their blocks' sequence tables (K1's sequence half,
// zd_k_tables PART 2, for the fused plans): the wave is idle until K2's
// literals anyway, and 64 lanes build a table far sooner than one lane's
// serial walk, which put K1's sequence half (0.25 ms) before every chain.
struct FzK1 {
  int16_t dist[3][256];
  uint16_t tab[3][FSE_TAB];          // compact entries (the slot format)
  uint16_t cum[260];                 // placements before each symbol
  uint16_t cnt[256];                 // nextState counters
  uint8_t sym[FSE_TAB];
  uint64_t lanes[64];                // fz_build_fse: a chunk's lanes by symbol (tables of <= 64 symbols)
};
struct FzInfo {                      // a block's table results, for wave 0
  uint32_t al;                       // LL | OF << 8 | ML << 16
  uint32_t err;                      // first failure: sub << 8 | -code (0: none)
  uint32_t bo, bsz;                  // sequence bitstream
};

__device__ inline uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// FseTable::from_distribution (fse.rs:110-202) by a whole wave, with
// build_fse's results and errors.  The spread visits positions j * step &
// mask (a permutation of the states: step is odd), skipping the -1 symbols'
// top positions, so placement r in symbol order lands on the r-th such
// position below zero_pos: each lane takes positions j and finds its
// symbol from the placement's rank (a search over the cumulative counts).
// nextState of state i is count(s) plus the earlier states of s: per 64
// states, one round per distinct symbol.
#ifndef ZD_FZ_LANEMASK
#define ZD_FZ_LANEMASK 1
#endif
__device__ int fz_build_fse(int al, const int16_t* dist, uint32_t nsym, uint16_t* tab, FzK1& W, int lane) {
  if (al > FSE_MAX_AL) return ZD_E_LARGE_ACCURACY_LOG;
  const uint32_t T = 1u << al, mask = T - 1, step = (T >> 1) + (T >> 3) + 3;
  uint32_t nneg = 0, placed = 0;
  for (uint32_t b = 0; b < nsym; b += 64) {
    const uint32_t s = b + lane;
    const int c = s < nsym ? dist[s] : 0;
    const uint64_t neg = __ballot(c == -1);
    if (c == -1) {                             // build_fse's first loop: sym[--zero_pos] = s
      const uint32_t m = nneg + lanes_below(neg);
      if (m < T) W.sym[T - 1 - m] = (uint8_t)s;
    }
    const uint32_t pc = c > 0 ? (uint32_t)c : 0u;
    const uint32_t inc = wave_scan_incl(pc);
    if (s < nsym) W.cum[s] = (uint16_t)(placed + inc - pc);
    placed += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    nneg += (uint32_t)__popcll(neg);
  }
  if (nneg > T) return ZD_E_REF_PANIC;
  const uint32_t zero_pos = T - nneg;
  if (placed > 0 && zero_pos == 0) return ZD_E_REF_PANIC;   // the reference loops forever
  if (placed != zero_pos) return ZD_E_CORRUPTED_TABLE;
  k4_sync();
  uint32_t rbase = 0;
  for (uint32_t j0 = 0; j0 < T; j0 += 64) {
    const uint32_t j = j0 + lane;
    const uint32_t x = (j * step) & mask;
    const bool v = j < T && x < zero_pos;
    const uint64_t bm = __ballot(v);
    if (v) {
      const uint32_t r = rbase + lanes_below(bm);
      uint32_t lo = 0, hi = nsym;                // the last symbol with cum <= r
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (W.cum[mid] <= r) lo = mid; else hi = mid;
      }
      W.sym[x] = (uint8_t)lo;
    }
    rbase += (uint32_t)__popcll(bm);
  }
  for (uint32_t s = lane; s < nsym; s += 64) {
    const int c = dist[s];
    W.cnt[s] = (uint16_t)(c > 0 ? c : (c == -1 ? 1 : 0));
  }
  k4_sync();
  const bool by_lds = ZD_FZ_LANEMASK && nsym <= 64;
  for (uint32_t i0 = 0; i0 < T; i0 += 64) {
    const uint32_t i = i0 + lane;
    const uint32_t s = i < T ? W.sym[i] : 0u;
    // the lane's rank among the chunk's states of its symbol, and their number
    uint32_t occ = 0, tot = 0;
    if (by_lds) {
      // the chunk's lanes of each symbol as a 64-bit mask in LDS (one OR
      // per lane), instead of one ballot round per distinct symbol (C3: the
      // three tables took ~31 us)
      if (i < T) W.lanes[s] = 0;
      k4_sync();
      if (i < T) __hip_atomic_fetch_or(&W.lanes[s], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      k4_sync();
      const uint64_t m = i < T ? W.lanes[s] : 0ull;
      occ = lanes_below(m);
      tot = (uint32_t)__popcll(m);
    } else {
      // (registers only: one round per distinct symbol)
      uint64_t rem = __ballot(i < T);
      while (rem) {
        const uint32_t sl = (uint32_t)__builtin_amdgcn_readlane((int)s, (int)__builtin_ctzll(rem));
        const uint64_t m = __ballot(s == sl) & rem;
        if ((m >> lane) & 1) { occ = lanes_below(m); tot = (uint32_t)__popcll(m); }
        rem &= ~m;
      }
    }
    const uint32_t ns = i < T ? W.cnt[s] + occ : 0u;
    k4_sync();
    if (i < T && occ + 1 == tot) W.cnt[s] = (uint16_t)(ns + 1);   // the symbol's last state in the chunk
    k4_sync();
    if (i < T) tab[i] = fse_entry(s, ns);
  }
  k4_sync();
  return 0;
}

// A K4 wave's block: k1_sequences_lane's walk (sequences.rs:91-187), each
// table built by the wave; then what zd_k_tables leaves (the tables the serial walk completes
// in the block's slot, their accuracy logs, the bitstream, a parse error's
// key), the K3 tables for wave 0 (tabs, when they fit) and the block's
// FzInfo.  Every lane returns.
__device__ __attribute__((always_inline)) inline void fz_tables(const uint8_t* __restrict__ src, const CompBlock& C, uint32_t ci, CompState* cstate,
                          FrameState* fstate, uint16_t* fses, FzK1& W, lds_u16* k3tab, FzInfo& I, int lane,
                          uint32_t f) {
  // the descriptions in order, by every lane on the same (wave-uniform)
  // values, so the walk runs on the scalar unit: one lane of a wave64 would
  // take four cycles an operation (0.03 ms for a block's three tables)
  const uint32_t base = C.seq_tables;
  const uint8_t* blk = src + C.src;
  // the description bytes in registers (512 from a 4-aligned base; a dword
  // that starts past the block reads as 0, none reaches past the input)
  const uint8_t* wb = (const uint8_t*)((uintptr_t)(blk + base) & ~(uintptr_t)3);
  const uint8_t* bend = blk + C.size;
  const uint32_t r0 = wb + 4 * lane < bend ? *(const uint32_t*)(wb + 4 * lane) : 0u;
  const uint32_t r1 = wb + 4 * (lane + 64) < bend ? *(const uint32_t*)(wb + 4 * (lane + 64)) : 0u;
#ifdef FZT_ON
  if (lane == 0) FZT(f, 9);
#endif
  int pst = 0, psub = 3;
  uint32_t alp = 0, nsp = 0, rle = 0, pos = base;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    if (pst) break;
    const int mode = C.modes[k];
    int st = 0, al = 0;
    uint32_t nsym = 0;
    if (mode == M_RLE) {
      if (pos >= C.size) st = ZD_E_NOT_ENOUGH_BYTES;
      else { rle |= (uint32_t)blk[pos] << (8 * k); pos++; }
    } else if (mode == M_FSE) {
      if (pos >= C.size) st = ZD_E_EMPTY_SLICE;
      else {
        FwBitsW fw{blk + pos, C.size - pos, 0, r0, r1, (uint32_t)(8 * (blk + pos - wb))};
        uint8_t a = 0;
        st = parse_ncount(fw, &a, W.dist[k], &nsym, 256);
        al = a;
        pos += fw.bytes_read();
      }
    } else if (mode == M_PREDEFINED) {
      al = k == 1 ? 5 : 6;
      nsym = k == 0 ? 36 : (k == 1 ? 29 : 53);
    }
    if (st) { pst = st; psub = k; }
    alp |= (uint32_t)al << (8 * k);
    nsp |= nsym << (9 * k);
  }
  pst = __builtin_amdgcn_readfirstlane(pst);
  psub = __builtin_amdgcn_readfirstlane(psub);
  alp = (uint32_t)__builtin_amdgcn_readfirstlane((int)alp);
  nsp = (uint32_t)__builtin_amdgcn_readfirstlane((int)nsp);
  rle = (uint32_t)__builtin_amdgcn_readfirstlane((int)rle);
  pos = (uint32_t)__builtin_amdgcn_readfirstlane((int)pos);
  k4_sync();
  if (lane == 0) FZT(f, 6);
  // the tables before the first parse failure, in order; a build failure
  // stops the walk there
  int fst = pst, fsub = pst ? psub : 4;
  // (modes packed: an index into C would put it in scratch)
  const uint32_t modes = (uint32_t)C.modes[0] | (uint32_t)C.modes[1] << 8 | (uint32_t)C.modes[2] << 16;
  for (int k = 0; k < 3 && k < psub; k++) {
    const int mode = (int)((modes >> (8 * k)) & 255);
    const int al = (int)((alp >> (8 * k)) & 255);
    const uint32_t nsym = (nsp >> (9 * k)) & 511;
    int st = 0;
    if (mode == M_RLE) {
      if (lane == 0) W.tab[k][0] = fse_entry((rle >> (8 * k)) & 255, 1);   // AL 0: nb 0, baseline 0
    } else if (mode == M_FSE || mode == M_PREDEFINED) {
      if (mode == M_PREDEFINED) {
        const int16_t* d = k == 0 ? c_ll_default : (k == 1 ? c_of_default : c_ml_default);
        for (uint32_t x = lane; x < nsym; x += 64) W.dist[k][x] = d[x];
        k4_sync();
      }
      st = fz_build_fse(al, W.dist[k], nsym, W.tab[k], W, lane);
    }
    if (st) { fst = st; fsub = k; break; }
  }
  k4_sync();
  if (lane == 0) FZT(f, 7);
  if (!fst && pos >= C.size) { fst = ZD_E_EMPTY_SLICE; fsub = 3; }   // seq.bitstream of the empty rest
  const uint32_t bo = fsub >= 3 ? pos : 0u;
  const uint32_t bsz = fsub >= 3 && pos < C.size ? C.size - pos : 0u;
  const int dst[3] = {0, K3_TL + K3_TM, K3_TL};      // wave 0's LL | ML | OF
  const int cap[3] = {K3_TL, K3_TO, K3_TM};
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int mode = (int)((modes >> (8 * k)) & 255);
    if (fsub <= k || mode == M_REPEAT) continue;
    const int al = (int)((alp >> (8 * k)) & 255);
    const int cnt = mode == M_RLE ? 1 : 1 << al;
    uint16_t* g = fses + (uint64_t)C.fse_slot * FSE_SLOT + k * FSE_TAB;
    for (int e = lane; e < cnt; e += 64) {
      const uint32_t v = W.tab[k][e];
      g[e] = (uint16_t)v;
      if (k3tab && cnt <= cap[k]) k3tab[dst[k] + e] = (uint16_t)K3_ENTRY(v, k, al);
    }
    if (lane == 0) cstate[ci].al[k] = (uint8_t)al;
  }
  if (lane == 0) {
    cstate[ci].bs_off = bo;
    cstate[ci].bs_size = bsz;
    if (fst) key_min(fstate, C.frame, make_key(PH_PARSE, C.block_in_frame, PS_SEQ_TABLES, (uint32_t)fsub, fst));
    I.al = alp;
    I.err = fst ? ((uint32_t)fsub << 8) | (uint32_t)((-fst) & 0xFF) : 0u;
    I.bo = bo;
    I.bsz = bsz;
  }
}

// K1's sequence half for plans of few blocks (zd_k_tables PART 2 there is
// one round of serial lanes, 0.25 ms for C3's 763 blocks): one wave per
// block, fz_tables' walk and wave-parallel builds, the same slot, CompState
// bytes and keys.
__global__ __launch_bounds__(64) void zd_k_tables_seqw(const uint8_t* __restrict__ src,
                                                       const CompBlock* __restrict__ comp, CompState* cstate,
                                                       FrameState* fstate, const uint32_t* __restrict__ list,
                                                       uint32_t n_list, uint16_t* fses) {
  __shared__ __attribute__((aligned(16))) FzK1 W;
  __shared__ FzInfo I;
  const uint32_t ci = (uint32_t)__builtin_amdgcn_readfirstlane((int)list[blockIdx.x]);
  const CompBlock C = comp[ci];
  if (C.prebuilt || C.nseq == 0 || C.host_stage <= PS_SEQ_TABLES) return;
  fz_tables(src, C, ci, cstate, fstate, fses, W, nullptr, I, (int)threadIdx.x, C.frame);
}

// (measured on C3, within noise: the chain wave at s_setprio 3; eight waves
// so the chain wave has a SIMD to itself; publishing every 32 records)
constexpr int FZ_FRAMES = 4;
constexpr int FZ_WAVES = 1 + FZ_FRAMES;
// LAT: the chains as K3L, one wave per frame (waves 0 .. FZ_FRAMES - 1; the
// K4 waves after them), the tables converted from the K3 format in LDS
template <bool LAT>
__global__ __launch_bounds__(64 * (LAT ? 2 * FZ_FRAMES : FZ_WAVES)) void zd_k_fused(
    const uint8_t* __restrict__ src, uint8_t* outbase, const FrameDesc* __restrict__ frames, FrameState* fstate,
    const BlockRec* __restrict__ blocks, const CompBlock* __restrict__ comp, CompState* cstate,
    const uint8_t* __restrict__ lits, uint64_t* __restrict__ seqs, uint16_t* __restrict__ fses,
    uint32_t n_frames, const uint32_t* k2done, uint32_t k2need, uint8_t* redo) {
  __shared__ __attribute__((aligned(4096))) uint64_t ltabs[LAT ? FZ_FRAMES : 1][LAT ? 12288 / 8 : 1];
  __shared__ __attribute__((aligned(16))) uint16_t tabs[FZ_FRAMES * K3_TAB];
  __shared__ __attribute__((aligned(16))) uint8_t win[FZ_FRAMES][K4_WPAD + K4_C];
  __shared__ __attribute__((aligned(16))) uint8_t pat[FZ_FRAMES][64];
  __shared__ __attribute__((aligned(16))) uint8_t stab[FZ_FRAMES][3 * FSE_TAB];
  __shared__ __attribute__((aligned(16))) uint8_t stg[FZ_FRAMES][K4_STG + 16];
  __shared__ uint32_t codelut[FZ_FRAMES][2 * 64];
  __shared__ uint32_t prog[FZ_FRAMES], trdy[FZ_FRAMES];
  __shared__ __attribute__((aligned(16))) FzK1 k1w[FZ_FRAMES];
  __shared__ FzInfo info[FZ_FRAMES];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (threadIdx.x < FZ_FRAMES) prog[threadIdx.x] = trdy[threadIdx.x] = 0;
  __syncthreads();
  constexpr int NCH = LAT ? FZ_FRAMES : 1;      // chain waves
  if (wave >= NCH) {
    // (readfirstlane: the compiler sees the frame as wave-uniform, so the
    // table walk below runs on the scalar unit)
    const int q = __builtin_amdgcn_readfirstlane(wave - NCH);
    const uint32_t f = blockIdx.x * FZ_FRAMES + q;
    if (f >= n_frames) return;
    if (lane == 0) FZT(f, 8);
    {
      // the block's sequence tables (the window is free until the waits)
      const FrameDesc F = frames[f];
      const int32_t c = F.nblocks ? blocks[F.first_block].comp : -1;
      bool build = false;
      CompBlock C;
      if (c >= 0) {
        C = comp[c];
        build = C.nseq > 0 && C.host_stage > PS_SEQ_TABLES && !C.prebuilt;
      }
      if (build) {
        fz_tables(src, C, (uint32_t)c, cstate, fstate, fses, k1w[q], (lds_u16*)tabs + q * K3_TAB, info[q], lane, f);
      } else if (lane == 0) {
        info[q] = FzInfo{0u, 0u, 0u, 0u};
      }
      // tables, CompState bytes and key in place before trdy (wave 0 and
      // this wave's k4f_wait_k2 acquire after it)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) *(volatile uint32_t*)&trdy[q] = 1;
      if (lane == 0) FZT(f, 1);
      k4_sync();
    }
    const K4Lds M{(l_u8*)win[q] + K4_WPAD, (l_u8*)pat[q], (l_u8*)stab[q], (l_u8*)stg[q], (l_u32*)codelut[q]};
    const K4Fuse z{(const volatile l_u32*)&prog[q], (const volatile l_u32*)&trdy[q], k2done, k2need, f};
    k4_body<true>(src, outbase, frames, fstate, blocks, comp, cstate, lits, seqs, fses, f, f + 1, 1, nullptr, M, &z,
                  redo);
    return;
  }
  if constexpr (LAT) {
    // wave q: frame q's chain (K3L), at the SIMD's issue priority over the K4 wave beside it
    const int q = __builtin_amdgcn_readfirstlane(wave);
    const uint32_t f = blockIdx.x * FZ_FRAMES + q;
    if (f >= n_frames) return;
    if (lane == 0) FZT(f, 0);
    const FrameDesc F = frames[f];
    const int32_t c = F.nblocks ? blocks[F.first_block].comp : -1;
    const uint32_t ci = c >= 0 ? (uint32_t)c : 0;
    CompBlock C;
    if (c >= 0) C = comp[ci];
    const uint64_t key0 = fstate[f].key;
    bool ready = false;
    for (uint32_t it = 0; it < (1u << 22) && !ready; it++) {
      ready = *(volatile uint32_t*)&trdy[q] != 0;
      if (!ready) __builtin_amdgcn_s_sleep(ZD_FZ_SLEEP);
    }
    asm volatile("" ::: "memory");
    const FzInfo I = info[q];
    const int al[3] = {(int)(I.al & 255), (int)((I.al >> 8) & 255), (int)((I.al >> 16) & 255)};
    const bool build = c >= 0 && C.nseq > 0 && C.host_stage > PS_SEQ_TABLES && !C.prebuilt;
    const bool act = ready && build && I.err == 0 && C.tab_src[0] == c && C.tab_src[1] == c && C.tab_src[2] == c &&
                     !(key0 != KEY_NONE && key_phase(key0) == PH_PARSE) && al[1] <= 8;
    int rej = ready ? 0 : 1;
    if (ready && build && I.err == 0 && !act && !(key0 != KEY_NONE && key_phase(key0) == PH_PARSE)) rej = 1;
    if (act) {
      // the K3-format entries (nextState | count << 10, K3F_BAD) -> K3L's
      const uint32_t tb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint64_t*)ltabs[q];
      const lds_u16* t16 = (const lds_u16*)tabs + q * K3_TAB;
      for (int k = 0; k < 3; k++) {
        const int a = al[k];
        const lds_u16* tk = t16 + (k == 0 ? 0 : k == 2 ? K3_TL : K3_TL + K3_TM);
        const uint32_t t = tb + (k == 0 ? 0u : k == 2 ? K3L_ML : K3L_OF);
        for (int e = lane; e < (1 << a); e += 64) {
          const uint32_t x = tk[e], ns = x & 1023, cnt = x >> 10;
          const bool bad = cnt == 63 || ns == 0 || hb32(ns) > a;
          const uint32_t nb = bad ? 0u : (uint32_t)(a - hb32(ns));
          const uint32_t lo = bad ? (1u << 16) : (nb | (cnt << 8));
          const uint32_t hi = t + 8 * (bad ? 0u : (ns << nb) - (1u << a));
          *(lds_u64*)(uintptr_t)(t + 8 * e) = (uint64_t)lo | ((uint64_t)hi << 32);
        }
      }
      k4_sync();
      __builtin_amdgcn_s_setprio(3);
      if (lane == 0) FZT(f, 5);
      rej = seq_chainl<true>(src + C.src + I.bo, I.bsz, (uintptr_t)src, tb, al[0], al[1], al[2], C.nseq,
                             seqs + C.seq_out, (volatile lds_u32*)&prog[q]);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) FZT(f, 2);
    if (lane == 0) {
      if (rej) redo[f] = 1;
      *(volatile uint32_t*)&prog[q] = rej ? K4F_PROG_ABANDON : K4F_PROG_FINAL;
    }
    return;
  }
  // wave 0: the chains (quad q: frame blockIdx.x * FZ_FRAMES + q)
  const int role = lane & 3, q = lane >> 2;
  const uint32_t f = blockIdx.x * FZ_FRAMES + q;
  const bool mine = q < FZ_FRAMES && f < n_frames;
  const int q4 = q < FZ_FRAMES ? q : 0;
  if (mine && role == 0) FZT(f, 0);
  int32_t c = -1;
  if (mine) {
    const FrameDesc F = frames[f];
    c = F.nblocks ? blocks[F.first_block].comp : -1;
  }
  const uint32_t ci = c >= 0 ? (uint32_t)c : 0;
  CompBlock C;
  if (c >= 0) C = comp[ci];
  const uint64_t key0 = mine ? fstate[f].key : KEY_NONE;
  // the tables from the K4 waves
  bool ready = false;
  for (uint32_t it = 0; it < (1u << 22) && !ready; it++) {
    ready = __ballot(mine && *(volatile uint32_t*)&trdy[q4] == 0) == 0;
    if (!ready) __builtin_amdgcn_s_sleep(ZD_FZ_SLEEP);
  }
  asm volatile("" ::: "memory");
  FzInfo I = FzInfo{0u, 0u, 0u, 0u};
  if (mine) I = info[q4];
  const int al[3] = {(int)(I.al & 255), (int)((I.al >> 8) & 255), (int)((I.al >> 16) & 255)};
  const bool build = c >= 0 && C.nseq > 0 && C.host_stage > PS_SEQ_TABLES && !C.prebuilt;
  // the blocks zd_k_sequences_q would run (list_seq, and its PH_PARSE skip),
  // on this block's own tables (a table from another block: the redo pass)
  bool act = ready && build && I.err == 0 && C.tab_src[0] >= 0 && C.tab_src[1] >= 0 && C.tab_src[2] >= 0 &&
             !(key0 != KEY_NONE && key_phase(key0) == PH_PARSE);
  int rej = mine && !ready ? 1 : 0;
  if (act && (C.tab_src[0] != c || C.tab_src[1] != c || C.tab_src[2] != c)) { act = false; rej = 1; }
  const bool use_lds = __ballot(act && al[1] > 8) == 0;
  lds_u16* mine_t = (lds_u16*)tabs + q4 * K3_TAB;
  if (mine && role == 0) FZT(f, 5);
  if (act) {
    if (use_lds) {
      const lds_u16* tab = role == 0 ? mine_t + K3_TL + K3_TM : role == 1 ? mine_t + K3_TL : mine_t;
      rej = seq_chainq<ZD_K3_LA, ZD_K3_WN, true>(src + C.src + I.bo, I.bsz, (uintptr_t)src, tab, role,
                                                 al[0], al[1], al[2], C.nseq, seqs + C.seq_out,
                                                 (volatile __attribute__((address_space(3))) uint32_t*)&prog[q]);
    } else {
      rej = 1;                                   // OF tables deeper than LDS holds: the redo pass
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (mine && role == 0) FZT(f, 2);
  if (mine && role == 0) {
    if (rej) redo[f] = 1;
    *(volatile uint32_t*)&prog[q] = rej ? K4F_PROG_ABANDON : K4F_PROG_FINAL;
  }
}

// ---------------------------------------------------------------------------
// K4F: execute with the whole frame resident in LDS (decoding_context.rs:
// 50-106 + block.rs:74-99), for frames whose output fits K4F_CAP (every
// 128 KiB single-segment frame).  One 1024-thread workgroup per frame; a
// block's sequences go in chunks of K4F_T x K4F_KC, each thread owning
// K4F_KC consecutive sequences:
//   values   records (K3) -> symbols (LDS) + extra bits (bitstream window)
//   offsets  decode_offset as an exclusive scan of the threads' repeat maps
//            (zd_common.h rep codes), then a concrete walk per thread
//   places   exclusive scans of literal/total lengths
//   checks   the first failing sequence of the chunk (min over threads),
//            reference order: decode_offset, ImpossibleValue, zero offset
//   literals every run copied into the LDS frame at once
//   matches  in rounds: a match copies once every byte of its source is
//            written (1 bit per frame byte in LDS); each round completes at
//            least the earliest pending match, typically 3-4 rounds in all
// The frame never leaves LDS until it is complete: no HBM re-reads of match
// sources, and one coalesced write of the frame at the end.
// ---------------------------------------------------------------------------
constexpr int K4F_T = 1024;
constexpr int K4F_W = K4F_T / 64;
#ifndef ZD_K4F_KC
#define ZD_K4F_KC 4
#endif
constexpr int K4F_KC = ZD_K4F_KC;
constexpr uint32_t K4F_CHUNK = (uint32_t)K4F_T * K4F_KC;
constexpr uint32_t K4F_LIST = 1024;
struct K4FShared {
  uint8_t buf[K4F_CAP + 64];
  uint32_t bits[K4F_CAP / 32 + 4];     // 1 = byte written (or not a pending match byte)
  uint8_t stab[3][FSE_TAB];            // LL | OF | ML symbols of the block
  uint32_t wmap[K4F_W][3];             // per-wave repeat maps, then their exclusive prefixes
  uint32_t wsum[K4F_W][2];             // per-wave length sums, then their exclusive prefixes
  uint64_t rep[2][3];                  // concrete repeat offsets into a chunk (double-buffered)
  unsigned long long err, lim;         // first failing sequence of the chunk
  uint32_t tot[2];                     // chunk output / literal totals
  uint32_t lq[K4F_LIST], lo[K4F_LIST], lm[K4F_LIST];   // matches left after the parallel round, in order
};

__device__ inline void k4f_bits_and(uint32_t* bits, uint32_t p, uint32_t n, bool set) {
  uint32_t w = p >> 5, e = p + n;
  while (p < e) {
    const uint32_t lo = p & 31, hi = min(32u, lo + (e - p));
    const uint32_t m = (hi == 32 ? ~0u : ((1u << hi) - 1)) & ~((1u << lo) - 1);
    if (set) atomicOr(&bits[w], m);
    else atomicAnd(&bits[w], ~m);
    p += hi - lo;
    w++;
  }
}
__device__ inline bool k4f_bits_all(const uint32_t* bits, uint32_t p, uint32_t n) {
  const uint32_t e = p + n;
  while (p < e) {
    const uint32_t lo = p & 31, hi = min(32u, lo + (e - p));
    const uint32_t m = (hi == 32 ? ~0u : ((1u << hi) - 1)) & ~((1u << lo) - 1);
    if ((bits[p >> 5] & m) != m) return false;
    p += hi - lo;
  }
  return true;
}
// wave-inclusive scan of a repeat map (lanes < d keep theirs)
__device__ inline void k4f_scan_map(uint32_t m[3], int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t a[3];
    a[0] = (uint32_t)__shfl_up((int)m[0], d, 64);
    a[1] = (uint32_t)__shfl_up((int)m[1], d, 64);
    a[2] = (uint32_t)__shfl_up((int)m[2], d, 64);
    if (lane >= d) rc_compose(a, m);
  }
}

// One match: ml bytes at q from q - o (overlap-safe, decoding_context.rs:95-98).
__device__ inline void k4f_match(l_u8* buf, uint32_t q, uint32_t o, uint32_t mk) {
  l_u8* d = buf + q;
  const l_u8* sp = buf + q - o;
  if (o >= 16) {
    for (uint32_t x = 0; x < mk; x += 16) sts_n(d + x, lds16(sp + x), mk - x);
  } else {                                        // small period: 16 bytes bytewise, then 16-byte steps
    const uint32_t m16 = o * ((16 + o - 1) / o);
    const uint32_t head = mk < 16 ? mk : 16;
    uint32_t r = 0;
    for (uint32_t x = 0; x < head; x++) {
      d[x] = sp[r];
      r = r + 1 == o ? 0 : r + 1;
    }
    for (uint32_t x = 16; x < mk; x += 16) sts_n(d + x, lds16(d + x - m16), mk - x);
  }
}
struct K4FShared;
// The matches the parallel round left, in sequence order, by one wave: 64 at
// a time in frontier rounds (a match copies once its source lies below the
// first unfinished match of the batch; everything before the batch is done).
template <typename SH>
__device__ inline void k4f_ordered(SH& L, uint32_t cnt, int lane) {
  for (uint32_t b = 0; b < cnt; b += 64) {
    const uint32_t i = b + lane;
    const bool v = i < cnt;
    const uint32_t q = v ? L.lq[i] : 0, o = v ? L.lo[i] : 1, mk = v ? L.lm[i] : 0;
    const uint32_t shi = q - o + (o < mk ? o : mk);
    uint64_t done = __ballot(!v);
    while (done != ~0ull) {
      const int U = __ffsll((long long)~done) - 1;
      const uint32_t qU = (uint32_t)__builtin_amdgcn_readlane((int)q, U);
      const bool mine = !((done >> lane) & 1) && (lane == U || shi <= qU);
      if (mine) k4f_match((l_u8*)L.buf, q, o, mk);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      done |= __ballot(mine);
    }
  }
}

__global__ __launch_bounds__(K4F_T) void zd_k_execute_lds(const uint8_t* __restrict__ src, uint8_t* outbase,
                                                          const FrameDesc* __restrict__ frames, FrameState* fstate,
                                                          const BlockRec* __restrict__ blocks,
                                                          const CompBlock* __restrict__ comp,
                                                          const CompState* __restrict__ cstate,
                                                          const uint8_t* __restrict__ lits,
                                                          const uint64_t* __restrict__ seqs,
                                                          const uint16_t* __restrict__ fses,
                                                          const uint32_t* __restrict__ flist) {
  __shared__ __attribute__((aligned(16))) K4FShared L;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t f = flist[blockIdx.x];
  const FrameDesc F = frames[f];
  FrameState* S = &fstate[f];
  const uint64_t key0 = S->key;
  if (key0 != KEY_NONE && key_phase(key0) == PH_PARSE) return;
  const uint32_t cap = (uint32_t)(F.out_cap < K4F_CAP ? F.out_cap : K4F_CAP);
  for (uint32_t x = t; x < K4F_CAP / 32 + 4; x += K4F_T) L.bits[x] = ~0u;
  if (t == 0) { L.rep[0][0] = S->rep[0]; L.rep[0][1] = S->rep[1]; L.rep[0][2] = S->rep[2]; }
  int rb = 0;                                     // which rep buffer holds the current state
  uint32_t pos = 0;                               // frame bytes produced (uniform)
  uint64_t err_key = KEY_NONE;
  __syncthreads();

  for (uint32_t j = 0; j < F.nblocks; j++) {
    const BlockRec B = blocks[F.first_block + j];
    // a decode error found before (K2), or a limit the plan found (a frame
    // past the int32 positions: block 0), ends the frame at its block
    if (key0 != KEY_NONE && key_phase(key0) != PH_PARSE && key_block(key0) <= j) break;
    if (B.type == 5) continue;
    if (B.type != 2) {                            // raw / RLE / skippable payload
      if ((uint64_t)pos + B.size > cap) { err_key = make_key(PH_LIMIT, j, LS_CAPACITY, 0, ZD_E_OUT_OF_DOMAIN); break; }
      const uint32_t fill = B.rle * 0x01010101u;
      const u32x4 f4 = (u32x4){fill, fill, fill, fill};
      for (uint32_t x = 16 * t; x < B.size; x += 16 * K4F_T) {
        const u32x4 v = B.type == 1 ? f4 : ldg16(src + B.src + x);
        sts_n((l_u8*)L.buf + pos + x, v, min(16u, B.size - x));
      }
      pos += B.size;
      __syncthreads();
      continue;
    }
    const CompBlock C = comp[B.comp];
    const CompState CS = cstate[B.comp];
    if (CS.stop) break;
    const uint8_t* lsrc = nullptr;
    uint32_t lfill = 0, nl;
    if (C.lit_type == LIT_RAW) { lsrc = src + C.src + C.lit_data; nl = C.lit_regen; }
    else if (C.lit_type == LIT_RLE) { lfill = C.lit_rle * 0x01010101u; nl = C.lit_regen; }
    else { lsrc = lits + C.lit_out; nl = CS.lit_count; }
    const u32x4 f4 = (u32x4){lfill, lfill, lfill, lfill};
    const uint32_t n = C.nseq;
    const bool direct = C.seq_direct != 0;
    const uint64_t* SQ = seqs + C.seq_out;
    const uint8_t* bsp = src + C.src + CS.bs_off;
    if (n && !direct) {
      for (int k = 0; k < 3; k++) {
        const uint32_t s = (uint32_t)C.tab_src[k];
        const uint16_t* g = fses + (uint64_t)comp[s].fse_slot * FSE_SLOT + k * FSE_TAB;
        const int cnt = 1 << cstate[s].al[k];
        for (int e = t; e < cnt; e += K4F_T) L.stab[k][e] = (uint8_t)(g[e] & 63);
      }
    }
    uint32_t lit_cursor = 0;
    __syncthreads();
    for (uint32_t c0 = 0; c0 < n; c0 += K4F_CHUNK) {
      const uint32_t cn = min(K4F_CHUNK, n - c0);
      const uint32_t b0 = (uint32_t)t * K4F_KC;
#ifdef ZD_K4F_PROF
      uint64_t tp[8]; int np = 0, rounds = 0;
      tp[np++] = __builtin_amdgcn_s_memtime();
#endif
      uint32_t ll[K4F_KC], ml[K4F_KC], oc[K4F_KC];
      // values (update_symbol_value, decoders/sequence.rs:41-55)
#pragma unroll
      for (int k = 0; k < K4F_KC; k++) {
        ll[k] = 0; ml[k] = 0; oc[k] = 4;          // padding: no bytes, a fresh offset
        if (b0 + k < cn) {
          const uint64_t sq = rec_get(SQ, c0 + b0 + k, direct);
          if (direct) {
            seq_values(sq, C.seq_side, c0 + b0 + k, &ll[k], &ml[k], &oc[k]);
          } else {
            const int32_t bp = (int32_t)(uint32_t)sq;
            const uint32_t stt = (uint32_t)(sq >> 32);
            const uint32_t llc = L.stab[0][stt & 1023], mlc = L.stab[2][(stt >> 10) & 1023];
            const uint32_t ofc = L.stab[1][stt >> 20] & 31;
            uint32_t llbase, llb, mlbase, mlb;
            ll_code(llc, &llbase, &llb);
            ml_code(mlc, &mlbase, &mlb);
            uint64_t tt = winu_top(winu_load(bsp, (uintptr_t)src, bp), 0);
            const uint32_t ob = take_top(tt, ofc), mb = take_top(tt, mlb), lb = take_top(tt, llb);
            oc[k] = (1u << ofc) + ob;             // offset_value for now
            ml[k] = mlbase + mb;
            ll[k] = llbase + lb;
          }
        }
      }
      // decode_offset (decoding_context.rs:50-75): this thread's map of the
      // repeat offsets, scanned over the workgroup
      uint32_t m[3];
      rep_ident(m);
#pragma unroll
      for (int k = 0; k < K4F_KC; k++) (void)rep_step(m, oc[k], ll[k]);
      k4f_scan_map(m, lane);
#ifdef ZD_K4F_PROF
      tp[np++] = __builtin_amdgcn_s_memtime();
#endif
      uint32_t ex[3];
      ex[0] = (uint32_t)__shfl_up((int)m[0], 1, 64);
      ex[1] = (uint32_t)__shfl_up((int)m[1], 1, 64);
      ex[2] = (uint32_t)__shfl_up((int)m[2], 1, 64);
      if (lane == 0) rep_ident(ex);
      // lengths: this thread's sums, scanned the same way
      uint32_t stot = 0, slit = 0;
#pragma unroll
      for (int k = 0; k < K4F_KC; k++) { stot += ll[k] + ml[k]; slit += ll[k]; }
      uint32_t it = stot, il = slit;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t a = (uint32_t)__shfl_up((int)it, d, 64), b = (uint32_t)__shfl_up((int)il, d, 64);
        if (lane >= d) { it += a; il += b; }
      }
      if (lane == 63) {
        L.wmap[wv][0] = m[0]; L.wmap[wv][1] = m[1]; L.wmap[wv][2] = m[2];
        L.wsum[wv][0] = it; L.wsum[wv][1] = il;
      }
      if (t == 0) { L.err = ~0ull; L.lim = ~0ull; }
      __syncthreads();
      if (wv == 0) {                              // exclusive prefixes over the waves
        uint32_t wm[3] = {OFF_SYM, OFF_SYM | (1u << 24), OFF_SYM | (2u << 24)};
        uint32_t w0 = 0, w1 = 0;
        if (lane < K4F_W) { wm[0] = L.wmap[lane][0]; wm[1] = L.wmap[lane][1]; wm[2] = L.wmap[lane][2];
                            w0 = L.wsum[lane][0]; w1 = L.wsum[lane][1]; }
        k4f_scan_map(wm, lane);
        uint32_t i0 = w0, i1 = w1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t a = (uint32_t)__shfl_up((int)i0, d, 64), b = (uint32_t)__shfl_up((int)i1, d, 64);
          if (lane >= d) { i0 += a; i1 += b; }
        }
        uint32_t pm[3];
        pm[0] = (uint32_t)__shfl_up((int)wm[0], 1, 64);
        pm[1] = (uint32_t)__shfl_up((int)wm[1], 1, 64);
        pm[2] = (uint32_t)__shfl_up((int)wm[2], 1, 64);
        if (lane == 0) rep_ident(pm);
        if (lane == K4F_W - 1) { L.tot[0] = i0; L.tot[1] = i1; }
        __builtin_amdgcn_wave_barrier();
        if (lane < K4F_W) {
          L.wmap[lane][0] = pm[0]; L.wmap[lane][1] = pm[1]; L.wmap[lane][2] = pm[2];
          L.wsum[lane][0] = i0 - w0; L.wsum[lane][1] = i1 - w1;
        }
      }
      __syncthreads();
      // the concrete state before this thread's sequences
#ifdef ZD_K4F_PROF
      tp[np++] = __builtin_amdgcn_s_memtime();
#endif
      uint32_t st3[3];
      {
        const uint32_t wp[3] = {L.wmap[wv][0], L.wmap[wv][1], L.wmap[wv][2]};
        rc_compose(wp, ex);                       // ex: chunk input -> before this thread
        const uint32_t in[3] = {rep_code(L.rep[rb][0]), rep_code(L.rep[rb][1]), rep_code(L.rep[rb][2])};
        st3[0] = rc_apply(ex[0], in); st3[1] = rc_apply(ex[1], in); st3[2] = rc_apply(ex[2], in);
      }
#pragma unroll
      for (int k = 0; k < K4F_KC; k++) oc[k] = rep_step(st3, oc[k], ll[k]);   // offset codes, concrete
      const uint32_t pbase = pos + L.wsum[wv][0] + (it - stot);      // frame position of the first literal
      const uint32_t lbase = lit_cursor + L.wsum[wv][1] + (il - slit);
      const uint32_t ctot = L.tot[0], clit = L.tot[1];
      if (cn - 1 >= b0 && cn - 1 < b0 + K4F_KC) {  // the chunk's last sequence: state out
        L.rep[rb ^ 1][0] = rep_value(st3[0]); L.rep[rb ^ 1][1] = rep_value(st3[1]); L.rep[rb ^ 1][2] = rep_value(st3[2]);
      }
      // checks (decoding_context.rs:84-90, D9) in sequence order
      {
        uint32_t p = pbase, lp = lbase;
        unsigned long long e = ~0ull, lim = ~0ull;
#pragma unroll
        for (int k = 0; k < K4F_KC; k++) {
          if (b0 + k < cn) {
            const uint32_t o = oc[k];
            int code = 0;
            if (o == OFF_NULL) code = ZD_E_NULL_OFFSET;
            else if (o == OFF_UNDERFLOW) code = ZD_E_REF_PANIC;
            else if ((uint64_t)lp + ll[k] > nl || (uint64_t)o > (uint64_t)p + ll[k]) code = ZD_E_IMPOSSIBLE_VALUE;
            else if (ml[k] != 0 && o == 0) code = ZD_E_REF_PANIC;
            const unsigned long long idx = c0 + b0 + k;
            if (code && e == ~0ull) e = (idx << 8) | (uint32_t)(-code);
            if ((uint64_t)p + ll[k] + ml[k] > cap && lim == ~0ull) lim = idx;
          }
          p += ll[k] + ml[k];
          lp += ll[k];
        }
        if (e != ~0ull) atomicMin(&L.err, e);
        if (lim != ~0ull) atomicMin(&L.lim, lim);
      }
      __syncthreads();
      if (L.err != ~0ull || L.lim != ~0ull) {
        if (L.err != ~0ull) err_key = make_key(PH_DECODE, j, DS_EXECUTE, (uint32_t)(L.err >> 8), -(int)(L.err & 0xFF));
        else err_key = make_key(PH_LIMIT, j, LS_CAPACITY, (uint32_t)L.lim, ZD_E_OUT_OF_DOMAIN);
        break;
      }
#ifdef ZD_K4F_PROF
      tp[np++] = __builtin_amdgcn_s_memtime();
#endif
      // match bytes start unwritten; literal runs go in at once
      {
        uint32_t p = pbase, lp = lbase;
#pragma unroll
        for (int k = 0; k < K4F_KC; k++) {
          if (ml[k]) k4f_bits_and(L.bits, p + ll[k], ml[k], false);
          for (uint32_t x = 0; x < ll[k]; x += 16) {
            const u32x4 v = lsrc ? ldg16(lsrc + lp + x) : f4;
            sts_n((l_u8*)L.buf + p + x, v, ll[k] - x);
          }
          p += ll[k] + ml[k];
          lp += ll[k];
        }
      }
      __syncthreads();
      // matches in rounds
      uint32_t pend = 0;
#ifdef ZD_K4F_PROF
      tp[np++] = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
      for (int k = 0; k < K4F_KC; k++) pend |= (ml[k] != 0 ? 1u : 0u) << k;
      // Parallel rounds while more matches wait than the ordered list holds
      // (normally one round), then the rest in sequence order by one wave.
      for (;;) {
#ifdef ZD_K4F_PROF
        rounds++;
#endif
        uint32_t q = pbase;
#pragma unroll
        for (int k = 0; k < K4F_KC; k++) {
          q += ll[k];
          if ((pend >> k) & 1) {
            const uint32_t o = oc[k], mk = ml[k];
            if (k4f_bits_all(L.bits, q - o, o < mk ? o : mk)) {
              k4f_match((l_u8*)L.buf, q, o, mk);
              __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the bytes land before their bits
              k4f_bits_and(L.bits, q, mk, true);
              pend &= ~(1u << k);
            }
          }
          q += ml[k];
        }
        // ordered list slots: exclusive scan of the pending counts
        const uint32_t c = (uint32_t)__popc(pend);
        uint32_t ic = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const uint32_t y = (uint32_t)__shfl_up((int)ic, d, 64);
          if (lane >= d) ic += y;
        }
        if (lane == 63) L.wsum[wv][0] = ic;
        __syncthreads();
        uint32_t wb = 0, all = 0;
        for (int w = 0; w < K4F_W; w++) {
          const uint32_t x = L.wsum[w][0];
          wb += w < wv ? x : 0;
          all += x;
        }
        if (all <= K4F_LIST) {
          uint32_t slot = wb + ic - c;
          uint32_t q2 = pbase;
#pragma unroll
          for (int k = 0; k < K4F_KC; k++) {
            q2 += ll[k];
            if ((pend >> k) & 1) {
              L.lq[slot] = q2; L.lo[slot] = oc[k]; L.lm[slot] = ml[k];
              slot++;
            }
            q2 += ml[k];
          }
          __syncthreads();
          if (wv == 0) k4f_ordered(L, all, lane);
          break;
        }
        __syncthreads();
      }
      __syncthreads();
      // every byte of the chunk is written now
      {
        const uint32_t w0 = pos >> 5, w1 = (pos + ctot + 31) >> 5;
        for (uint32_t w = w0 + t; w < w1; w += K4F_T) L.bits[w] = ~0u;
      }
      pos += ctot;
      lit_cursor += clit;
#ifdef ZD_K4F_PROF
      tp[np++] = __builtin_amdgcn_s_memtime();
      if (t == 0 && blockIdx.x < 2)
        printf("K4F wg %u chunk %u cn %u: dec %llu scan %llu chk %llu lit %llu match %llu rounds %d\n", blockIdx.x, c0, cn,
               (unsigned long long)(tp[1] - tp[0]), (unsigned long long)(tp[2] - tp[1]), (unsigned long long)(tp[3] - tp[2]),
               (unsigned long long)(tp[4] - tp[3]), (unsigned long long)(tp[5] - tp[4]), rounds);
#endif
      rb ^= 1;
      __syncthreads();
    }
    if (err_key != KEY_NONE) break;
    // leftover literals (decoding_context.rs:101-103)
    if (lit_cursor < nl) {
      const uint32_t rest = nl - lit_cursor;
      if ((uint64_t)pos + rest > cap) { err_key = make_key(PH_LIMIT, j, LS_CAPACITY, n, ZD_E_OUT_OF_DOMAIN); break; }
      for (uint32_t x = 16 * t; x < rest; x += 16 * K4F_T) {
        const u32x4 v = lsrc ? ldg16(lsrc + lit_cursor + x) : f4;
        sts_n((l_u8*)L.buf + pos + x, v, min(16u, rest - x));
      }
      pos += rest;
    }
    __syncthreads();
  }
  if (err_key != KEY_NONE) {
    if (t == 0) key_min(fstate, f, err_key);
    return;
  }
  // the frame -> HBM: aligned 16-byte stores, head and tail bytewise
  uint8_t* out = outbase + F.out;
  const uintptr_t oa = (uintptr_t)out;
  const uint32_t head = (uint32_t)(((oa + 15) & ~(uintptr_t)15) - oa);
  const uint32_t h = head < pos ? head : pos;
  if ((uint32_t)t < h) out[t] = L.buf[t];
  for (uint32_t x = h + 16 * t; x + 16 <= pos; x += 16 * K4F_T) *(g_u32x4*)(out + x) = lds16((const l_u8*)L.buf + x);
  const uint32_t tail0 = pos > h ? h + ((pos - h) & ~15u) : pos;
  if (tail0 + t < pos) out[tail0 + t] = L.buf[tail0 + t];
  if (t == 0) {
    S->out_len = pos;
    S->rep[0] = L.rep[rb][0];
    S->rep[1] = L.rep[rb][1];
    S->rep[2] = L.rep[rb][2];
  }
}

// ---------------------------------------------------------------------------
// K4J: execute of frames of many blocks, block-parallel (decoding_context.rs:
// 50-106 + block.rs:74-99).  The streaming K4 runs a frame's sequences in
// order on one wave: a 100 MB frame (the stock `zstd enwik8` shape) is ~11 M
// sequences one batch after another.  K4J takes the frame's serial
// dependencies apart:
//   KJ1 zd_k_jsum     one wave per J_SEG sequences of a block: the segment's
//                     output and literal bytes and its repeat-offset map
//                     (decode_offset as a function of the three offsets coming
//                     in, jr codes); then zd_k_jsum_blocks, one lane per block,
//                     turns its segments' sums into checkpoints (JSeg: the
//                     bytes and map before each segment) and gives the block's
//                     output size (literals + match lengths) and map
//   KJ2 zd_k_jprefix  one wave per frame: scans over the blocks give each
//                     block's output position and the concrete repeat offsets
//                     entering it; the capacity check
//   KJ3 zd_k_jscatter one wave per J_SEG sequences: concrete offsets from the
//                     checkpoint, the reference's checks; every literal byte's
//                     state word is J_FINAL | byte, every match byte's the
//                     distance to the byte it copies (off, plus off per period
//                     passed in an overlapping match: the reference's
//                     byte-by-byte push)
//   KJ4 zd_k_jround   pointer jumping, in place: S[p] = S[p - S[p]] for every
//                     pending word, up to j_hops (6) hops per word and round (a final
//                     source hands over its byte, a pending one adds its
//                     distance), one word per lane.
//                     A chain ends at a literal after at most one hop per
//                     earlier match, and every hop of a round follows pointers
//                     earlier rounds have already shortened: a 100 MB text
//                     frame resolves in 2-3 rounds (the rounds launched for
//                     the deepest possible chain exit at once once nothing is
//                     pending).  Any version of a word is true of its byte,
//                     so lanes need no ordering within a round.  A piece of
//                     16 words is written to the output in the round that
//                     resolves its last word.
// ---------------------------------------------------------------------------
__device__ inline bool j_live(uint64_t key, uint32_t j) {
  // a parse error ends the frame before any block decodes (frame.rs:198-230);
  // a decode error (or a capacity limit) at block b leaves blocks < b to run
  return key == KEY_NONE || (key_phase(key) != PH_PARSE && key_block(key) > j);
}

__device__ inline uint64_t shfl_up_u64(uint64_t x, int d) {
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)x, d, 64);
  const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(x >> 32), d, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint64_t wave_scan_u64(uint64_t x, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = shfl_up_u64(x, d);
    if (lane >= d) x += y;
  }
  return x;
}
// wave-inclusive composition of repeat-offset maps, lane order
__device__ inline void j_scan_map(uint64_t m[3], int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t a[3];
    a[0] = shfl_up_u64(m[0], d);
    a[1] = shfl_up_u64(m[1], d);
    a[2] = shfl_up_u64(m[2], d);
    if (lane >= d) {
      const uint64_t c0 = jr_apply(m[0], a), c1 = jr_apply(m[1], a), c2 = jr_apply(m[2], a);
      m[0] = c0; m[1] = c1; m[2] = c2;
    }
  }
}

// The block's LL/OF/ML symbols (K1's sym entries) -> LDS.
__device__ inline void j_stab(uint8_t (*stab)[FSE_TAB], const CompBlock& C, const CompBlock* __restrict__ comp,
                              const CompState* __restrict__ cstate, const uint16_t* __restrict__ fses, int lane) {
  for (int k = 0; k < 3; k++) {
    const uint32_t s = (uint32_t)C.tab_src[k];
    const uint16_t* g = fses + (uint64_t)comp[s].fse_slot * FSE_SLOT + k * FSE_TAB;
    const int cnt = 1 << cstate[s].al[k];
    for (int e = lane; e < cnt; e += 64) stab[k][e] = (uint8_t)(g[e] & 63);
  }
  k4_sync();
}

// update_symbol_value (decoders/sequence.rs:41-55) from a K3 record: OF, ML,
// LL extra bits below the recorded position, in that order.
__device__ inline void j_values(uint64_t rec, const WinU& w, const uint8_t (*stab)[FSE_TAB], uint32_t& ll,
                                uint32_t& ml, uint32_t& ofv) {
  const uint32_t stt = (uint32_t)(rec >> 32);
  const uint32_t llc = stab[0][stt & 1023], mlc = stab[2][(stt >> 10) & 1023], ofc = stab[1][stt >> 20] & 31;
  uint32_t llbase, llb, mlbase, mlb;
  ll_code(llc, &llbase, &llb);
  ml_code(mlc, &mlbase, &mlb);
  uint64_t t = winu_top(w, 0);
  const uint32_t ob = take_top(t, ofc), mb = take_top(t, mlb), lb = take_top(t, llb);
  ofv = (1u << ofc) + ob;
  ml = mlbase + mb;
  ll = llbase + lb;
}

// decode_offset (decoding_context.rs:50-75) over lanes [0, k) of a batch, in
// order: fresh offsets (offset_value > 3) push their value, the rare repeat
// codes are walked on the scalar unit.  SYM: the state holds jr codes (KJ1's
// maps; no errors: a null offset leaves the state, and the block that holds
// it reports it in KJ3), else concrete values with the reference's errors
// (*bad_lane = the first failing lane, -1 if none).  Returns each lane's
// offset; rep[] becomes the state after lane k - 1.
template <bool SYM>
__device__ inline uint64_t j_offsets(uint32_t ofv, uint32_t ll, int k, uint64_t rep[3], int* bad_lane, int* bad_code) {
  const int lane = threadIdx.x & 63;
  const bool fresh = ofv > 3;
  const uint64_t val = (uint64_t)ofv - 3;
  uint64_t off = val;
  uint64_t rm = __ballot(lane < k && !fresh);
  uint64_t r0 = rep[0], r1 = rep[1], r2 = rep[2];
  int prev = -1;
  *bad_lane = -1;
  *bad_code = 0;
  while (rm) {
    const int ri = __ffsll((long long)rm) - 1;
    rm &= rm - 1;
    uint64_t a0, a1, a2;
    rep_push(val, ri - prev - 1, ri, r0, r1, r2, &a0, &a1, &a2);
    const uint32_t oi = (uint32_t)__builtin_amdgcn_readlane((int)ofv, ri);
    const uint32_t li = (uint32_t)__builtin_amdgcn_readlane((int)ll, ri);
    uint64_t o = a0;
    int e = 0;
    if (oi == 0) {
      e = SYM ? 0 : ZD_E_NULL_OFFSET;
    } else {
      const uint32_t idx = oi - (li != 0 ? 1u : 0u);
      if (idx == 0) { o = a0; }
      else if (idx == 1) { o = a1; a1 = a0; a0 = o; }
      else if (idx == 2) { o = a2; a2 = a1; a1 = a0; a0 = o; }
      else if (!SYM && a0 == 0) { e = ZD_E_REF_PANIC; }     // usize underflow of offsets[0] -= 1
      else { o = SYM ? jr_dec1(a0) : a0 - 1; a2 = a1; a1 = a0; a0 = o; }
    }
    if (lane == ri) off = o;
    r0 = a0; r1 = a1; r2 = a2;
    prev = ri;
    if (e) {
      *bad_lane = ri;
      *bad_code = e;
      return off;
    }
  }
  rep_push(val, k - 1 - prev, k, r0, r1, r2, &rep[0], &rep[1], &rep[2]);
  return off;
}

__device__ inline uint64_t wave_sum_u64(uint64_t x) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, d, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), d, 64);
    x += ((uint64_t)hi << 32) | lo;
  }
  return x;
}

// Software pipeline over a block's records shared by KJ1 and KJ3: records two
// batches ahead, bitstream windows one ahead (K4's order).
struct JRecs {
  const uint64_t* SQ;
  const uint8_t* bsp;
  uintptr_t base;
  uint32_t n;
  bool direct;
  uint64_t recA, recB;
  WinU winA;
  // record i (K3's pairs, zd_common.h, or a direct word)
  __device__ inline uint64_t at(uint32_t i) const {
    if (i >= n) return 0;
    if (direct) return SQ[i];
    const u32x4g v = *(const g_u32x4g*)(SQ + (i & ~1u));
    return rec_unpack(v.x, v.y, v.z, v.w, i & 1);
  }
  __device__ inline WinU win(uint64_t r, bool v) const { return winu_load(bsp, base, v ? (int32_t)(uint32_t)r : 0); }
  __device__ inline void start(uint32_t s0, int lane) {
    recA = at(s0 + lane);
    recB = at(s0 + 64 + lane);
    winA = win(recA, s0 + lane < n);
  }
  // this batch's (rec, window) in recA / winA; issues the next loads
  __device__ inline void next(uint32_t s0, int lane) {
    const WinU wb = win(recB, s0 + 64 + lane < n);
    const uint64_t rc = at(s0 + 128 + lane);
    recA = recB; winA = wb; recB = rc;
  }
};

__global__ __launch_bounds__(64) void zd_k_jsum(const uint8_t* __restrict__ src, const FrameState* __restrict__ fstate,
                                                const BlockRec* __restrict__ blocks, const CompBlock* __restrict__ comp,
                                                const CompState* __restrict__ cstate, const uint64_t* __restrict__ seqs,
                                                const uint16_t* __restrict__ fses, const JFrame* __restrict__ jframes,
                                                const JBlkDesc* __restrict__ jd, const JSegDesc* __restrict__ jsd,
                                                JSeg* __restrict__ jseg) {
  __shared__ __attribute__((aligned(16))) uint8_t stab[3][FSE_TAB];
  const int lane = threadIdx.x;
  const JSegDesc SD = jsd[blockIdx.x];
  const JBlkDesc D = jd[SD.jblk];
  const uint64_t key0 = fstate[jframes[D.jframe].frame].key;
  const BlockRec B = blocks[D.block];
  // the segment's sums, written in place of its checkpoint (zd_k_jsum_blocks)
  uint64_t rep[3] = {jr_sym(0), jr_sym(1), jr_sym(2)};
  uint64_t out = 0;                                 // uniform
  uint32_t lit = 0;
  if (j_live(key0, D.j) && B.type == 2) {
    const CompState CS = cstate[B.comp];
    const CompBlock C = comp[B.comp];
    const uint32_t n = C.nseq, sb = SD.k * J_SEG, se = min(n, sb + J_SEG);
    if (!CS.stop && se > sb) {
      j_stab(stab, C, comp, cstate, fses, lane);
      JRecs R{seqs + C.seq_out, src + C.src + CS.bs_off, (uintptr_t)src, se, C.seq_direct != 0};
      R.start(sb, lane);
      for (uint32_t s0 = sb; s0 < se; s0 += 64) {
        const int k = (int)min(64u, se - s0);
        uint32_t ll = 0, ml = 0, ofv = 4;
        if (lane < k) j_values(R.recA, R.winA, stab, ll, ml, ofv);
        R.next(s0, lane);
        int bl, bc;
        (void)j_offsets<true>(ofv, ll, k, rep, &bl, &bc);
        const uint32_t it = wave_scan_incl(ll + ml), il = wave_scan_incl(ll);
        out += (uint32_t)__builtin_amdgcn_readlane((int)it, 63);
        lit += (uint32_t)__builtin_amdgcn_readlane((int)il, 63);
      }
    }
  }
  if (lane == 0) {
    JSeg g{};
    g.out_rel = out;
    g.lit_rel = lit;
    g.map[0] = rep[0]; g.map[1] = rep[1]; g.map[2] = rep[2];
    jseg[D.seg0 + SD.k] = g;
  }
}

// KJ1, second part: one lane per block.  Its segments' sums become the
// checkpoints KJ3 starts from (bytes before the segment, the map before it as
// jr codes of the block's incoming offsets: the maps compose with jr_apply);
// the block's output size is its literals plus its match lengths.
__global__ __launch_bounds__(64) void zd_k_jsum_blocks(const FrameState* __restrict__ fstate,
                                                       const BlockRec* __restrict__ blocks,
                                                       const CompBlock* __restrict__ comp,
                                                       const CompState* __restrict__ cstate,
                                                       const JFrame* __restrict__ jframes,
                                                       const JBlkDesc* __restrict__ jd, uint32_t n_jblk,
                                                       JBlk* __restrict__ jb, JSeg* __restrict__ jseg) {
  const uint32_t e = blockIdx.x * 64 + threadIdx.x;
  if (e >= n_jblk) return;
  const JBlkDesc D = jd[e];
  const uint64_t key0 = fstate[jframes[D.jframe].frame].key;
  const BlockRec B = blocks[D.block];
  uint64_t map[3] = {jr_sym(0), jr_sym(1), jr_sym(2)};
  uint64_t size = 0;
  uint32_t dead = j_live(key0, D.j) ? 0u : 1u;
  if (!dead && B.type != 2) {
    size = B.size;                                  // raw / RLE (block.rs:76-79)
  } else if (!dead) {
    const CompState CS = cstate[B.comp];
    const CompBlock C = comp[B.comp];
    if (CS.stop) {
      dead = 1;
    } else {
      const uint32_t nl = (C.lit_type == LIT_RAW || C.lit_type == LIT_RLE) ? C.lit_regen : CS.lit_count;
      const uint32_t nseg = C.nseq > J_SEG ? (C.nseq + J_SEG - 1) / J_SEG : 1;
      uint64_t out = 0;
      uint32_t lit = 0;
      JSeg tn = jseg[D.seg0];                       // (the next segment's sums loaded a step ahead)
      for (uint32_t k = 0; k < nseg; k++) {
        JSeg& g = jseg[D.seg0 + k];
        const JSeg t = tn;                          // the segment's own sums
        if (k + 1 < nseg) tn = jseg[D.seg0 + k + 1];
        g.out_rel = out;
        g.lit_rel = lit;
        g.map[0] = map[0]; g.map[1] = map[1]; g.map[2] = map[2];
        out += t.out_rel;
        lit += t.lit_rel;
        const uint64_t m0 = jr_apply(t.map[0], map), m1 = jr_apply(t.map[1], map), m2 = jr_apply(t.map[2], map);
        map[0] = m0; map[1] = m1; map[2] = m2;
      }
      size = (uint64_t)nl + out - lit;              // literals + match lengths
    }
  }
  jb[e].size = size;
  jb[e].map[0] = map[0];
  jb[e].map[1] = map[1];
  jb[e].map[2] = map[2];
  jb[e].dead = dead;
}

// The frame's blocks one 64-block chunk after another from block c_start,
// entering (pos, rep): a dead block (a failure before it) or one past the
// frame's capacity stops the frame there.  One wave; writes the frame's
// outcome to S.
__device__ inline void jp_serial(const JFrame& JF, uint64_t cap, FrameState* S, FrameState* fstate,
                                 const JBlkDesc* __restrict__ jd, JBlk* jb, uint32_t c_start, uint64_t pos,
                                 uint64_t rep[3], int lane) {
  bool stop = false;
  // the next chunk's blocks are loaded while this one's scans run
  struct Ld { uint64_t size, m0, m1, m2; uint32_t dead; };
  auto load = [&](uint32_t c) -> Ld {
    const uint32_t e = JF.jb0 + c + lane;
    if (c + lane >= JF.njb) return Ld{0, jr_sym(0), jr_sym(1), jr_sym(2), 1u};
    return Ld{jb[e].size, jb[e].map[0], jb[e].map[1], jb[e].map[2], jb[e].dead};
  };
  Ld nx = load(c_start);
  for (uint32_t c = c_start; c < JF.njb; c += 64) {
    const uint32_t e = JF.jb0 + c + lane;
    const bool v = c + lane < JF.njb;
    const Ld cur = nx;
    if (c + 64 < JF.njb) nx = load(c + 64);
    uint64_t size = 0, m[3] = {jr_sym(0), jr_sym(1), jr_sym(2)};
    uint32_t dead = 1;
    if (v && !stop) {
      size = cur.size;
      m[0] = cur.m0; m[1] = cur.m1; m[2] = cur.m2;
      dead = cur.dead;
    }
    // blocks from the first dead one on do not run
    const uint64_t dm = __ballot(v && dead);
    const int fd = dm ? __ffsll((long long)dm) - 1 : 64;
    bool live = v && !stop && lane < fd;
    if (!live) { size = 0; m[0] = jr_sym(0); m[1] = jr_sym(1); m[2] = jr_sym(2); }
    uint64_t incl = wave_scan_u64(size, lane);
    // past the frame's capacity (its Frame_Content_Size; the reference checks
    // none): out of the GPU path's domain from that block on
    const uint64_t om = __ballot(live && pos + incl > cap);
    if (om) {
      const int fo = __ffsll((long long)om) - 1;
      if (lane == fo) key_min(fstate, JF.frame, make_key(PH_LIMIT, jd[e].j, LS_CAPACITY, 0, ZD_E_OUT_OF_DOMAIN));
      if (lane >= fo) { live = false; size = 0; m[0] = jr_sym(0); m[1] = jr_sym(1); m[2] = jr_sym(2); }
      incl = wave_scan_u64(size, lane);
    }
    j_scan_map(m, lane);
    uint64_t ex[3] = {shfl_up_u64(m[0], 1), shfl_up_u64(m[1], 1), shfl_up_u64(m[2], 1)};
    if (lane == 0) { ex[0] = jr_sym(0); ex[1] = jr_sym(1); ex[2] = jr_sym(2); }
    if (v) {
      jb[e].out_start = pos + incl - size;
      jb[e].rep_in[0] = jr_apply(ex[0], rep);
      jb[e].rep_in[1] = jr_apply(ex[1], rep);
      jb[e].rep_in[2] = jr_apply(ex[2], rep);
      jb[e].dead = live ? 0u : 1u;
    }
    // dead lanes hold identity maps and no bytes: lane 63 composes the live ones
    const uint64_t mt[3] = {readlane_u64(m[0], 63), readlane_u64(m[1], 63), readlane_u64(m[2], 63)};
    const uint64_t nr0 = jr_apply(mt[0], rep), nr1 = jr_apply(mt[1], rep), nr2 = jr_apply(mt[2], rep);
    rep[0] = nr0; rep[1] = nr1; rep[2] = nr2;
    pos += readlane_u64(incl, 63);
    if (fd < 64 || om) stop = true;
  }
  if (lane == 0) {
    S->out_len = pos;
    S->rep[0] = rep[0];
    S->rep[1] = rep[1];
    S->rep[2] = rep[2];
  }
}

// KJ2: one workgroup of JP_WAVES waves per frame.  Blocks in super-chunks of
// 64 x JP_WAVES: each wave scans its 64 blocks' sizes and repeat-offset maps,
// one lane composes the waves' totals in order, and every block gets its
// output start and entering offsets at once (c3s: the one-wave loop over 12
// chunks took ~22 us).  A super-chunk with a dead block or a block past the
// frame's capacity goes to jp_serial from its start (the same outcome).
constexpr int JP_WAVES = 16;
__global__ __launch_bounds__(64 * JP_WAVES) void zd_k_jprefix(const FrameDesc* __restrict__ frames, FrameState* fstate,
                                                              const JFrame* __restrict__ jframes,
                                                              const JBlkDesc* __restrict__ jd, JBlk* jb) {
  __shared__ uint64_t wsz[JP_WAVES], wmap[JP_WAVES][3], wpos[JP_WAVES + 1], wrep[JP_WAVES + 1][3];
  __shared__ uint32_t flag;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const JFrame JF = jframes[blockIdx.x];
  const uint64_t cap = frames[JF.frame].out_cap;
  FrameState* S = &fstate[JF.frame];
  uint64_t pos = 0;
  uint64_t rep[3] = {S->rep[0], S->rep[1], S->rep[2]};
  uint32_t c0 = 0;
  for (; c0 < JF.njb; c0 += 64 * JP_WAVES) {
    const uint32_t i = c0 + (uint32_t)t, e = JF.jb0 + i;
    const bool v = i < JF.njb;
    uint64_t size = 0, m[3] = {jr_sym(0), jr_sym(1), jr_sym(2)};
    uint32_t dead = 0;
    if (v) {
      size = jb[e].size;
      m[0] = jb[e].map[0]; m[1] = jb[e].map[1]; m[2] = jb[e].map[2];
      dead = jb[e].dead;
    }
    if (t == 0) flag = 0;
    __syncthreads();
    if (v && dead) flag = 1;
    const uint64_t incl = wave_scan_u64(size, lane);
    j_scan_map(m, lane);                           // m: the wave's inclusive composites
    if (lane == 63) {
      wsz[wv] = incl;
      wmap[wv][0] = m[0]; wmap[wv][1] = m[1]; wmap[wv][2] = m[2];
    }
    __syncthreads();
    if (t == 0) {                                  // the waves' entering states, in order
      uint64_t p = pos, r0 = rep[0], r1 = rep[1], r2 = rep[2];
      for (int w = 0; w < JP_WAVES; w++) {
        wpos[w] = p;
        wrep[w][0] = r0; wrep[w][1] = r1; wrep[w][2] = r2;
        p += wsz[w];
        const uint64_t r[3] = {r0, r1, r2};
        r0 = jr_apply(wmap[w][0], r); r1 = jr_apply(wmap[w][1], r); r2 = jr_apply(wmap[w][2], r);
      }
      wpos[JP_WAVES] = p;
      wrep[JP_WAVES][0] = r0; wrep[JP_WAVES][1] = r1; wrep[JP_WAVES][2] = r2;
    }
    __syncthreads();
    const uint64_t wp = wpos[wv];
    const uint64_t wr[3] = {wrep[wv][0], wrep[wv][1], wrep[wv][2]};
    if (v && wp + incl > cap) flag = 1;            // past the frame's capacity
    __syncthreads();
    if (flag) break;                               // (uniform: read after the barrier)
    uint64_t ex[3] = {shfl_up_u64(m[0], 1), shfl_up_u64(m[1], 1), shfl_up_u64(m[2], 1)};
    if (lane == 0) { ex[0] = jr_sym(0); ex[1] = jr_sym(1); ex[2] = jr_sym(2); }
    if (v) {
      jb[e].out_start = wp + incl - size;
      jb[e].rep_in[0] = jr_apply(ex[0], wr);
      jb[e].rep_in[1] = jr_apply(ex[1], wr);
      jb[e].rep_in[2] = jr_apply(ex[2], wr);
      jb[e].dead = 0;
    }
    pos = wpos[JP_WAVES];
    rep[0] = wrep[JP_WAVES][0]; rep[1] = wrep[JP_WAVES][1]; rep[2] = wrep[JP_WAVES][2];
    __syncthreads();                               // (the LDS totals are rewritten next)
  }
  if (c0 < JF.njb) {                               // a dead or over-capacity block in this super-chunk
    if (wv == 0) jp_serial(JF, cap, S, fstate, jd, jb, c0, pos, rep, lane);
    return;
  }
  if (t == 0) {
    S->out_len = pos;
    S->rep[0] = rep[0];
    S->rep[1] = rep[1];
    S->rep[2] = rep[2];
  }
}

typedef __attribute__((address_space(1))) u32x4a1 g_u32x4a1;

// Words [0, n) of 16 state words to p (n <= 16): four 16-byte stores, or one by one.
__device__ inline void j_store_words(uint32_t* p, const uint32_t w[16], uint32_t n) {
  if (n == 16) {
#pragma unroll
    for (int q = 0; q < 4; q++) *(g_u32x4a1*)(p + 4 * q) = (u32x4){w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
    return;
  }
#pragma unroll
  for (uint32_t b = 0; b < 16; b++)
    if (b < n) p[b] = w[b];
}
// n literal bytes from s (HBM) or the fill byte at frame position P0: final.
// 16-byte pieces aligned in the state array's 64-byte lines.
__device__ void j_fill_lits(uint32_t* st, uint64_t P0, uint32_t n, const uint8_t* s, uint32_t fill, int lane) {
  if (!n) return;
  const uint32_t g = (16 - (P0 & 15)) & 15;
  const uint32_t np = n > g ? 1 + (n - g + 15) / 16 : 1;
  for (uint32_t pi = lane; pi < np; pi += 64) {
    const uint32_t x0 = pi == 0 ? 0 : g + 16 * (pi - 1);
    const uint32_t x1 = pi == 0 ? min(g, n) : min(n, g + 16 * pi);
    if (x0 >= x1) continue;
    uint32_t w[16];
    if (s && x1 - x0 == 16) {
      const u32x4 v = ldg16(s + x0);
#pragma unroll
      for (uint32_t b = 0; b < 16; b++) w[b] = J_FINAL | ((v[b >> 2] >> (8 * (b & 3))) & 255);
    } else {
#pragma unroll
      for (uint32_t b = 0; b < 16; b++) w[b] = J_FINAL | (s ? (x0 + b < x1 ? s[x0 + b] : 0u) : fill);
    }
    j_store_words(st + P0 + x0, w, x1 - x0);
  }
}

// The scatter's literal stage (ZD_JS_STAGE 0: every literal byte its own HBM
// load and every overlapping match byte a division, the round-5 form)
#ifndef ZD_JS_STAGE
#define ZD_JS_STAGE 1
#endif
constexpr uint32_t JS_STG = 2048;
__global__ __launch_bounds__(64) void zd_k_jscatter(const uint8_t* __restrict__ src, FrameState* fstate,
                                                    const BlockRec* __restrict__ blocks,
                                                    const CompBlock* __restrict__ comp,
                                                    const CompState* __restrict__ cstate,
                                                    const uint8_t* __restrict__ lits, const uint64_t* __restrict__ seqs,
                                                    const uint16_t* __restrict__ fses,
                                                    const JFrame* __restrict__ jframes,
                                                    const JBlkDesc* __restrict__ jd, const JBlk* __restrict__ jb,
                                                    const JSeg* __restrict__ jseg, const JSegDesc* __restrict__ jsd,
                                                    uint32_t* jst) {
  __shared__ __attribute__((aligned(16))) uint8_t stab[3][FSE_TAB];
  __shared__ uint32_t sa[65], sll[64], soff[64], slp[64];
#if ZD_JS_STAGE
  __shared__ __attribute__((aligned(16))) uint8_t slit_[JS_STG];
  l_u8* const slit = (l_u8*)slit_;
#endif
  const int lane = threadIdx.x;
  const JSegDesc SD = jsd[blockIdx.x];
  const uint32_t e = SD.jblk;
  if (jb[e].dead) return;
  const JBlkDesc D = jd[e];
  const JFrame JF = jframes[D.jframe];
  uint32_t* st = jst + JF.base;
  const BlockRec B = blocks[D.block];
  uint64_t pos = jb[e].out_start;
  if (B.type != 2) {
    j_fill_lits(st, pos, B.size, B.type == 1 ? nullptr : src + B.src, B.rle, lane);
    return;
  }
  const CompBlock C = comp[B.comp];
  const CompState CS = cstate[B.comp];
  const uint8_t* lsrc = nullptr;
  uint32_t lfill = 0, nl;
  if (C.lit_type == LIT_RAW) { lsrc = src + C.src + C.lit_data; nl = C.lit_regen; }
  else if (C.lit_type == LIT_RLE) { lfill = C.lit_rle; nl = C.lit_regen; }
  else { lsrc = lits + C.lit_out; nl = CS.lit_count; }
  const JSeg G = jseg[D.seg0 + SD.k];
  const uint64_t rin[3] = {jb[e].rep_in[0], jb[e].rep_in[1], jb[e].rep_in[2]};
  uint64_t rep[3] = {jr_apply(G.map[0], rin), jr_apply(G.map[1], rin), jr_apply(G.map[2], rin)};
  pos += G.out_rel;
  uint32_t lit_cursor = G.lit_rel;
  const uint32_t n = C.nseq;
  const uint32_t sb = SD.k * J_SEG, se = min(n, sb + J_SEG);
  if (se > sb) {
    j_stab(stab, C, comp, cstate, fses, lane);
    JRecs R{seqs + C.seq_out, src + C.src + CS.bs_off, (uintptr_t)src, se, C.seq_direct != 0};
    R.start(sb, lane);
    for (uint32_t s0 = sb; s0 < se; s0 += 64) {
      const int k = (int)min(64u, se - s0);
      const bool valid = lane < k;
      uint32_t ll = 0, ml = 0, ofv = 4;
      if (valid) j_values(R.recA, R.winA, stab, ll, ml, ofv);
      R.next(s0, lane);
      int bl, bc;
      const uint64_t off = j_offsets<false>(ofv, ll, k, rep, &bl, &bc);
      const uint32_t tot = ll + ml;
      const uint32_t inc_tot = wave_scan_incl(tot), inc_ll = wave_scan_incl(ll);
      const uint32_t opos = inc_tot - tot, lpos = inc_ll - ll;
      // checks (decoding_context.rs:84-90, D9), in sequence order
      const uint64_t before = (uint64_t)pos + opos;
      const bool dbad = valid && lane == bl;
      const bool imp = valid && !dbad && ((uint64_t)lit_cursor + lpos + ll > nl || off > before + ll);
      const bool panic = valid && !dbad && !imp && ml != 0 && off == 0;
      // a match byte's state word is its distance to the byte it copies
      // (< J_FINAL): only a frame past 2 GiB reaches further (the streaming
      // K4 is no way out there: out of the GPU path's domain)
      const bool far = valid && !dbad && !imp && !panic && ml != 0 && off + ml >= J_FINAL;
      const uint64_t badm = __ballot(dbad || imp || panic || far);
      if (badm) {
        const int b = __ffsll((long long)badm) - 1;
        const bool lim = __shfl((int)far, b, 64) != 0;
        const int code = __shfl(dbad ? bc : (imp ? ZD_E_IMPOSSIBLE_VALUE : ZD_E_REF_PANIC), b, 64);
        if (lane == 0)
          key_min(fstate, JF.frame, lim ? make_key(PH_LIMIT, D.j, LS_JROUNDS, s0 + (uint32_t)b, ZD_E_OUT_OF_DOMAIN)
                                        : make_key(PH_DECODE, D.j, DS_EXECUTE, s0 + (uint32_t)b, code));
        return;
      }
      const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)inc_tot, k - 1);
      const uint32_t Lsum = (uint32_t)__builtin_amdgcn_readlane((int)inc_ll, k - 1);
      if (valid) {
        sa[lane] = opos;
        sll[lane] = ll;
        soff[lane] = (uint32_t)off;
        slp[lane] = lit_cursor + lpos;
      }
      if (lane == 0) sa[k] = T;
#if ZD_JS_STAGE
      // the batch's literal bytes [lit_cursor, + Lsum) staged in LDS when
      // they fit (16 bytes a lane; the literal buffers carry 16 readable
      // bytes past their end), else read byte by byte from HBM
      const bool staged = lsrc && Lsum <= JS_STG;
      if (staged)
        for (uint32_t c = 16 * (uint32_t)lane; c < Lsum; c += 1024) *(l_u32x4*)(slit + c) = ldg16(lsrc + lit_cursor + c);
#endif
      k4_sync();
      // the batch's bytes [pos, pos + T) in 16-byte pieces (aligned in the
      // state array): the sequence of each byte by a search of the starts
      const uint32_t g = (16 - (pos & 15)) & 15;
      const uint32_t np = T > g ? 1 + (T - g + 15) / 16 : 1;
#if ZD_JS_STAGE
      for (uint32_t pi = lane; pi < np; pi += 64) {
        const uint32_t x0 = pi == 0 ? 0 : g + 16 * (pi - 1);
        const uint32_t x1 = pi == 0 ? min(g, T) : min(T, g + 16 * pi);
        if (x0 >= x1) continue;
        int i = 0;
#pragma unroll
        for (int stp = 32; stp; stp >>= 1)
          if (i + stp < k && sa[i + stp] <= x0) i += stp;
        uint32_t a = sa[i], nx = sa[i + 1], l = sll[i], o = soff[i], lp = slp[i];
        // a match byte at jj of its match copies the byte o + jj - (jj mod o)
        // back (the reference's byte-by-byte push, decoding_context.rs:95-98):
        // jj mod o by one division at the piece's first byte, then counted
        uint32_t jj = 0, r = 0;
        bool inm = x0 - a >= l;
        if (inm) {
          jj = x0 - a - l;
          r = jj < o ? jj : jj % o;
        }
        uint32_t w[16];
#pragma unroll
        for (uint32_t b = 0; b < 16; b++) {
          const uint32_t x = x0 + b;
          w[b] = 0;
          if (x < x1) {
            if (b) {
              if (x >= nx) {                   // the next sequence (one with no bytes is passed over)
                do { i++; a = nx; nx = sa[i + 1]; } while (x >= nx);
                l = sll[i]; o = soff[i]; lp = slp[i];
                jj = 0; r = 0;
                inm = l == 0;
              } else if (inm) {
                jj++;
                r = r + 1 == o ? 0u : r + 1;
              } else if (x - a >= l) {
                inm = true;
              }
            }
            const uint32_t q = lp + (x - a) - lit_cursor;   // the byte's literal, relative to the stage
            w[b] = inm ? o + jj - r : J_FINAL | (staged ? (uint32_t)slit[q] : lsrc ? (uint32_t)lsrc[lp + (x - a)] : lfill);
          }
        }
        j_store_words(st + pos + x0, w, x1 - x0);
      }
#else
      for (uint32_t pi = lane; pi < np; pi += 64) {
        const uint32_t x0 = pi == 0 ? 0 : g + 16 * (pi - 1);
        const uint32_t x1 = pi == 0 ? min(g, T) : min(T, g + 16 * pi);
        if (x0 >= x1) continue;
        int i = 0;
#pragma unroll
        for (int stp = 32; stp; stp >>= 1)
          if (i + stp < k && sa[i + stp] <= x0) i += stp;
        uint32_t a = sa[i], nx = sa[i + 1], l = sll[i], o = soff[i], lp = slp[i];
        uint32_t w[16];
#pragma unroll
        for (uint32_t b = 0; b < 16; b++) {
          const uint32_t x = x0 + b;
          w[b] = 0;
          if (x < x1) {
            while (x >= nx) { i++; a = nx; nx = sa[i + 1]; l = sll[i]; o = soff[i]; lp = slp[i]; }
            const uint32_t rel = x - a;
            if (rel < l) {
              w[b] = J_FINAL | (lsrc ? (uint32_t)lsrc[lp + rel] : lfill);
            } else {
              const uint32_t jj = rel - l;     // distance: o, or o times the periods passed
              w[b] = o + (jj < o ? 0u : jj - jj % o);
            }
          }
        }
        j_store_words(st + pos + x0, w, x1 - x0);
      }
#endif
      k4_sync();
      lit_cursor += Lsum;
      pos += T;
    }
  }
  // leftover literals (decoding_context.rs:101-103), by the block's last segment
  if (se == n && lit_cursor < nl)
    j_fill_lits(st, pos, nl - lit_cursor, lsrc ? lsrc + lit_cursor : nullptr, lfill, lane);
}

// The frame and 16-word piece of piece number pc (K4J rounds and emit).
__device__ inline uint32_t j_frame_of(const JFrame* __restrict__ jframes, uint32_t n_jframes, uint64_t pc) {
  uint32_t lo = 0, hi = n_jframes;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (jframes[mid].piece0 <= pc) lo = mid;
    else hi = mid;
  }
  return lo;
}

typedef __attribute__((address_space(1))) uint32_t g_u32a1 __attribute__((aligned(1)));
#ifndef ZD_J_SUB
#define ZD_J_SUB 1                      // parts per region, each swept by its share of the workgroups
#endif
#ifndef ZD_J_XREG
#define ZD_J_XREG 8                     // regions over the chip (8: one an XCD)
#endif
#ifndef ZD_JW_K
#define ZD_JW_K 2
#endif
constexpr int JW_K = ZD_JW_K;   // pieces per lane in flight (each hop issues JW_K independent loads)
// Pointer-jumping round r, one state word per lane: sixteen lanes (a DPP row)
// take a piece, and each lane JW_K pieces at once, so a wave holds 4 * JW_K
// consecutive pieces.  A hop is one load per pending word, S[p] = S[p - S[p]]:
// the words of one match point at one contiguous source run, so a wave's 64
// loads fall on a few cache lines (one piece per lane made each word a
// lane-private gather), and the JW_K loads of a lane are independent, so a
// wave keeps JW_K dependent chains in flight (the rounds are bound by the
// latency of those chains: a wave walks ~200 tiles one after another).  A
// piece whose sixteen words are final is emitted -- four dword stores -- and
// marked done.  The grid is what fits on the chip at once (8 workgroups of
// 256 per CU), each XCD sweeping one contiguous eighth of the pieces in
// ascending order (workgroups b and b + 8 share an XCD, speed only): match
// sources lie at most a window behind, so they were updated earlier in the
// same round more often and sit in that XCD's L2.  pend[r] counts the waves
// that left a piece pending; a round after one that left none exits at once.
// The rounds past the second run as one launch of `sweeps` sweeps: no round
// needs another's words in any order (every version of a word is true of its
// byte, and every chain ends at a literal the scatter wrote), so each wave
// sweeps its own pieces until it leaves none pending, and the tail of empty
// rounds costs one launch instead of one each.
__global__ __launch_bounds__(256) void zd_k_jround(uint8_t* outbase, const FrameDesc* __restrict__ frames,
                                                   FrameState* fstate, const JFrame* __restrict__ jframes,
                                                   uint32_t n_jframes, uint64_t n_pieces, uint32_t* jst,
                                                   uint32_t* pend, uint8_t* done, uint32_t hops, uint32_t r,
                                                   uint32_t last, uint32_t sweeps) {
  if (r > 1 && *(volatile uint32_t*)&pend[r - 1] == 0) return;
  // ZD_J_XREG regions over the chip, each swept by the workgroups of 8 / XREG
  // XCDs (workgroup b runs on XCD b mod 8)
  constexpr uint32_t XR = ZD_J_XREG, XG = 8 / ZD_J_XREG;
  static_assert(XR * XG == 8, "ZD_J_XREG: 1, 2, 4 or 8 regions");
  const uint32_t x = (blockIdx.x & 7) % XR, nk = (gridDim.x >> 3) * XG;
  const uint32_t jw = (blockIdx.x >> 3) * XG + (blockIdx.x & 7) / XR;   // the workgroup within its region
  const uint32_t sub = threadIdx.x & 15, row = threadIdx.x >> 4, wrow = row & 3;
  const uint64_t R = (n_pieces + XR - 1) / XR;
  // the region in S parts, each swept by nk / S of its workgroups
  const uint32_t S = (nk % ZD_J_SUB == 0) ? ZD_J_SUB : 1u, nu = nk / S;
  const uint32_t rg = jw % S, u = jw / S;
  const uint64_t Rs = (R + S - 1) / S, rb = (uint64_t)rg * Rs;
  bool mine = false;
  for (uint32_t sw = 0; sw < sweeps; sw++) {
  const bool fin = last && sw + 1 == sweeps;
  mine = false;
  for (uint64_t i0 = (uint64_t)u * (16 * JW_K); i0 < Rs; i0 += (uint64_t)nu * (16 * JW_K)) {
    uint64_t pc[JW_K], p0[JW_K], total[JW_K];
    uint32_t* st[JW_K];
    uint32_t w[JW_K], fr[JW_K];
    bool act[JW_K], pw[JW_K], had[JW_K];
#pragma unroll
    for (int k = 0; k < JW_K; k++) {
      const uint64_t i = i0 + 16 * k + row;           // a wave's rows: four consecutive pieces per k
      pc[k] = x * R + rb + i;
      act[k] = i < Rs && rb + i < R && pc[k] < n_pieces;
    }
    JFrame JF[JW_K];
    uint8_t dn[JW_K];
#pragma unroll
    for (int k = 0; k < JW_K; k++) {
      JF[k] = act[k] ? jframes[j_frame_of(jframes, n_jframes, pc[k])] : JFrame{};
      dn[k] = act[k] ? done[pc[k]] : (uint8_t)1;
    }
    uint64_t key[JW_K];
#pragma unroll
    for (int k = 0; k < JW_K; k++) {
      act[k] = act[k] && !dn[k];
      fr[k] = JF[k].frame;
      st[k] = jst + JF[k].base;
      p0[k] = 16 * (pc[k] - JF[k].piece0);
      const FrameState* S = &fstate[fr[k]];
      key[k] = act[k] ? S->key : KEY_NONE;
      total[k] = act[k] ? S->out_len : 0;
      // the word itself, in parallel with the frame's state (bounded by the region)
      w[k] = act[k] && p0[k] + sub < JF[k].cap ? st[k][p0[k] + sub] : J_FINAL;
    }
#pragma unroll
    for (int k = 0; k < JW_K; k++) {
      act[k] = act[k] && key[k] == KEY_NONE && p0[k] < total[k];
      const bool inw = act[k] && p0[k] + sub < total[k];
      if (!inw) w[k] = J_FINAL;
      pw[k] = !(w[k] & J_FINAL);
      had[k] = pw[k];
    }
    for (uint32_t h = 0; h < hops; h++) {
      bool any = false;
#pragma unroll
      for (int k = 0; k < JW_K; k++) any |= pw[k];
      if (!__ballot(any)) break;
      uint32_t v[JW_K];
#pragma unroll
      for (int k = 0; k < JW_K; k++) {
        const uint64_t p = p0[k] + sub;
        v[k] = pw[k] ? st[k][w[k] <= p ? p - w[k] : 0u] : w[k];
      }
#pragma unroll
      for (int k = 0; k < JW_K; k++) {
        if (pw[k]) {
          // a final source hands over its byte, a pending one adds its distance
          const uint32_t d = w[k] + v[k];
          w[k] = (v[k] & J_FINAL) ? v[k] : (d < J_FINAL ? d : w[k]);
        }
        pw[k] = !(w[k] & J_FINAL);
      }
    }
#pragma unroll
    for (int k = 0; k < JW_K; k++) {
      if (had[k]) st[k][p0[k] + sub] = w[k];
      const uint64_t pm = __ballot(pw[k]);
      const bool piece_pending = ((pm >> (16 * wrow)) & 0xFFFFull) != 0;
      if (act[k] && piece_pending) {
        mine = true;
        if (fin && sub == 0) key_min(fstate, fr[k], make_key(PH_LIMIT, 0, LS_JROUNDS, 0, ZD_E_OUT_OF_DOMAIN));
      }
      if (act[k] && !piece_pending) {
        // bytes of four lanes into each lane of the quad (quad_perm broadcasts)
        const uint32_t bt = w[k] & 255;
        const uint32_t d = qdpp<0x00>(bt) | (qdpp<0x55>(bt) << 8) | (qdpp<0xAA>(bt) << 16) | (qdpp<0xFF>(bt) << 24);
        uint8_t* o = outbase + frames[fr[k]].out + p0[k];
        const uint64_t nb = total[k] - p0[k];
        if (nb >= 16) {
          if ((sub & 3) == 0) *(g_u32a1*)(o + sub) = d;
        } else if (sub < nb) {
          o[sub] = (uint8_t)bt;
        }
        if (sub == 0) done[pc[k]] = 1;
      }
    }
  }
  if (!__ballot(mine)) break;                      // the wave's pieces are all emitted
  }
  const uint64_t bm = __ballot(mine);
  if ((threadIdx.x & 63) == 0 && bm) atomicAdd(&pend[r], 1u);
}

// ---------------------------------------------------------------------------
// K0: raw / RLE blocks at the head of a frame (block.rs:78-79: Raw appends
// the bytes, RLE the byte `size` times), whose output offsets the planner
// knows.  A piece of <= 32 KiB takes K0_SPLIT workgroups of 256 threads,
// one 16-byte chunk per thread (C2 at 1 GiB: 0.356 ms with one workgroup
// per piece looping over its chunks, 0.278 with one chunk per thread, as
// many memory operations in flight as the chip holds workgroups); 16-byte
// aligned stores, head and tail bytewise (the piece's first workgroup).
// ---------------------------------------------------------------------------
constexpr uint32_t K0_SPLIT = COPY_PIECE / (16 * 256);
static_assert(K0_SPLIT * 16 * 256 == COPY_PIECE, "K0: a piece is K0_SPLIT workgroups of one chunk per thread");
__global__ __launch_bounds__(256) void zd_k_rawcopy(const uint8_t* __restrict__ src, uint8_t* outbase,
                                                    const CopyDesc* __restrict__ copies) {
  const uint32_t sub = blockIdx.x % K0_SPLIT;
  const CopyDesc c = copies[blockIdx.x / K0_SPLIT];
  const uint8_t* s = src + c.src;
  uint8_t* d = outbase + c.dst;
  const bool rle = c.fill != 0;
  const uint8_t b = (uint8_t)c.fill;
  const uint32_t f = b * 0x01010101u;
  const u32x4 f4 = (u32x4){f, f, f, f};
  const uint32_t head = min(c.size, (uint32_t)((16 - ((uintptr_t)d & 15)) & 15));
  const int t = threadIdx.x;
  const uint32_t x = head + 16 * (256 * sub + (uint32_t)t);
  if (x + 16 <= c.size) *(g_u32x4*)(d + x) = rle ? f4 : ldg16(s + x);
  if (sub == 0) {
    if ((uint32_t)t < head) d[t] = rle ? b : s[t];
    const uint32_t tail0 = head + ((c.size - head) & ~15u);
    if (tail0 + t < c.size) d[tail0 + t] = rle ? b : s[tail0 + t];
  }
}

// ---------------------------------------------------------------------------
// XXH64 of decoded frames (zd_plan_checksums; the reference's frame.rs:
// 239-255 computes and never enforces it).  Four lanes per frame, one per
// XXH64 accumulator, 16 frames per wave; lane 0 of a frame folds the four
// accumulators, hashes the tail and writes the digest.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(1))) const uint64_t g_cu64a1 __attribute__((aligned(1)));
__global__ __launch_bounds__(64) void zd_k_xxh64(const uint8_t* __restrict__ base, const uint64_t* __restrict__ off,
                                                 const uint64_t* __restrict__ len, uint32_t n, uint64_t* hash) {
  const int lane = threadIdx.x, sub = lane & 3;
  const uint32_t f = blockIdx.x * 16 + (lane >> 2);
  const bool act = f < n;
  const uint8_t* p = act ? base + off[f] : base;
  const uint64_t L = act ? len[f] : 0;
  const uint64_t nst = L / 32;
  uint64_t v = xx_acc_init(sub);
  uint64_t s = 0;
  for (; s + 4 <= nst; s += 4) {                  // four stripes per trip, loads first
    const uint64_t w0 = *(g_cu64a1*)(p + 32 * s + 8 * sub), w1 = *(g_cu64a1*)(p + 32 * (s + 1) + 8 * sub);
    const uint64_t w2 = *(g_cu64a1*)(p + 32 * (s + 2) + 8 * sub), w3 = *(g_cu64a1*)(p + 32 * (s + 3) + 8 * sub);
    v = xx_round(xx_round(xx_round(xx_round(v, w0), w1), w2), w3);
  }
  for (; s < nst; s++) v = xx_round(v, *(g_cu64a1*)(p + 32 * s + 8 * sub));
  const int l0 = lane & ~3;
  uint64_t acc[4];
  for (int i = 0; i < 4; i++) acc[i] = readlane_any_u64(v, l0 + i);
  if (act && sub == 0) hash[f] = xx_finish(L, acc, p + 32 * nst, (uint32_t)(L - 32 * nst));
}

hipError_t launch_xxh64(const uint8_t* base, const uint64_t* d_off, const uint64_t* d_len, uint32_t n,
                        uint64_t* d_hash, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(zd_k_xxh64, dim3((n + 15) / 16), dim3(64), 0, s, base, d_off, d_len, n, d_hash);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// compaction (frames without an exact FCS layout)
// ---------------------------------------------------------------------------
// One frame per blockIdx.x, COMPACT_SPLIT workgroups (blockIdx.y) over
// its bytes: 16-byte loads and aligned 16-byte stores, head and tail bytewise
// (as K0: more workgroups with less work each keep more copies in flight).
constexpr uint32_t COMPACT_SPLIT = 8;
__global__ __launch_bounds__(256) void zd_k_compact(const uint8_t* __restrict__ staging, uint8_t* dst,
                                                    const uint64_t* from, const uint64_t* to, const uint64_t* len) {
  const uint32_t f = blockIdx.x;
  const uint8_t* s = staging + from[f];
  uint8_t* d = dst + to[f];
  const uint64_t n = len[f];
  const uint64_t head = min(n, (uint64_t)((16 - ((uintptr_t)d & 15)) & 15));
  const uint64_t nch = (n - head) / 16;                       // whole 16-byte chunks after the head
  const uint64_t per = (nch + COMPACT_SPLIT - 1) / COMPACT_SPLIT;
  const uint64_t c0 = per * blockIdx.y, c1 = min(nch, c0 + per);
  for (uint64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x)
    *(g_u32x4*)(d + head + 16 * c) = ldg16(s + head + 16 * c);
  if (blockIdx.y == 0) {
    if (threadIdx.x < head) d[threadIdx.x] = s[threadIdx.x];
    const uint64_t tail0 = head + 16 * nch;
    if (tail0 + threadIdx.x < n) d[tail0 + threadIdx.x] = s[tail0 + threadIdx.x];
  }
}

// ---------------------------------------------------------------------------
// launch
// ---------------------------------------------------------------------------
hipError_t launch_pipeline(const LaunchArgs& a) {
  uint8_t* ws = a.ws;
  const Workspace& W = a.W;
  auto* comp = (const CompBlock*)(ws + W.comp);
  auto* cstate = (CompState*)(ws + W.comp_state);
  auto* blocks = (const BlockRec*)(ws + W.blocks);
  auto* frames = (const FrameDesc*)(ws + W.frames);
  auto* fstate = (FrameState*)(ws + W.frame_state);
  auto* luts = (uint16_t*)(ws + W.luts);
  auto* fses = (uint16_t*)(ws + W.fses);
  auto* seqs = (uint64_t*)(ws + W.seqs);
  hipStream_t s = a.stream;
  hipError_t e;
  // mode 2: events around launch group g on s
  auto dom = [&](int g, int end) -> hipError_t {
    if (!a.dom_events) return hipSuccess;
    if (end) *a.dom_used |= 1u << g;
    return hipEventRecord(a.dom_events[2 * g + end], s);
  };
  if (a.events) if ((e = hipEventRecord(a.events[0], s)) != hipSuccess) return e;
  if (a.n_copies) {
    if ((e = dom(DOM_K0, 0)) != hipSuccess) return e;
    hipLaunchKernelGGL(zd_k_rawcopy, dim3(a.n_copies * K0_SPLIT), dim3(256), 0, s, a.src, a.out,
                       (const CopyDesc*)(ws + W.copies));
    if ((e = dom(DOM_K0, 1)) != hipSuccess) return e;
  }
  if (a.events) if ((e = hipEventRecord(a.events[1], s)) != hipSuccess) return e;
  // K2 and K3 are independent once their tables exist: with the fork, K1's
  // Huffman half and K2 run on the aux stream beside K1's sequence half and
  // K3 (not when timing kernels one by one)
  const bool fork = a.aux && !a.k1_fork && !a.events && a.n_huf && a.n_seq;
  // without it, K1's two halves may still run on the two streams (joined
  // before K2)
  const bool k1f = a.aux && a.k1_fork && !a.events && a.n_tables;
  hipStream_t s2 = fork ? a.aux : s;
  if (fork || k1f) {
    if ((e = hipEventRecord(a.fork, s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(a.aux, a.fork, 0)) != hipSuccess) return e;
  }
  auto* huge = (uint32_t*)(ws + W.huge);
  auto k1 = [&](auto pass_small, auto pass_big, hipStream_t st, bool huf) {
    const dim3 g((a.n_tables + K1_LANES - 1) / K1_LANES), b(K1_LANES);
    const uint32_t* lt = (const uint32_t*)(ws + W.list_tables);
    hipLaunchKernelGGL(pass_small, g, b, 0, st, a.src, a.src_size, comp, cstate, fstate, lt, a.n_tables, luts, fses,
                       huge);
    hipLaunchKernelGGL(pass_big, g, b, 0, st, a.src, a.src_size, comp, cstate, fstate, lt, a.n_tables, luts, fses,
                       huge);
    if (huf) {                                 // the trees of more than 256 symbols the two passes listed
      hipLaunchKernelGGL(zd_k_tables_huge, dim3(K1H_GRID), dim3(K1H_LANES), 0, st, a.src, a.src_size, comp, cstate,
                         fstate, (const uint32_t*)huge, luts, (uint32_t*)(ws + W.deep));
      // K2's pair tables, from the LUTs of maxBits <= 11
      hipLaunchKernelGGL(zd_k_huf_pairs, dim3((a.n_tables + PR_WAVES - 1) / PR_WAVES), dim3(64 * PR_WAVES), 0, st,
                         comp, (const CompState*)cstate, lt, a.n_tables, luts);
    }
  };
  const bool fz = a.fused && !a.events;
  auto k1seqw = [&](hipStream_t st) {
    hipLaunchKernelGGL(zd_k_tables_seqw, dim3(a.n_tables), dim3(64), 0, st, a.src, comp, cstate, fstate,
                       (const uint32_t*)(ws + W.list_tables), a.n_tables, fses);
  };
  if (a.n_tables) {
    if (fz) {                                  // the sequence half runs in zd_k_fused
      k1(zd_k_tables<false, 1>, zd_k_tables<true, 1>, s2, true);
    } else if (a.k1_seq_waves) {               // few blocks: the sequence half one wave per block
      k1(zd_k_tables<false, 1>, zd_k_tables<true, 1>, k1f ? a.aux : s2, true);
      k1seqw(s);
    } else if (fork || k1f) {
      k1(zd_k_tables<false, 1>, zd_k_tables<true, 1>, k1f ? a.aux : s2, true);
      k1(zd_k_tables<false, 2>, zd_k_tables<true, 2>, s, false);
    } else {
      k1(zd_k_tables<false, 3>, zd_k_tables<true, 3>, s, true);
    }
  }
  if (a.events) if ((e = hipEventRecord(a.events[2], s)) != hipSuccess) return e;
  if (k1f) {
    if ((e = hipEventRecord(a.join, a.aux)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(s, a.join, 0)) != hipSuccess) return e;
  }
  if (a.n_huf)
    hipLaunchKernelGGL(zd_k_huffman, dim3((a.n_huf + K2_BLOCKS - 1) / K2_BLOCKS), dim3(K2_LANES), 0, s2, a.src, comp,
                       cstate, fstate, (const uint32_t*)(ws + W.list_huf), a.n_huf, (const uint16_t*)luts, ws + W.lits,
                       (a.fused && fork) ? (uint32_t*)(ws + W.k2done) : (uint32_t*)nullptr,
                       (const uint8_t*)(ws + W.deep + 16));
  if (fork)
    if ((e = hipEventRecord(a.join, a.aux)) != hipSuccess) return e;
  if (a.events) if ((e = hipEventRecord(a.events[3], s)) != hipSuccess) return e;
  auto k3 = [&](const uint32_t* list, uint32_t n, hipStream_t st, const uint8_t* redo) {
    if (n) {
      if (a.k3_lat && a.k3_quad)
        hipLaunchKernelGGL(zd_k_sequences_l, dim3(n), dim3(64), 0, st, a.src, comp, cstate, fstate, list, n,
                           (const uint16_t*)fses, seqs, redo);
      else if (a.k3_quad)
        hipLaunchKernelGGL(zd_k_sequences_q, dim3((n + K3Q_CHAINS - 1) / K3Q_CHAINS), dim3(64), 0, st, a.src, comp,
                           cstate, fstate, list, n, (const uint16_t*)fses, seqs, redo);
      else
        hipLaunchKernelGGL(zd_k_sequences, dim3((n + K3_LANES - 1) / K3_LANES), dim3(K3_LANES), 0, st, a.src, comp,
                           cstate, fstate, list, n, (const uint16_t*)fses, seqs);
    }
  };
  // the streaming K4 runs when some frame is not K4F's, K4J's or K0's alone
  // (the others exit at once in it)
  const bool k4_work = a.n_frames > a.n_k4f + a.n_jframes + a.n_k0only;
  auto k4 = [&](uint32_t f0, uint32_t f1, hipStream_t st, const uint8_t* redo) -> hipError_t {
    const uint32_t n = f1 - f0;
    if (n && k4_work) {  // frames on the streaming K4 (K4F's, K4J's and K0's exit at once)
      const bool tm = !redo && k4_work;
      if (tm) if ((e = dom(DOM_K4, 0)) != hipSuccess) return e;
      hipLaunchKernelGGL(zd_k_execute, dim3(n),
                         dim3(64), 0, st, a.src, a.out, frames, fstate, blocks, comp, (const CompState*)cstate,
                         (const uint8_t*)(ws + W.lits), (const uint64_t*)seqs, (const uint16_t*)fses, f0, f1, redo);
      if (tm) if ((e = dom(DOM_K4, 1)) != hipSuccess) return e;
    }
    return hipSuccess;
  };
  auto k4f = [&](const uint32_t* list, uint32_t n, hipStream_t st) -> hipError_t {
    if (n) {
      if ((e = dom(DOM_K4F, 0)) != hipSuccess) return e;
      hipLaunchKernelGGL(zd_k_execute_lds, dim3(n), dim3(K4F_T), 0, st, a.src, a.out, frames, fstate, blocks, comp,
                         (const CompState*)cstate, (const uint8_t*)(ws + W.lits), (const uint64_t*)seqs,
                         (const uint16_t*)fses, list);
      if ((e = dom(DOM_K4F, 1)) != hipSuccess) return e;
    }
    return hipSuccess;
  };
  if (fz) {
    // K1's sequence half + K3 + K4 per group of four frames; K2 (forked) signals its workgroups;
    // then the redo pass for the frames the fused kernel flagged (normally none:
    // two launches whose workgroups exit at once)
    uint8_t* redo = ws + W.redo;
    const uint32_t k2need = fork ? (a.n_huf + K2_BLOCKS - 1) / K2_BLOCKS : 0;
    if ((e = dom(DOM_FUSED, 0)) != hipSuccess) return e;
    if (a.k3_lat)
      hipLaunchKernelGGL(zd_k_fused<true>, dim3((a.n_frames + FZ_FRAMES - 1) / FZ_FRAMES), dim3(128 * FZ_FRAMES), 0, s,
                         a.src, a.out, frames, fstate, blocks, comp, cstate, (const uint8_t*)(ws + W.lits), seqs,
                         fses, a.n_frames, (const uint32_t*)(ws + W.k2done), k2need, redo);
    else
      hipLaunchKernelGGL(zd_k_fused<false>, dim3((a.n_frames + FZ_FRAMES - 1) / FZ_FRAMES), dim3(64 * FZ_WAVES), 0, s,
                         a.src, a.out, frames, fstate, blocks, comp, cstate, (const uint8_t*)(ws + W.lits), seqs,
                         fses, a.n_frames, (const uint32_t*)(ws + W.k2done), k2need, redo);
    if ((e = dom(DOM_FUSED, 1)) != hipSuccess) return e;
    if (fork)
      if ((e = hipStreamWaitEvent(s, a.join, 0)) != hipSuccess) return e;
    k3((const uint32_t*)(ws + W.list_seq), a.n_seq, s, redo);
    if ((e = k4(0, a.n_frames, s, redo)) != hipSuccess) return e;
  } else {
    k3((const uint32_t*)(ws + W.list_seq), a.n_seq, s, nullptr);
    if (fork)
      if ((e = hipStreamWaitEvent(s, a.join, 0)) != hipSuccess) return e;
    if (a.events) if ((e = hipEventRecord(a.events[4], s)) != hipSuccess) return e;
    if ((e = k4(0, a.n_frames, s, nullptr)) != hipSuccess) return e;
    if ((e = k4f((const uint32_t*)(ws + W.list_k4f), a.n_k4f, s)) != hipSuccess) return e;
  }
  if (a.events) if ((e = hipEventRecord(a.events[5], s)) != hipSuccess) return e;
  if (a.n_jframes) {
    auto* jframes = (const JFrame*)(ws + W.jframes);
    auto* jd = (const JBlkDesc*)(ws + W.jblkd);
    auto* jb = (JBlk*)(ws + W.jblk);
    auto* jseg = (JSeg*)(ws + W.jseg);
    auto* jsd = (const JSegDesc*)(ws + W.jsegd);
    auto* jst = (uint32_t*)(ws + W.jst);
    auto* pend = (uint32_t*)(ws + W.jpend);
    if ((e = dom(DOM_K4J, 0)) != hipSuccess) return e;
    hipLaunchKernelGGL(zd_k_jsum, dim3(a.n_jseg), dim3(64), 0, s, a.src, (const FrameState*)fstate, blocks, comp,
                       (const CompState*)cstate, (const uint64_t*)seqs, (const uint16_t*)fses, jframes, jd, jsd, jseg);
    hipLaunchKernelGGL(zd_k_jsum_blocks, dim3((a.n_jblk + 63) / 64), dim3(64), 0, s, (const FrameState*)fstate,
                       blocks, comp, (const CompState*)cstate, jframes, jd, a.n_jblk, jb, jseg);
    hipLaunchKernelGGL(zd_k_jprefix, dim3(a.n_jframes), dim3(64 * JP_WAVES), 0, s, frames, fstate, jframes, jd, jb);
    hipLaunchKernelGGL(zd_k_jscatter, dim3(a.n_jseg), dim3(64), 0, s, a.src, fstate, blocks, comp,
                       (const CompState*)cstate, (const uint8_t*)(ws + W.lits), (const uint64_t*)seqs,
                       (const uint16_t*)fses, jframes, jd, (const JBlk*)jb, (const JSeg*)jseg, jsd, jst);
    const uint64_t gw = (a.j_pieces + 16 * JW_K - 1) / (16 * JW_K);   // pieces per workgroup sweep
    const uint64_t gmax = 8ull * a.cus;                              // what fits at once: 8 workgroups per CU
    const dim3 gr((uint32_t)(gw < gmax ? (gw + 7) & ~7ull : (gmax + 7) & ~7ull));   // a multiple of 8 (one eighth per XCD)
    // round 1 one launch, the rest as one launch of sweeps
    // (one launch of all the sweeps: 1.43 ms for the rounds of c3s, against
    // 1.38 with the first round launched alone; three launches, 1.38 too)
    const uint32_t nr = a.j_rounds < 2 ? a.j_rounds : 2u;
    for (uint32_t r = 1; r <= nr; r++)
      hipLaunchKernelGGL(zd_k_jround, gr, dim3(256), 0, s, a.out, frames, fstate, jframes, a.n_jframes,
                         a.j_pieces, jst, pend, ws + W.jdone, r > 1 ? a.j_hops2 : a.j_hops, r, (uint32_t)(r == nr),
                         r == nr ? a.j_rounds - nr + 1 : 1u);
    if ((e = dom(DOM_K4J, 1)) != hipSuccess) return e;
  }
  if (a.events) if ((e = hipEventRecord(a.events[6], s)) != hipSuccess) return e;
  return hipGetLastError();
}

#ifdef ZD_FZ_TRACE
}  // namespace zd
extern "C" int zd_debug_fz_trace(uint64_t* out, uint64_t* k2end) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(zd::fz_tr), sizeof(zd::fz_tr), 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(k2end, HIP_SYMBOL(zd::fz_k2end), 8, 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return 0;
}
namespace zd {
#endif
#ifdef ZD_K1_PROF
}  // namespace zd
extern "C" int zd_debug_k1_prof(uint64_t out[8], int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(zd::k1_prof), 64, 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (reset) {
    static const uint64_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(zd::k1_prof), z, 64, 0, hipMemcpyHostToDevice) != hipSuccess) return -1;
  }
  return 0;
}
namespace zd {
#endif
// The per-launch state reset of zd_decode_async in one launch: frame states
// from their device copies, block states, K1's tree list and deep-pool
// counters, K4J's round counters and done flags (six copy / fill launches
// before, ~5 us each on the path of a few-frame plan).
__global__ __launch_bounds__(256) void zd_k_reset(uint8_t* ws, Workspace W, uint64_t fs_words, uint64_t cs_words,
                                                  uint32_t jp_words, uint64_t jdone_bytes) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x, nt = (uint64_t)gridDim.x * 256;
  uint32_t* fs = (uint32_t*)(ws + W.frame_state);
  const uint32_t* fs0 = (const uint32_t*)(ws + W.frame_state0);
  for (uint64_t i = t; i < fs_words; i += nt) fs[i] = fs0[i];
  uint32_t* cs = (uint32_t*)(ws + W.comp_state);
  for (uint64_t i = t; i < cs_words; i += nt) cs[i] = 0;
  if (t == 0) {
    *(uint32_t*)(ws + W.huge) = 0;
    *(uint32_t*)(ws + W.deep) = 0;
  }
  uint32_t* jp = (uint32_t*)(ws + W.jpend);
  for (uint64_t i = t; i < jp_words; i += nt) jp[i] = 0;
  u32x4* jd = (u32x4*)(ws + W.jdone);
  const uint64_t n16 = jdone_bytes / 16;
  for (uint64_t i = t; i < n16; i += nt) jd[i] = (u32x4){0, 0, 0, 0};
  if (t < jdone_bytes % 16) (ws + W.jdone)[16 * n16 + t] = 0;
}
hipError_t launch_reset(uint8_t* ws, const Workspace& W, uint64_t n_frames, uint64_t n_comps, bool k4j,
                        uint64_t j_pieces, hipStream_t s) {
  const uint64_t fs_words = n_frames * sizeof(FrameState) / 4, cs_words = std::max<uint64_t>(n_comps, 1) * sizeof(CompState) / 4;
  const uint32_t jp_words = k4j ? (uint32_t)(J_MAX_ROUNDS + 1) : 0u;
  const uint64_t jdone = k4j ? std::max<uint64_t>(j_pieces, 1) : 0;
  const uint64_t work = std::max(std::max(fs_words, cs_words), jdone / 16 + 16);
  const uint32_t grid = (uint32_t)std::min<uint64_t>(2048, (work + 1023) / 1024);
  static_assert(sizeof(FrameState) % 4 == 0 && sizeof(CompState) % 4 == 0, "zd_k_reset: u32 words");
  hipLaunchKernelGGL(zd_k_reset, dim3(grid), dim3(256), 0, s, ws, W, fs_words, cs_words, jp_words, jdone);
  return hipGetLastError();
}

hipError_t launch_compact(const uint8_t* staging, uint8_t* dst, const uint64_t* d_from, const uint64_t* d_to,
                          const uint64_t* d_len, uint32_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(zd_k_compact, dim3(n, COMPACT_SPLIT), dim3(256), 0, s, staging, dst, d_from, d_to, d_len);
  return hipGetLastError();
}


// ---------------------------------------------------------------------------
// Device header walk: the frame / block header walk of the host
// planner (zd_host.cpp plan_index) for an input resident in HBM, with the
// same code (zd_walk.h index_frame: Frame::parse / Header::parse /
// Block::parse, frame.rs:61-230, block.rs:43-72, and the fixed-size parts of
// LiteralsSection::parse / Sequences::parse, literals.rs:88-206,
// sequences.rs:52-143).  One wave per byte range [lo, hi): a range other than
// the first finds its first frame magic number (64 lanes x 16 positions per
// step), then lane 0 walks the chain of frames that start inside the range; a
// candidate whose frame fails at once was a magic number inside data and the
// scan goes on after it (the host walk's rule).  Count pass: the range's
// summary (WalkRange); fill pass: its frames and blocks at f_off / b_off
// (block indices global, so all ranges share one block array).
// ---------------------------------------------------------------------------
struct WalkCount {
  uint32_t n = 0;
  __device__ size_t size() const { return n; }
  __device__ void push(const HostBlock&) { n++; }
};
struct WalkFill {
  HostBlock* out;
  uint64_t base;
  uint32_t n = 0;
  __device__ size_t size() const { return base + n; }
  __device__ void push(const HostBlock& b) { out[base + n++] = b; }
};

// First position q in [p, hi) with a frame magic number at src[q..q+4)
// (q + 4 <= n), else hi.  Whole wave, 4 KiB a step: each lane checks 64
// positions from 68 loaded bytes (four 16-byte loads in flight), a
// position's word is one alignbyte of two loaded dwords.  (1 KiB steps of
// 16 positions per lane took ~11 us each: latency-bound.)
__device__ uint64_t walk_scan(const uint8_t* __restrict__ src, uint64_t n, uint64_t p, uint64_t hi, int lane) {
  typedef uint32_t u32a1 __attribute__((aligned(1)));
  for (uint64_t base = p; base < hi; base += 4096) {
    const uint64_t q0 = base + 64 * (uint64_t)lane;
    uint64_t hit = 0;                            // bit j: a magic number at q0 + j
    if (q0 < hi) {
      uint32_t d[17];
      if (q0 + 68 <= n) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const u32x4a1 v = *(const u32x4a1*)(src + q0 + 16 * i);
          d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
        }
        d[16] = *(const u32a1*)(src + q0 + 64);
      } else {
        for (int i = 0; i < 17; i++) {
          uint32_t w = 0;
          for (int b = 0; b < 4; b++) {
            const uint64_t q = q0 + 4 * i + b;
            w |= (uint32_t)(q < n ? src[q] : 0) << (8 * b);
          }
          d[i] = w;
        }
      }
#pragma unroll
      for (int j = 0; j < 64; j++) {
        const uint32_t m = __builtin_amdgcn_alignbyte(d[(j >> 2) + 1], d[j >> 2], j & 3);
        hit |= (uint64_t)magic_word(m) << j;
      }
      // positions at or past hi, or whose word runs past n, do not count
      const uint64_t lim = min(hi, n >= 3 ? n - 3 : 0);
      if (q0 + 64 > lim) hit &= lim > q0 ? ((1ull << (lim - q0)) - 1) : 0;
    }
    const uint64_t m = __ballot(hit != 0);
    if (m) {
      const int l = __ffsll((long long)m) - 1;
      const uint32_t fj = (uint32_t)__shfl((int)(hit ? __ffsll((long long)hit) - 1 : 0), l, 64);
      return base + 64 * (uint64_t)l + fj;
    }
  }
  return hi;
}

template <bool FILL>
__global__ __launch_bounds__(64) void zd_k_walk(const uint8_t* __restrict__ src, uint64_t n, uint64_t first,
                                               uint64_t chunk, uint32_t nranges, WalkRange* wr,
                                               HostFrame* frames, HostBlock* blocks) {
  const uint32_t k = blockIdx.x;
  const int lane = threadIdx.x;
  if (k >= nranges) return;
  const uint64_t lo = first + (uint64_t)k * chunk;
  const uint64_t hi = lo + chunk < n ? lo + chunk : n;
  if (FILL) {
    if (lane) return;
    WalkRange R = wr[k];
    if (!R.nframes) return;
    Bytes in{src + R.p0, n - R.p0};
    WalkFill sink{blocks, R.b_off};
    for (uint32_t f = 0; f < R.nframes; f++) {
      HostFrame hf;
      index_frame(src, in, &hf, sink);
      frames[R.f_off + f] = hf;
    }
    return;
  }
  uint64_t p = lo;
#ifdef ZD_WALK_PROF
  uint64_t t_scan = 0, t_walk = 0, t0 = __builtin_amdgcn_s_memtime();
  uint32_t tries = 0;
#endif
  for (;;) {
    if (k) {
      p = walk_scan(src, n, p, hi, lane);
#ifdef ZD_WALK_PROF
      t_scan += __builtin_amdgcn_s_memtime() - t0; t0 = __builtin_amdgcn_s_memtime(); tries++;
#endif
      if (p >= hi) break;
    }
    uint32_t nf = 0, nb = 0;
    int st = 0;
    uint64_t end = 0;
    if (lane == 0) {
      Bytes in{src + p, n - p};
      WalkCount sink;
      while (in.n && (uint64_t)(in.p - src) < hi) {
        HostFrame hf;
        const int r = index_frame(src, in, &hf, sink);
        nf++;
        if (r) { st = r; break; }
      }
      nb = sink.n;
      end = (uint64_t)(in.p - src);
    }
    st = __shfl(st, 0, 64);
    nf = (uint32_t)__shfl((int)nf, 0, 64);
#ifdef ZD_WALK_PROF
    t_walk += __builtin_amdgcn_s_memtime() - t0; t0 = __builtin_amdgcn_s_memtime();
    if (lane == 0 && (k == 1 || k == 100 || k == 1000 || k == 5000))
      printf("walk range %u: lo %llu p %llu scan %llu walk %llu cycles, tries %u, frames %u\n", k,
             (unsigned long long)lo, (unsigned long long)p, (unsigned long long)t_scan, (unsigned long long)t_walk,
             tries, nf);
#endif
    if (k && st && nf == 1) { p++; continue; }       // a magic number inside data: look further
    if (lane == 0) {
      WalkRange R{};
      R.p0 = p; R.end = end; R.nframes = nf; R.nblocks = nb; R.status = st;
      wr[k] = R;
    }
    return;
  }
  if (lane == 0) {
    WalkRange R{};
    R.p0 = hi; R.end = hi;
    wr[k] = R;
  }
}

// ---------------------------------------------------------------------------
// Device descriptors (zd_plan_create_device): the planner's
// per-frame pass (zd_plan.h plan_frame, the host planner's own code) over the
// device walk's frame / block index, one lane per frame.  A shape pass (the
// plan-wide inputs of routing: frames that are not single-block zstd frames,
// K4J candidates), a count pass (each frame's PlanCounts from zero, and the
// largest K4J frame's sequence count), an
// exclusive scan over frames (per 256-frame tile, then the tiles), and a fill
// pass that writes CompBlock / BlockRec / FrameDesc / FrameState, the work
// lists, K0's pieces and the K4J descriptors straight into the plan's workspace.  Only the plan's
// totals and the frames' output offsets and capacities go back to the host.
// ---------------------------------------------------------------------------
struct DevJMax {              // the largest K4J frame's sequence count (PlanShape::jmaxseq)
  unsigned long long* m;
  __device__ void note(uint64_t n) { if (n) atomicMax(m, (unsigned long long)n); }
};
__global__ __launch_bounds__(256) void zd_k_plan_shape(const HostFrame* __restrict__ frames, uint64_t nf,
                                                       uint32_t k4j_min, PlanShape* out) {
  const uint64_t f = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  bool multi = false, jc = false;
  if (f < nf) {
    const HostFrame& hf = frames[f];
    multi = hf.d.kind != ZD_FRAME_ZSTD || hf.key != KEY_NONE || hf.nb != 1;
    jc = hf.key == KEY_NONE && hf.ncomp >= k4j_min;
  }
  const uint32_t m = (uint32_t)__popcll(__ballot(multi)), j = (uint32_t)__popcll(__ballot(jc));
  if ((threadIdx.x & 63) == 0) {
    if (m) atomicAdd(&out->multi, m);
    if (j) atomicAdd(&out->jcand, j);
  }
}
__global__ __launch_bounds__(256) void zd_k_plan_count(PlanCtx X, const HostFrame* __restrict__ frames,
                                                       const HostBlock* __restrict__ blocks, uint64_t nf,
                                                       PlanCounts* cnt, PlanShape* shape) {
  const uint64_t f = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (f >= nf) return;
  PlanCounts c{};
  const Sink none{};
  DevJMax jm{(unsigned long long*)&shape->jmaxseq};
  plan_frame<false, DevJMax>(X, frames[f], blocks, c, none, &jm);
  cnt[f] = c;
}
// Exclusive scan of the PlanCounts words over frames, in place: tile t's
// words (256 frames) scanned in LDS, its totals to tot[t]; then one
// workgroup scans the tiles (lane j: word j); then every frame adds its
// tile's start.  tot[ntiles] = the plan's totals.
__global__ __launch_bounds__(256) void zd_k_plan_scan_tiles(uint64_t* cnt, uint64_t nf, uint64_t* tot) {
  __shared__ uint64_t s[256];
  const uint64_t f = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (int w = 0; w < PLAN_FIELDS; w++) {
    const uint64_t v = f < nf ? cnt[f * PLAN_FIELDS + w] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
      const uint64_t a = threadIdx.x >= (unsigned)d ? s[threadIdx.x - d] : 0;
      __syncthreads();
      s[threadIdx.x] += a;
      __syncthreads();
    }
    if (f < nf) cnt[f * PLAN_FIELDS + w] = s[threadIdx.x] - v;    // exclusive within the tile
    if (threadIdx.x == 255) tot[(uint64_t)blockIdx.x * PLAN_FIELDS + w] = s[255];
    __syncthreads();
  }
}
__global__ __launch_bounds__(64) void zd_k_plan_scan_sums(uint64_t* tot, uint64_t ntiles) {
  const int w = threadIdx.x;
  if (w >= PLAN_FIELDS) return;
  uint64_t acc = 0;
  for (uint64_t t = 0; t < ntiles; t++) {
    const uint64_t v = tot[t * PLAN_FIELDS + w];
    tot[t * PLAN_FIELDS + w] = acc;
    acc += v;
  }
  tot[ntiles * PLAN_FIELDS + w] = acc;
}
__global__ __launch_bounds__(256) void zd_k_plan_fill(PlanCtx X, const HostFrame* __restrict__ frames,
                                                      const HostBlock* __restrict__ blocks, uint64_t nf,
                                                      const uint64_t* __restrict__ cnt, const uint64_t* __restrict__ tot,
                                                      Sink S) {
  const uint64_t f = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (f >= nf) return;
  PlanCounts c;
  uint64_t* cw = (uint64_t*)&c;
  for (int w = 0; w < PLAN_FIELDS; w++) cw[w] = cnt[f * PLAN_FIELDS + w] + tot[(uint64_t)blockIdx.x * PLAN_FIELDS + w];
  plan_frame<true, DevJMax>(X, frames[f], blocks, c, S, (DevJMax*)nullptr);
}

hipError_t launch_plan_shape(const HostFrame* frames, uint64_t nf, uint32_t k4j_min, PlanShape* out, hipStream_t s) {
  hipError_t e = hipMemsetAsync(out, 0, sizeof(PlanShape), s);
  if (e != hipSuccess) return e;
  if (nf) hipLaunchKernelGGL(zd_k_plan_shape, dim3((uint32_t)((nf + 255) / 256)), dim3(256), 0, s, frames, nf, k4j_min, out);
  return hipGetLastError();
}
hipError_t launch_plan_count(const PlanCtx& X, const HostFrame* frames, const HostBlock* blocks, uint64_t nf,
                             uint64_t* cnt, uint64_t* tot, PlanShape* shape, hipStream_t s) {
  const uint32_t nt = (uint32_t)((nf + 255) / 256);
  if (nf) {
    hipLaunchKernelGGL(zd_k_plan_count, dim3(nt), dim3(256), 0, s, X, frames, blocks, nf, (PlanCounts*)cnt, shape);
    hipLaunchKernelGGL(zd_k_plan_scan_tiles, dim3(nt), dim3(256), 0, s, cnt, nf, tot);
  }
  hipLaunchKernelGGL(zd_k_plan_scan_sums, dim3(1), dim3(64), 0, s, tot, (uint64_t)nt);
  return hipGetLastError();
}
hipError_t launch_plan_fill(const PlanCtx& X, const HostFrame* frames, const HostBlock* blocks, uint64_t nf,
                            const uint64_t* cnt, const uint64_t* tot, const Sink& S, hipStream_t s) {
  if (nf)
    hipLaunchKernelGGL(zd_k_plan_fill, dim3((uint32_t)((nf + 255) / 256)), dim3(256), 0, s, X, frames, blocks, nf, cnt,
                       tot, S);
  return hipGetLastError();
}

hipError_t launch_walk(const uint8_t* src, uint64_t n, uint64_t first, uint64_t chunk, uint32_t nranges, WalkRange* wr,
                       HostFrame* frames, HostBlock* blocks, bool fill, hipStream_t s) {
  if (!nranges) return hipSuccess;
  if (fill)
    hipLaunchKernelGGL(zd_k_walk<true>, dim3(nranges), dim3(64), 0, s, src, n, first, chunk, nranges, wr, frames, blocks);
  else
    hipLaunchKernelGGL(zd_k_walk<false>, dim3(nranges), dim3(64), 0, s, src, n, first, chunk, nranges, wr, frames, blocks);
  return hipGetLastError();
}

}  // namespace zd
