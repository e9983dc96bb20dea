// zd_kernels.hip — gfx950 kernels of the ZSTD block-decode path.
//
//   K1 zd_k_tables     one wave per compressed block: Huffman tree description
//                      -> LUT, FSE table descriptions -> decode tables
//                      (replaces huffman.rs:80-203, fse.rs:16-202,
//                      sequences.rs:91-187 table construction)
//   K2 zd_k_huffman    one wave per Huffman-literal block, LUT in LDS, one lane
//                      per stream (replaces literals.rs:49-86 + huffman.rs:205-218)
//   K3 zd_k_sequences  one wave per block, tables in LDS, FSE state machine
//                      (replaces sequences.rs:191-237 + decoders/sequence.rs)
//   K4 zd_k_execute    one wave per frame, 8 KiB LDS window ring, 64 sequences
//                      per step: repeat-offset transforms by wave scan, literal
//                      and match copies into the ring, aligned 16-B flushes to
//                      HBM (replaces decoding_context.rs:50-106 + block.rs:74-99)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/zd.h"
#include "zd_common.h"
#include "zd_launch.h"

namespace zd {

const char* const kKernelNames[N_KERNELS] = {"zd_k_tables", "zd_k_huffman", "zd_k_sequences", "zd_k_execute"};

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

// ForwardBitParser (parsing.rs:114-189), LSB-first, byte loads (headers only).
struct FwBits {
  const uint8_t* d;
  uint32_t nbytes;
  uint32_t pos;
  __device__ inline uint32_t bits(uint32_t at, int len) const {   // len <= 24, within range
    uint32_t v = 0;
    uint32_t b0 = at >> 3, b1 = (at + len - 1) >> 3;
    for (uint32_t b = b1 + 1; b-- > b0;) v = (v << 8) | d[b];
    v >>= (at & 7);
    return len >= 32 ? v : (v & ((1u << len) - 1));
  }
  __device__ inline int peek(int len, uint32_t* v) const {
    if ((int64_t)nbytes * 8 - pos < len) return ZD_E_NOT_ENOUGH_BITS;
    *v = len ? bits(pos, len) : 0;
    return 0;
  }
  __device__ inline int take(int len, uint32_t* v) {
    if (int r = peek(len, v)) return r;
    pos += len;
    return 0;
  }
  __device__ inline uint32_t bytes_read() const { return pos / 8 + (pos % 8 > 0); }
};

// parse_fse_table (fse.rs:16-69)
__device__ int parse_ncount(FwBits& in, uint8_t* al_out, int16_t* dist, uint32_t* nsym_out) {
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
    uint32_t lower_mask = (1u << (bits - 1)) - 1;
    uint32_t threshold = (1u << bits) - 1 - ((uint32_t)remaining + 1);
    int32_t decoded;
    if ((pk & lower_mask) < threshold) {
      if (int r = in.take(bits - 1, &v)) return r;
      decoded = (int32_t)v;
    } else if (pk > lower_mask) {
      if (int r = in.take(bits, &v)) return r;
      decoded = (int32_t)v - (int32_t)threshold;
    } else {
      if (int r = in.take(bits, &v)) return r;
      decoded = (int32_t)v;
    }
    int32_t proba = decoded - 1;
    remaining -= proba < 0 ? -proba : proba;
    if (n_sym < 256) dist[n_sym] = (int16_t)proba;
    n_sym++;
    if (proba == 0) {
      for (;;) {
        if (int r = in.take(2, &v)) return r;
        for (uint32_t z = 0; z < v; z++) {
          if (n_sym < 256) dist[n_sym] = 0;
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
// (in position order) gets nextState = count(s) + u, nbits = al -
// highbit(nextState), baseline = (nextState << nbits) - T, which equals the
// reference's parts/base_width construction (fse.rs:169-189).  `-1` symbols
// count as 1.  sym/next are LDS scratch (T and 256 entries).
__device__ int build_fse(int al, const int16_t* dist, uint32_t nsym, uint32_t* table, uint16_t* sym, uint16_t* next) {
  if (al > FSE_MAX_AL) return ZD_E_LARGE_ACCURACY_LOG;
  uint32_t T = 1u << al;
  uint32_t zero_pos = T;
  for (uint32_t s = 0; s < nsym; s++) {
    if (dist[s] == -1) {
      if (zero_pos == 0) return ZD_E_REF_PANIC;
      sym[--zero_pos] = (uint16_t)s;
    }
  }
  uint32_t pos = 0, step = (T >> 1) + (T >> 3) + 3, mask = T - 1, placed = 0;
  for (uint32_t s = 0; s < nsym; s++) {
    for (int k = 0; k < dist[s]; k++) {
      if (zero_pos == 0) return ZD_E_REF_PANIC;   // the reference loops forever
      sym[pos] = (uint16_t)s;
      placed++;
      pos = (pos + step) & mask;
      while (pos >= zero_pos) pos = (pos + step) & mask;
    }
  }
  if (placed != zero_pos) return ZD_E_CORRUPTED_TABLE;
  for (uint32_t s = 0; s < nsym; s++) next[s] = dist[s] > 0 ? (uint16_t)dist[s] : (dist[s] == -1 ? 1 : 0);
  for (uint32_t i = 0; i < T; i++) {
    uint32_t s = sym[i];
    uint32_t ns = next[s]++;
    int nb = al - highbit32(ns);
    uint32_t base = (ns << nb) - T;
    table[i] = fse_entry(s, (uint32_t)nb, base);
  }
  return 0;
}

// ---------------------------------------------------------------------------
// K1: tables
// ---------------------------------------------------------------------------
struct K1Smem {
  uint16_t lut[LUT_ENTRIES];        // 8 KiB
  uint16_t prefix[LUT_ENTRIES + 1]; // rare path: filled-entry prefix counts
  uint32_t fse[FSE_ENTRIES];        // 2 KiB
  uint16_t sym[FSE_ENTRIES];
  uint16_t next[256];
  int16_t dist[256];
  uint8_t weights[MAX_WEIGHTS];
  uint8_t widths[MAX_WEIGHTS + 1];
  int status;
  int p;
  uint32_t n;
  int holes;
};

// Huffman description -> LUT (huffman.rs:80-203).  Lane 0 parses; the wave fills.
__device__ void k1_huffman(const uint8_t* src, const uint8_t* src_end, const CompBlock& C, uint32_t ci,
                           CompState* cstate, FrameState* fstate, uint16_t* luts, K1Smem& sm) {
  const int lane = threadIdx.x;
  const uint8_t* desc = src + C.src + C.lit_data;
  if (lane == 0) {
    int st = 0;
    uint32_t nw = 0;
    uint8_t h = desc[0];
    if (h < 128) {
      // parse_fse (huffman.rs:108-130)
      FwBits fw{desc + 1, h, 0};
      uint8_t al;
      uint32_t nsym;
      st = parse_ncount(fw, &al, sm.dist, &nsym);
      if (!st) st = build_fse(al, sm.dist, nsym, sm.fse, sm.sym, sm.next);
      BwBits bs;
      if (!st) st = bs.init(desc + 1 + fw.bytes_read(), h - fw.bytes_read(), src, src_end);
      if (!st) {
        // AlternatingDecoder (alternating.rs): initialize first, second
        uint32_t sa = 0, sb = 0, v;
        st = bs.take(al, &sa);
        if (!st) st = bs.take(al, &sb);
        bool last_updated_is_first = false, last_read_is_first = false;
        bool has_a = true, has_b = true;
        while (!st) {
          uint32_t cur = last_updated_is_first ? sb : sa;
          uint32_t nb = (sm.fse[cur] >> 8) & 0xFF;
          if ((int64_t)nb > bs.bitpos) break;
          // symbol()
          uint32_t w;
          if (last_read_is_first) { last_read_is_first = false; if (!has_b) { st = ZD_E_REF_PANIC; break; } w = sm.fse[sb] & 0xFF; has_b = false; }
          else { last_read_is_first = true; if (!has_a) { st = ZD_E_REF_PANIC; break; } w = sm.fse[sa] & 0xFF; has_a = false; }
          if (nw >= MAX_WEIGHTS - 2) { st = ZD_E_OUT_OF_DOMAIN; break; }
          sm.weights[nw++] = (uint8_t)w;
          // update_bits()
          uint32_t& s = last_updated_is_first ? sb : sa;
          bool& has = last_updated_is_first ? has_b : has_a;
          if (has) { st = ZD_E_REF_PANIC; break; }
          st = bs.take((int)nb, &v);
          if (st) break;
          s = (sm.fse[s] >> 16) + v;
          has = true;
          last_updated_is_first = !last_updated_is_first;
        }
        for (int k = 0; k < 2 && !st; k++) {
          uint32_t w;
          if (last_read_is_first) { last_read_is_first = false; if (!has_b) { st = ZD_E_REF_PANIC; break; } w = sm.fse[sb] & 0xFF; has_b = false; }
          else { last_read_is_first = true; if (!has_a) { st = ZD_E_REF_PANIC; break; } w = sm.fse[sa] & 0xFF; has_a = false; }
          sm.weights[nw++] = (uint8_t)w;
        }
      }
    } else {
      // parse_direct (huffman.rs:92-106): high nibble first
      nw = (uint32_t)h - 127;
      for (uint32_t i = 0; i < nw; i++) {
        uint8_t b = desc[1 + i / 2];
        sm.weights[i] = (i & 1) ? (b & 15) : (b >> 4);
      }
    }
    // from_weights (huffman.rs:177-203)
    int p = 0;
    if (!st) {
      uint32_t sum = 0;
      for (uint32_t i = 0; i < nw && !st; i++) {
        uint32_t w = sm.weights[i];
        if (!w) continue;
        if (w - 1 >= 32) { st = ZD_E_REF_PANIC; break; }
        uint32_t add = 1u << (w - 1);
        if (sum > 0xFFFFFFFFu - add) { st = ZD_E_REF_PANIC; break; }
        sum += add;
      }
      if (!st && sum == 0) st = ZD_E_REF_PANIC;
      if (!st) {
        p = highbit32(sum);
        if ((1ull << p) < sum) p++;
        if (p >= 32) st = ZD_E_REF_PANIC;
      }
      uint32_t manquant = 0;
      if (!st) {
        uint8_t rest = (uint8_t)((1u << p) - sum);
        if (rest == 0) st = ZD_E_REF_PANIC;   // D3
        else manquant = (uint32_t)highbit32(rest) + 1;
      }
      for (uint32_t i = 0; i < nw && !st; i++) {
        uint32_t w = sm.weights[i];
        if (w && w > (uint32_t)p + 1) st = ZD_E_REF_PANIC;
        sm.widths[i] = w ? (uint8_t)(p + 1 - w) : 0;
      }
      if (!st && manquant > (uint32_t)p + 1) st = ZD_E_REF_PANIC;
      if (!st) sm.widths[nw] = (uint8_t)(p + 1 - manquant);
      if (!st && p > LUT_MAX_BITS) st = ZD_E_OUT_OF_DOMAIN;
    }
    // from_number_of_bits + insert (huffman.rs:132-175): canonical placement,
    // longest codes first, ascending symbol (u8), leftmost free aligned slot.
    int holes = 0;
    if (!st) {
      uint32_t n = nw + 1, T = 1u << p, pos = 0;
      for (uint32_t e = 0; e < T; e++) sm.lut[e] = 0xFFFF;
      for (int w = p; w >= 1; w--) {
        uint32_t S = 1u << (p - w);
        for (uint32_t v = 0; v < 256; v++) {
          for (uint32_t i = v; i < n; i += 256) {
            if (sm.widths[i] != w) continue;
            pos = (pos + S - 1) & ~(S - 1);
            if (pos + S > T) continue;            // insert() returned false
            for (uint32_t e = pos; e < pos + S; e++) sm.lut[e] = (uint16_t)(v | (w << 8));
            pos += S;
          }
        }
      }
      // width-0 codes are never inserted (huffman.rs:163-165); anything left
      // unfilled is an Absent tree node
      if (pos != T) holes = 1;
      sm.n = n;
    }
    sm.status = st;
    sm.p = p;
    sm.holes = holes;
  }
  __syncthreads();
  const int st = sm.status, p = sm.p;
  if (st) {
    if (lane == 0) {
      uint32_t ph = (st == ZD_E_OUT_OF_DOMAIN) ? PH_LIMIT : PH_PARSE;
      key_min(fstate, C.frame, make_key(ph, C.block_in_frame, PS_HUF_DESC, 0, st));
    }
    return;
  }
  const uint32_t T = 1u << p;
  if (sm.holes) {
    // absent tree nodes: depth of the Absent node on each unfilled index's path
    if (lane == 0) {
      uint32_t c = 0;
      for (uint32_t e = 0; e < T; e++) { sm.prefix[e] = (uint16_t)c; c += sm.lut[e] != 0xFFFF; }
      sm.prefix[T] = (uint16_t)c;
    }
    __syncthreads();
    for (uint32_t e = lane; e < T; e += 64) {
      if (sm.lut[e] != 0xFFFF) continue;
      int d = 0;
      for (; d <= p; d++) {
        uint32_t lo = (e >> (p - d)) << (p - d), hi = lo + (1u << (p - d));
        if (sm.prefix[hi] == sm.prefix[lo]) break;
      }
      sm.lut[e] = (uint16_t)(LUT_ABSENT | (d << 8));
    }
    __syncthreads();
  }
  uint16_t* dst = luts + (uint64_t)C.lut_slot * LUT_ENTRIES;
  for (uint32_t e = lane; e < T; e += 64) dst[e] = sm.lut[e];
  if (lane == 0) cstate[ci].huf_bits = (uint8_t)p;
}

// Sequence tables (sequences.rs:91-187): RLE bytes, FSE descriptions, predefined.
__device__ void k1_sequences(const uint8_t* src, const CompBlock& C, uint32_t ci, CompState* cstate,
                             FrameState* fstate, uint32_t* fses, K1Smem& sm) {
  const int lane = threadIdx.x;
  const uint8_t* blk = src + C.src;
  uint32_t* slot = fses + (uint64_t)C.fse_slot * 3 * FSE_ENTRIES;
  uint32_t pos = C.seq_tables;
  for (int k = 0; k < 3; k++) {
    int mode = C.modes[k];
    if (lane == 0) {
      int st = 0, al = 0;
      if (mode == M_RLE) {
        if (pos >= C.size) st = ZD_E_NOT_ENOUGH_BYTES;
        else { sm.fse[0] = fse_entry(blk[pos], 0, 0); pos++; }
      } else if (mode == M_FSE) {
        if (pos >= C.size) st = ZD_E_EMPTY_SLICE;
        else {
          FwBits fw{blk + pos, C.size - pos, 0};
          uint8_t a;
          uint32_t nsym;
          st = parse_ncount(fw, &a, sm.dist, &nsym);
          if (!st) st = build_fse(a, sm.dist, nsym, sm.fse, sm.sym, sm.next);
          al = a;
          pos += fw.bytes_read();
        }
      } else if (mode == M_PREDEFINED) {
        const int16_t* d = k == 0 ? c_ll_default : (k == 1 ? c_of_default : c_ml_default);
        uint32_t nsym = k == 0 ? 36 : (k == 1 ? 29 : 53);
        al = k == 1 ? 5 : 6;
        for (uint32_t s = 0; s < nsym; s++) sm.dist[s] = d[s];
        st = build_fse(al, sm.dist, nsym, sm.fse, sm.sym, sm.next);
      }
      sm.status = st;
      sm.p = al;
    }
    __syncthreads();
    if (sm.status) {
      if (lane == 0) key_min(fstate, C.frame, make_key(PH_PARSE, C.block_in_frame, PS_SEQ_TABLES, k, sm.status));
      return;
    }
    if (mode != M_REPEAT) {
      uint32_t T = 1u << sm.p;
      for (uint32_t e = lane; e < T; e += 64) slot[k * FSE_ENTRIES + e] = sm.fse[e];
      if (lane == 0) cstate[ci].al[k] = (uint8_t)sm.p;
    }
    __syncthreads();
  }
  if (lane == 0) {
    // seq.bitstream = input.slice(input.len()) (sequences.rs:72)
    if (pos >= C.size) key_min(fstate, C.frame, make_key(PH_PARSE, C.block_in_frame, PS_SEQ_TABLES, 3, ZD_E_EMPTY_SLICE));
    cstate[ci].bs_off = pos;
    cstate[ci].bs_size = pos < C.size ? C.size - pos : 0;
  }
}

__global__ __launch_bounds__(64) void zd_k_tables(const uint8_t* __restrict__ src, uint64_t src_size,
                                                  const CompBlock* __restrict__ comp, CompState* cstate,
                                                  FrameState* fstate, const uint32_t* __restrict__ list,
                                                  uint16_t* luts, uint32_t* fses) {
  __shared__ K1Smem sm;
  const uint32_t ci = list[blockIdx.x];
  const CompBlock C = comp[ci];
  if (C.prebuilt) return;
  if (C.lit_type == LIT_COMPRESSED && C.host_stage > PS_HUF_DESC)
    k1_huffman(src, src + src_size, C, ci, cstate, fstate, luts, sm);
  __syncthreads();
  if (C.nseq > 0 && C.host_stage > PS_SEQ_TABLES) k1_sequences(src, C, ci, cstate, fstate, fses, sm);
}

// ---------------------------------------------------------------------------
// K2: Huffman literals.  Stream k decodes to k * ceil(R/4) (RFC 8878 §3.1.1.3.1.6);
// the reference concatenates streams decoded until empty (literals.rs:68-81),
// which is the same bytes whenever each stream holds its RFC share.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void zd_k_huffman(const uint8_t* __restrict__ src, uint64_t src_size,
                                                   const CompBlock* __restrict__ comp, CompState* cstate,
                                                   FrameState* fstate, const uint32_t* __restrict__ list,
                                                   const uint16_t* __restrict__ luts, uint8_t* lits) {
  __shared__ uint16_t lut[LUT_ENTRIES];
  __shared__ uint32_t counts[4];
  __shared__ int errs[4];
  const int lane = threadIdx.x;
  const uint32_t ci = list[blockIdx.x];
  const CompBlock C = comp[ci];
  const uint64_t key0 = fstate[C.frame].key;
  if (key0 != KEY_NONE && key_phase(key0) == PH_PARSE) return;
  const uint32_t hs = (uint32_t)C.huf_src;
  const int p = cstate[hs].huf_bits;
  if (p == 0) {   // LUT not built (K1 stopped: parse error or out of domain)
    if (lane == 0) cstate[ci].stop = 1;
    return;
  }
  const uint32_t T = 1u << p;
  const uint16_t* g = luts + (uint64_t)comp[hs].lut_slot * LUT_ENTRIES;
  for (uint32_t e = lane; e < T; e += 64) lut[e] = g[e];
  __syncthreads();
  const int m = C.nstreams;
  const uint32_t R = C.lit_regen;
  const uint32_t seg = (R + 3) / 4;
  if (lane < m) {
    const uint32_t* ssz = comp[ci].stream_size;
    uint32_t off = C.streams;
    for (int j = 0; j < lane; j++) off += ssz[j];
    const uint32_t start = (uint32_t)lane * seg;
    const uint32_t cap = lane < m - 1 ? seg : (R > start ? R - start : 0);
    uint8_t* out = lits + C.lit_out + start;
    BwBits bs;
    int st = bs.init(src + C.src + off, ssz[lane], src, src + src_size);
    uint32_t count = 0;
    while (!st && bs.bitpos > 0) {
      uint32_t idx = bs.peek(p);
      uint32_t e = lut[idx];
      uint32_t nb = (e >> 8) & 0x7F;
      if (e & LUT_ABSENT) {
        st = ((int64_t)nb <= bs.bitpos) ? ZD_E_REF_PANIC : ZD_E_NOT_ENOUGH_BITS;
        break;
      }
      if ((int64_t)nb > bs.bitpos) { st = ZD_E_NOT_ENOUGH_BITS; break; }
      bs.bitpos -= nb;
      if (count < cap) out[count] = (uint8_t)e;
      count++;
    }
    counts[lane] = count;
    errs[lane] = st;
    if (st) key_min(fstate, C.frame, make_key(PH_DECODE, C.block_in_frame, DS_LITERALS, lane, st));
  }
  __syncthreads();
  if (lane == 0) {
    bool err = false, ood = false;
    for (int k = 0; k < m; k++) err |= errs[k] != 0;
    uint32_t total = 0;
    for (int k = 0; k < m && !err; k++) {
      uint32_t cap = k < m - 1 ? seg : (R > (uint32_t)k * seg ? R - (uint32_t)k * seg : 0);
      if (k < m - 1 ? counts[k] != seg : counts[k] > cap) ood = true;
      total += counts[k];
    }
    if (ood && !err) key_min(fstate, C.frame, make_key(PH_LIMIT, C.block_in_frame, DS_LITERALS, 0, ZD_E_OUT_OF_DOMAIN));
    cstate[ci].lit_count = total;
    if (err || ood) cstate[ci].stop = 1;
  }
}

// ---------------------------------------------------------------------------
// K3: sequences (sequences.rs:191-237, decoders/sequence.rs:41-88)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void zd_k_sequences(const uint8_t* __restrict__ src, uint64_t src_size,
                                                     const CompBlock* __restrict__ comp, CompState* cstate,
                                                     FrameState* fstate, const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ fses, uint32_t* seq_ll,
                                                     uint32_t* seq_of, uint32_t* seq_ml) {
  __shared__ uint32_t tab[3][FSE_ENTRIES];
  __shared__ int als[3];
  const int lane = threadIdx.x;
  const uint32_t ci = list[blockIdx.x];
  const CompBlock C = comp[ci];
  const uint64_t key0 = fstate[C.frame].key;
  if (key0 != KEY_NONE && key_phase(key0) == PH_PARSE) return;
  for (int k = 0; k < 3; k++) {
    const uint32_t s = (uint32_t)C.tab_src[k];
    const int al = cstate[s].al[k];
    const uint32_t* g = fses + ((uint64_t)comp[s].fse_slot * 3 + k) * FSE_ENTRIES;
    for (uint32_t e = lane; e < (1u << al); e += 64) tab[k][e] = g[e];
    if (lane == 0) als[k] = al;
  }
  __syncthreads();
  if (lane != 0) return;
  const CompState cs = cstate[ci];
  BwBits bs;
  int st = bs.init(src + C.src + cs.bs_off, cs.bs_size, src, src + src_size);
  uint32_t sLL = 0, sOF = 0, sML = 0, v;
  // SequenceDecoder::initialize: LL, OF, ML (sequence.rs:59-65)
  if (!st) st = bs.take(als[0], &sLL);
  if (!st) st = bs.take(als[1], &sOF);
  if (!st) st = bs.take(als[2], &sML);
  uint32_t* oll = seq_ll + C.seq_out;
  uint32_t* oof = seq_of + C.seq_out;
  uint32_t* oml = seq_ml + C.seq_out;
  const uint32_t n = C.nseq;
  for (uint32_t i = 0; i < n && !st; i++) {
    const uint32_t eLL = tab[0][sLL], eOF = tab[1][sOF], eML = tab[2][sML];
    const uint32_t llc = eLL & 0xFF, ofc = eOF & 0xFF, mlc = eML & 0xFF;
    if (llc > 35 || mlc > 52 || ofc > 31) { st = ZD_E_SEQUENCE_CODE_MAX_EXCEEDED; break; }
    uint32_t ob, mb, lb;
    if ((st = bs.take((int)ofc, &ob))) break;
    if ((st = bs.take(c_ml_bits[mlc], &mb))) break;
    if ((st = bs.take(c_ll_bits[llc], &lb))) break;
    oof[i] = (1u << ofc) + ob;
    oml[i] = c_ml_base[mlc] + mb;
    oll[i] = c_ll_base[llc] + lb;
    if (i + 1 == n) break;
    // update_bits: LL, ML, OF (sequence.rs:80-88)
    if ((st = bs.take((eLL >> 8) & 0xFF, &v))) break;
    sLL = (eLL >> 16) + v;
    if ((st = bs.take((eML >> 8) & 0xFF, &v))) break;
    sML = (eML >> 16) + v;
    if ((st = bs.take((eOF >> 8) & 0xFF, &v))) break;
    sOF = (eOF >> 16) + v;
  }
  if (st) {
    key_min(fstate, C.frame, make_key(PH_DECODE, C.block_in_frame, DS_SEQUENCES, 0, st));
    cstate[ci].stop = 1;
  }
}

// ---------------------------------------------------------------------------
// K4: execute
// ---------------------------------------------------------------------------
constexpr int RING = 8192;
constexpr uint32_t RMASK = RING - 1;
constexpr uint32_t BATCH = 2048;

// Repeat-offset update as a transform of the 3-entry state: entry j of the
// result is either state[src_j] + val_j (src_j in 0..2) or the constant val_j
// (src_j == 3).  decoding_context.rs:50-75 per (offset_value, ll).
struct RepT {
  uint32_t src;      // 2 bits per entry
  int64_t v[3];
};

__device__ inline RepT rep_of(uint32_t ofv, uint32_t ll) {
  RepT t;
  t.v[0] = t.v[1] = t.v[2] = 0;
  auto S = [](uint32_t a, uint32_t b, uint32_t c) { return a | (b << 2) | (c << 4); };
  if (ofv > 3) { t.src = S(3, 0, 1); t.v[0] = (int64_t)ofv - 3; }
  else if (ofv == 3 && ll == 0) { t.src = S(0, 0, 1); t.v[0] = -1; }
  else if (ofv == 3 || (ofv == 2 && ll == 0)) t.src = S(2, 0, 1);
  else if (ofv == 2 || (ofv == 1 && ll == 0)) t.src = S(1, 0, 2);
  else t.src = S(0, 1, 2);   // (1, ll > 0): unchanged
  return t;
}

// (g after f)
__device__ inline int64_t sel3(int64_t a, int64_t b, int64_t c, uint32_t s) { return s == 0 ? a : (s == 1 ? b : c); }

__device__ inline RepT rep_compose(const RepT& g, const RepT& f) {
  RepT r;
  r.src = 0;
#pragma unroll
  for (int j = 0; j < 3; j++) {
    uint32_t s = (g.src >> (2 * j)) & 3;
    if (s == 3) { r.src |= 3u << (2 * j); r.v[j] = g.v[j]; }
    else { r.src |= ((f.src >> (2 * s)) & 3) << (2 * j); r.v[j] = sel3(f.v[0], f.v[1], f.v[2], s) + g.v[j]; }
  }
  return r;
}

__device__ inline int64_t shfl_up_i64(int64_t x, int d) {
  int lo = __shfl_up((int)(uint32_t)x, d, 64);
  int hi = __shfl_up((int)(uint32_t)((uint64_t)x >> 32), d, 64);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ inline int64_t readlane_i64(int64_t x, int l) {
  int lo = __shfl((int)(uint32_t)x, l, 64);
  int hi = __shfl((int)(uint32_t)((uint64_t)x >> 32), l, 64);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ inline uint32_t scan_incl_u32(uint32_t x, int lane) {
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

struct Exec {
  uint8_t* ring;
  uint8_t* out;          // frame output position 0
  uintptr_t out_abs;
  uint64_t pos;          // frame-relative decoded length
  uint64_t frontier;     // bytes [0, frontier) are in HBM
  uint64_t cap;
  int lane;

  __device__ inline uint8_t& R(uint64_t p) { return ring[(out_abs + p) & RMASK]; }

  // aligned 16-B stores of the completed chunks; the frame's head chunk by bytes
  __device__ void flush() {
    uintptr_t A = out_abs + frontier, E = out_abs + pos;
    uintptr_t c0 = A & ~(uintptr_t)15, c1 = E & ~(uintptr_t)15;
    for (uintptr_t c = c0 + 16 * (uintptr_t)lane; c < c1; c += 16 * 64) {
      if (c >= out_abs) {
        *(uint4*)c = *(const uint4*)&ring[c & RMASK];
      } else {
        for (uintptr_t b = out_abs; b < c + 16; b++) *(uint8_t*)b = ring[b & RMASK];
      }
    }
    if (c1 > A) frontier = c1 - out_abs;
  }
  __device__ void final_flush() {
    uintptr_t A = out_abs + frontier, E = out_abs + pos;
    for (uintptr_t b = A + lane; b < E; b += 64) *(uint8_t*)b = ring[b & RMASK];
    frontier = pos;
  }
  // append n bytes from s (or the fill byte when s == nullptr), through the ring
  __device__ bool emit(const uint8_t* s, uint8_t fill, uint64_t n) {
    for (uint64_t done = 0; done < n;) {
      uint32_t chunk = (uint32_t)min((uint64_t)BATCH, n - done);
      if (pos + chunk > cap) return false;
      for (uint32_t x = lane; x < chunk; x += 64) R(pos + x) = s ? s[done + x] : fill;
      __syncthreads();
      pos += chunk;
      done += chunk;
      flush();
    }
    return true;
  }
};

__device__ inline void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__global__ __launch_bounds__(64) void zd_k_execute(const uint8_t* __restrict__ src, uint8_t* outbase,
                                                   const FrameDesc* __restrict__ frames, FrameState* fstate,
                                                   const BlockRec* __restrict__ blocks,
                                                   const CompBlock* __restrict__ comp,
                                                   const CompState* __restrict__ cstate,
                                                   const uint8_t* __restrict__ lits,
                                                   const uint32_t* __restrict__ seq_ll,
                                                   const uint32_t* __restrict__ seq_of,
                                                   const uint32_t* __restrict__ seq_ml) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[RING];
  __shared__ uint8_t stage[BATCH];
  const int lane = threadIdx.x;
  const uint32_t f = blockIdx.x;
  const FrameDesc F = frames[f];
  FrameState* S = &fstate[f];
  const uint64_t key0 = S->key;
  if (key0 != KEY_NONE && key_phase(key0) == PH_PARSE) return;

  Exec X;
  X.ring = ring;
  X.out = outbase + F.out;
  X.out_abs = (uintptr_t)X.out;
  X.pos = F.out_len0;
  X.frontier = F.out_len0;
  X.cap = F.out_cap;
  X.lane = lane;
  // context API: the window ring starts with the tail of the existing output
  if (X.pos) {
    uint64_t lo = X.pos > (uint64_t)RING ? X.pos - RING : 0;
    for (uint64_t p = lo + lane; p < X.pos; p += 64) X.R(p) = X.out[p];
  }
  int64_t rep[3] = {(int64_t)S->rep[0], (int64_t)S->rep[1], (int64_t)S->rep[2]};
  uint64_t err_key = KEY_NONE;

  for (uint32_t j = 0; j < F.nblocks && err_key == KEY_NONE; j++) {
    const BlockRec B = blocks[F.first_block + j];
    if (key0 != KEY_NONE && key_phase(key0) == PH_DECODE && key_block(key0) <= j) break;
    if (B.type == 5) continue;
    if (B.type == 0 || B.type == 4) {
      if (!X.emit(src + B.src, 0, B.size)) err_key = make_key(PH_LIMIT, j, 0, 0, ZD_E_DST_TOO_SMALL);
      continue;
    }
    if (B.type == 1) {
      if (!X.emit(nullptr, B.rle, B.size)) err_key = make_key(PH_LIMIT, j, 0, 0, ZD_E_DST_TOO_SMALL);
      continue;
    }
    const CompBlock C = comp[B.comp];
    const CompState CS = cstate[B.comp];
    if (CS.stop) break;
    const uint8_t* lsrc = nullptr;
    uint8_t lfill = 0;
    uint64_t nl;
    if (C.lit_type == LIT_RAW) { lsrc = src + C.src + C.lit_data; nl = C.lit_regen; }
    else if (C.lit_type == LIT_RLE) { lfill = C.lit_rle; nl = C.lit_regen; }
    else { lsrc = lits + C.lit_out; nl = CS.lit_count; }
    uint64_t lit_cursor = 0;
    const uint32_t* LL = seq_ll + C.seq_out;
    const uint32_t* OF = seq_of + C.seq_out;
    const uint32_t* ML = seq_ml + C.seq_out;
    const uint32_t n = C.nseq;
    for (uint32_t s0 = 0; s0 < n && err_key == KEY_NONE;) {
      const uint32_t i = s0 + lane;
      const bool valid = i < n;
      const uint32_t ll = valid ? LL[i] : 0;
      const uint32_t ofv = valid ? OF[i] : 1;
      const uint32_t ml = valid ? ML[i] : 0;
      // repeat offsets: inclusive scan of transforms, then apply to `rep`
      RepT t = valid ? rep_of(ofv, ll) : rep_of(1, 1);
      for (int d = 1; d < 64; d <<= 1) {
        RepT u;
        u.src = __shfl_up(t.src, d, 64);
        u.v[0] = shfl_up_i64(t.v[0], d);
        u.v[1] = shfl_up_i64(t.v[1], d);
        u.v[2] = shfl_up_i64(t.v[2], d);
        if (lane >= d) t = rep_compose(t, u);
      }
      int64_t after[3];
#pragma unroll
      for (int k = 0; k < 3; k++) {
        uint32_t s = (t.src >> (2 * k)) & 3;
        after[k] = s == 3 ? t.v[k] : sel3(rep[0], rep[1], rep[2], s) + t.v[k];
      }
      const int64_t off = after[0];
      // positions
      const uint32_t tot = ll + ml;
      const uint32_t inc_tot = scan_incl_u32(tot, lane);
      const uint32_t inc_ll = scan_incl_u32(ll, lane);
      const uint32_t opos = inc_tot - tot, lpos = inc_ll - ll;
      // checks (decoding_context.rs:86-90, D9)
      const uint64_t before = X.pos + opos;
      const bool imp = valid && ((uint64_t)ll > nl - (lit_cursor + lpos) || lit_cursor + lpos > nl ||
                                 (off > 0 && (uint64_t)off > before + ll));
      const bool panic = valid && !imp && off <= 0;
      const uint64_t badm = __ballot(imp || panic);
      // batch: sequences whose bytes fit in BATCH
      const uint64_t fitm = __ballot(valid && inc_tot <= BATCH);
      uint32_t k = (uint32_t)__popcll(fitm);
      if (badm) {
        const int b = __ffsll((long long)badm) - 1;
        if ((uint32_t)b < (k ? k : 1u)) {
          const bool bimp = __shfl((int)imp, b, 64);
          err_key = make_key(PH_DECODE, j, DS_EXECUTE, s0 + b, bimp ? ZD_E_IMPOSSIBLE_VALUE : ZD_E_REF_PANIC);
          break;
        }
      }
      if (k > 0) {
        // ---- small path: lanes < k ----
        const uint32_t T = __shfl(inc_tot, k - 1, 64);
        const uint32_t L = __shfl(inc_ll, k - 1, 64);
        if (X.pos + T > X.cap) { err_key = make_key(PH_LIMIT, j, DS_EXECUTE, s0, ZD_E_DST_TOO_SMALL); break; }
        for (uint32_t x = lane; x < L; x += 64) stage[x] = lsrc ? lsrc[lit_cursor + x] : lfill;
        __syncthreads();
        const bool act = (uint32_t)lane < k;
        if (act) for (uint32_t x = 0; x < ll; x++) X.R(X.pos + opos + x) = stage[lpos + x];
        // matches
        const uint64_t q = X.pos + opos + ll;
        const uint64_t batch_end = X.pos + T;
        const uint64_t ring_lo = batch_end > (uint64_t)RING ? batch_end - RING : 0;
        const uint64_t slo = act && ml ? q - (uint64_t)off : 0;
        const uint64_t shi = act && ml ? slo + min((uint64_t)off, (uint64_t)ml) : 0;
        if (__ballot(act && ml && slo < ring_lo)) wait_vm();
        uint64_t done = __ballot(!act || ml == 0);
        __syncthreads();
        while (done != ~0ull) {
          const int U = __ffsll((long long)~done) - 1;
          const uint64_t qU = (uint64_t)readlane_i64((int64_t)q, U);
          const bool mine = !((done >> lane) & 1) && (lane == U || shi <= qU);
          if (mine) {
            uint64_t p = slo;
            for (uint32_t x = 0; x < ml; x++) {
              uint8_t byte = p >= ring_lo ? X.R(p) : X.out[p];
              X.R(q + x) = byte;
              p++;
              if (p == q) p = slo;
            }
          }
          done |= __ballot(mine);
          __syncthreads();
        }
        // advance
        const int last = (int)k - 1;
        rep[0] = readlane_i64(after[0], last);
        rep[1] = readlane_i64(after[1], last);
        rep[2] = readlane_i64(after[2], last);
        lit_cursor += L;
        X.pos += T;
        s0 += k;
        X.flush();
      } else {
        // ---- big path: lane 0's sequence alone ----
        const uint32_t ll0 = __shfl(ll, 0, 64), ml0 = __shfl(ml, 0, 64);
        const uint64_t off0 = (uint64_t)readlane_i64(off, 0);
        if (!X.emit(lsrc ? lsrc + lit_cursor : nullptr, lfill, ll0)) {
          err_key = make_key(PH_LIMIT, j, DS_EXECUTE, s0, ZD_E_DST_TOO_SMALL);
          break;
        }
        lit_cursor += ll0;
        for (uint32_t k0 = 0; k0 < ml0;) {
          const uint32_t P = min(BATCH, ml0 - k0);
          if (X.pos + P > X.cap) { err_key = make_key(PH_LIMIT, j, DS_EXECUTE, s0, ZD_E_DST_TOO_SMALL); break; }
          const uint64_t ps = X.pos;
          const uint64_t ring_lo = ps + P > (uint64_t)RING ? ps + P - RING : 0;
          const uint64_t lowest = ps > off0 ? ps - off0 : 0;
          if (lowest < ring_lo) wait_vm();
          for (uint32_t x = lane; x < P; x += 64) {
            const uint64_t m = off0 > P ? 0 : x / (uint32_t)off0;
            const uint64_t p = ps + x - off0 * (m + 1);
            X.R(ps + x) = p >= ring_lo ? X.R(p) : X.out[p];
          }
          __syncthreads();
          X.pos += P;
          k0 += P;
          X.flush();
        }
        rep[0] = readlane_i64(after[0], 0);
        rep[1] = readlane_i64(after[1], 0);
        rep[2] = readlane_i64(after[2], 0);
        s0 += 1;
      }
    }
    if (err_key != KEY_NONE) break;
    // leftover literals (decoding_context.rs:101-103)
    if (lit_cursor < nl && !X.emit(lsrc ? lsrc + lit_cursor : nullptr, lfill, nl - lit_cursor))
      err_key = make_key(PH_LIMIT, j, DS_EXECUTE, n, ZD_E_DST_TOO_SMALL);
  }
  if (err_key != KEY_NONE) {
    if (lane == 0) key_min(fstate, f, err_key);
    return;
  }
  X.final_flush();
  if (lane == 0) {
    S->out_len = X.pos;
    S->rep[0] = (uint64_t)rep[0];
    S->rep[1] = (uint64_t)rep[1];
    S->rep[2] = (uint64_t)rep[2];
  }
}

// ---------------------------------------------------------------------------
// compaction (frames without an exact FCS layout)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void zd_k_compact(const uint8_t* __restrict__ staging, uint8_t* dst,
                                                    const uint64_t* from, const uint64_t* to, const uint64_t* len) {
  const uint32_t f = blockIdx.x;
  const uint8_t* s = staging + from[f];
  uint8_t* d = dst + to[f];
  const uint64_t n = len[f];
  for (uint64_t x = threadIdx.x; x < n; x += blockDim.x) d[x] = s[x];
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
  auto* fses = (uint32_t*)(ws + W.fses);
  auto* sll = (uint32_t*)(ws + W.seq_ll);
  auto* sof = (uint32_t*)(ws + W.seq_of);
  auto* sml = (uint32_t*)(ws + W.seq_ml);
  hipStream_t s = a.stream;
  hipError_t e;
  if (a.events) if ((e = hipEventRecord(a.events[0], s)) != hipSuccess) return e;
  if (a.n_tables)
    hipLaunchKernelGGL(zd_k_tables, dim3(a.n_tables), dim3(64), 0, s, a.src, a.src_size, comp, cstate, fstate,
                       (const uint32_t*)(ws + W.list_tables), luts, fses);
  if (a.events) if ((e = hipEventRecord(a.events[1], s)) != hipSuccess) return e;
  if (a.n_huf)
    hipLaunchKernelGGL(zd_k_huffman, dim3(a.n_huf), dim3(64), 0, s, a.src, a.src_size, comp, cstate, fstate,
                       (const uint32_t*)(ws + W.list_huf), (const uint16_t*)luts, ws + W.lits);
  if (a.events) if ((e = hipEventRecord(a.events[2], s)) != hipSuccess) return e;
  if (a.n_seq)
    hipLaunchKernelGGL(zd_k_sequences, dim3(a.n_seq), dim3(64), 0, s, a.src, a.src_size, comp, cstate, fstate,
                       (const uint32_t*)(ws + W.list_seq), (const uint32_t*)fses, sll, sof, sml);
  if (a.events) if ((e = hipEventRecord(a.events[3], s)) != hipSuccess) return e;
  if (a.n_frames)
    hipLaunchKernelGGL(zd_k_execute, dim3(a.n_frames), dim3(64), 0, s, a.src, a.out, frames, fstate, blocks, comp,
                       (const CompState*)cstate, (const uint8_t*)(ws + W.lits), (const uint32_t*)sll,
                       (const uint32_t*)sof, (const uint32_t*)sml);
  if (a.events) if ((e = hipEventRecord(a.events[4], s)) != hipSuccess) return e;
  return hipGetLastError();
}

hipError_t launch_compact(const uint8_t* staging, uint8_t* dst, const uint64_t* d_from, const uint64_t* d_to,
                          const uint64_t* d_len, uint32_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(zd_k_compact, dim3(n), dim3(256), 0, s, staging, dst, d_from, d_to, d_len);
  return hipGetLastError();
}

}  // namespace zd
