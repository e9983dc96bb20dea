// zd_walk.h — the frame / block header walk (FrameIterator, Frame::parse,
// Header::parse, Block::parse and the fixed-size parts of
// LiteralsSection::parse and Sequences::parse), shared by the host planner
// (zd_host.cpp: index_frames, one thread per byte range) and the device walk
// (zd_kernels.hip: zd_k_walk, one wave per byte range, for inputs that are
// resident in HBM).  One source for both, so the two walks agree byte for
// byte by construction; tests/test_gpu_walk.py checks the plans they give.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/zd.h"
#include "zd_common.h"

namespace zd {

constexpr uint32_t MAGIC_ZSTD = 0xFD2FB528u;   // frame.rs:41
constexpr uint32_t MAGIC_SKIP = 0x184D2A50u;   // frame.rs:42

struct WalkErr {
  int code = 0;
  uint32_t stage = PS_STRUCT;
};

// ForwardByteParser (parsing.rs:9-112)
struct Bytes {
  const uint8_t* p;
  size_t n;
  ZD_HD int u8(uint8_t* v) {
    if (!n) return ZD_E_NOT_ENOUGH_BYTES;
    *v = *p++; n--; return 0;
  }
  ZD_HD int slice(size_t len, const uint8_t** s) {
    if (len == 0) return ZD_E_EMPTY_SLICE;
    if (n < len) return ZD_E_NOT_ENOUGH_BYTES;
    *s = p; p += len; n -= len; return 0;
  }
  ZD_HD int le(size_t k, uint64_t* v) {
    if (n < k) return ZD_E_NOT_ENOUGH_BYTES;
    uint64_t r = 0;
    for (size_t i = 0; i < k; i++) r |= (uint64_t)p[i] << (8 * i);
    p += k; n -= k; *v = r; return 0;
  }
};

struct HostBlock {
  uint64_t src;          // absolute offset of the block content
  uint32_t size;
  uint8_t type, last, rle;
  // compressed only
  CompBlock cb;
};

// A frame; its blocks are blocks[b0, b0 + nb) of the part that holds it.
struct HostFrame {
  zd_frame_desc d;
  uint32_t b0 = 0, nb = 0;
  uint32_t ncomp = 0;         // compressed blocks
  uint64_t key = KEY_NONE;    // walk-detected parse error (frame stops here)
  int status = 0;
};

ZD_HD inline void zero_bytes(void* p, size_t n) {
  uint8_t* b = (uint8_t*)p;
  for (size_t i = 0; i < n; i++) b[i] = 0;
}

// Literals section header + the walk-visible parts of the section
// (literals.rs:88-206) and of the sequences header (sequences.rs:52-87 and
// the mode byte of 91-143).  The block content is base[off, off + size).
ZD_HD inline int parse_compressed(const uint8_t* base, uint64_t off, uint32_t size, CompBlock* cb, WalkErr* e) {
  Bytes np{base + off, size};
  const uint8_t* start = np.p;
  auto rel = [&]() { return (uint32_t)(np.p - start); };
  e->stage = PS_STRUCT;
  uint8_t h;
  if (int r = np.u8(&h)) return e->code = r;
  int lt = h & 3, sf = (h >> 2) & 3;
  uint32_t regen = 0, csize = 0;
  int nstreams = 1;
  if (lt == LIT_RAW || lt == LIT_RLE) {
    uint8_t b1, b2;
    if (sf == 0 || sf == 2) regen = h >> 3;
    else if (sf == 1) { if (int r = np.u8(&b1)) return e->code = r; regen = (h >> 4) + ((uint32_t)b1 << 4); }
    else {
      if (int r = np.u8(&b1)) return e->code = r;
      if (int r = np.u8(&b2)) return e->code = r;
      regen = (h >> 4) + ((uint32_t)b1 << 4) + ((uint32_t)b2 << 12);
    }
  } else {
    const uint8_t* s;
    uint32_t nb = sf <= 1 ? 2 : (uint32_t)sf + 1;
    if (int r = np.slice(nb, &s)) return e->code = r;
    uint32_t x = 0;
    for (uint32_t i = 0; i < nb; i++) x |= (uint32_t)s[i] << (8 * i);
    if (sf <= 1) { regen = (h >> 4) + ((x & 0x3F) << 4); csize = x >> 6; nstreams = sf == 0 ? 1 : 4; }
    else if (sf == 2) { regen = (h >> 4) + ((x & 0x3FF) << 4); csize = (x >> 10) & 0x3FFF; nstreams = 4; }
    else { regen = (h >> 4) + ((x & 0x3FFF) << 4); csize = (x >> 14) & 0x3FFFF; nstreams = 4; }
  }
  cb->lit_type = (uint8_t)lt;
  cb->lit_regen = regen;
  cb->nstreams = 0;
  if (lt == LIT_RAW) {
    const uint8_t* s;
    cb->lit_data = rel();
    if (int r = np.slice(regen, &s)) return e->code = r;
  } else if (lt == LIT_RLE) {
    if (int r = np.u8(&cb->lit_rle)) return e->code = r;
  } else {
    const uint8_t* cs;
    if (int r = np.slice(csize, &cs)) return e->code = r;
    Bytes ni{cs, csize};
    if (lt == LIT_COMPRESSED) {      // HuffmanDecoder::parse header + description slice (huffman.rs:80-130)
      e->stage = PS_HUF_DESC;
      cb->lit_data = (uint32_t)(cs - start);
      uint8_t hh;
      if (int r = ni.u8(&hh)) return e->code = r;
      size_t dl = hh < 128 ? hh : ((size_t)(hh - 127) / 2 + (hh - 127) % 2);
      const uint8_t* d;
      if (int r = ni.slice(dl, &d)) return e->code = r;
      cb->huf_desc_size = (uint32_t)(1 + dl);
    }
    e->stage = PS_JUMP;
    size_t total = ni.n;
    uint32_t ss[4] = {0, 0, 0, 0};
    if (nstreams == 4) {
      uint64_t s1, s2, s3;
      if (int r = ni.le(2, &s1)) return e->code = r;
      if (int r = ni.le(2, &s2)) return e->code = r;
      if (int r = ni.le(2, &s3)) return e->code = r;
      if (s1 + s2 + s3 > total - 6) return e->code = ZD_E_CORRUPTED_STREAMS_SIZE;
      size_t s4 = total - 6 - s1 - s2 - s3;
      ss[0] = (uint32_t)s1; ss[1] = (uint32_t)s2; ss[2] = (uint32_t)s3; ss[3] = (uint16_t)s4;
    } else {
      ss[0] = (uint16_t)ni.n;
    }
    cb->streams = (uint32_t)(ni.p - start);
    const uint8_t* d;
    if (int r = ni.slice(ni.n, &d)) return e->code = r;
    // literals.rs:70-73: the stream loop stops at the first empty stream
    for (int k = 0; k < 4; k++) {
      if (ss[k] == 0) break;
      cb->stream_size[k] = ss[k];
      cb->nstreams = (uint8_t)(k + 1);
    }
  }
  // Sequences::parse (sequences.rs:52-75)
  e->stage = PS_SEQ_HDR;
  uint8_t b0;
  if (int r = np.u8(&b0)) return e->code = r;
  uint32_t nseq;
  if (b0 == 0) nseq = 0;
  else if (b0 < 128) nseq = b0;
  else if (b0 < 255) { uint8_t b1; if (int r = np.u8(&b1)) return e->code = r; nseq = ((uint32_t)(b0 - 128) << 8) + b1; }
  else {
    uint8_t b1, b2;
    if (int r = np.u8(&b1)) return e->code = r;
    if (int r = np.u8(&b2)) return e->code = r;
    nseq = (uint32_t)b1 + ((uint32_t)b2 << 8) + 0x7F;     // D1 (sequences.rs:84)
  }
  cb->nseq = nseq;
  cb->modes[0] = cb->modes[1] = cb->modes[2] = M_REPEAT;
  if (nseq) {
    const uint8_t* mb;
    if (int r = np.slice(1, &mb)) return e->code = r;
    if (mb[0] & 3) return e->code = ZD_E_SEQ_RESERVED_SET;
    cb->modes[0] = (mb[0] >> 6) & 3;
    cb->modes[1] = (mb[0] >> 4) & 3;
    cb->modes[2] = (mb[0] >> 2) & 3;
  }
  cb->seq_tables = rel();
  return 0;
}

// Header::parse (frame.rs:111-177)
ZD_HD inline int parse_header(Bytes& in, zd_frame_desc* f) {
  const uint8_t* b;
  if (int r = in.slice(1, &b)) return r;
  unsigned fhd = b[0];
  unsigned dict_flag = fhd & 3, csum = (fhd >> 2) & 1, reserved = (fhd >> 3) & 1;
  unsigned single = (fhd >> 5) & 1, fcs_flag = fhd >> 6;
  if (reserved) return ZD_E_FRAME_RESERVED_SET;
  int fcs_size = (fcs_flag == 0) ? (single ? 1 : -1) : (1 << fcs_flag);
  uint64_t window = 0;
  if (!single) {
    uint8_t wd;
    if (int r = in.u8(&wd)) return r;
    uint64_t base = 1ull << ((wd >> 3) + 10);
    window = base + (base / 8) * (wd & 7);
  }
  f->dict_id = UINT64_MAX;
  if (dict_flag) {
    const uint8_t* a;
    size_t dl = (size_t)1 << (dict_flag - 1);
    if (int r = in.slice(dl, &a)) return r;
    uint64_t v = 0;
    for (size_t i = 0; i < dl; i++) v |= (uint64_t)a[i] << (8 * i);
    f->dict_id = v;
  }
  f->content_size = UINT64_MAX;
  if (fcs_size > 0) {
    const uint8_t* a;
    if (int r = in.slice((size_t)fcs_size, &a)) return r;
    uint64_t v = 0;
    for (int i = 0; i < fcs_size; i++) v |= (uint64_t)a[i] << (8 * i);
    if (fcs_size == 2) v += 256;
    f->content_size = v;
  }
  f->window_size = single ? f->content_size : window;
  f->has_checksum = csum;
  return 0;
}

// Walks one frame at in, handing its blocks to the sink (S.size(): blocks
// so far; S.push(block)).  On error, hf->key/status hold the failure; the
// blocks parsed before (and the failing one, with its host_stage) are kept.
template <typename SINK>
ZD_HD inline int index_frame(const uint8_t* base, Bytes& in, HostFrame* hf, SINK& S) {
  zd_frame_desc& f = hf->d;
  zero_bytes(&f, sizeof f);
  f.src_offset = (uint64_t)(in.p - base);
  f.content_size = UINT64_MAX;
  f.dict_id = UINT64_MAX;
  hf->b0 = (uint32_t)S.size();
  hf->nb = 0;
  hf->ncomp = 0;
  hf->key = KEY_NONE;
  hf->status = 0;
  auto push = [&](const HostBlock& hb) {
    S.push(hb);
    hf->nb++;
    hf->ncomp += hb.type == 2;
  };
  auto fail = [&](int code, uint32_t blk, uint32_t stage) {
    hf->status = code;
    hf->key = make_key(PH_PARSE, blk, stage, 0, code);
    f.src_size = (uint64_t)(in.p - base) - f.src_offset;
    return code;
  };
  uint64_t magic;
  if (int r = in.le(4, &magic)) return fail(r, 0, PS_STRUCT);
  f.magic = (uint32_t)magic;
  if (f.magic == MAGIC_ZSTD) {
    f.kind = ZD_FRAME_ZSTD;
    if (int r = parse_header(in, &f)) return fail(r, 0, PS_STRUCT);
    if (f.window_size > MAX_WIN_SIZE) return fail(ZD_E_WINDOW_SIZE_TOO_BIG, 0, PS_STRUCT);
    for (uint32_t bi = 0;; bi++) {
      const uint8_t* h;
      if (int r = in.slice(3, &h)) return fail(r, bi, PS_STRUCT);
      uint32_t x = h[0] | (h[1] << 8) | ((uint32_t)h[2] << 16);
      HostBlock hb;
      zero_bytes(&hb, sizeof hb);
      hb.last = x & 1;
      hb.type = (x >> 1) & 3;
      hb.size = x >> 3;
      hb.src = (uint64_t)(in.p - base);
#ifndef __HIP_DEVICE_COMPILE__
      // the next block (or frame) header: a cache miss that now overlaps
      // this block's own header parse
      if (hb.type != 1 && hb.size < in.n) __builtin_prefetch(in.p + hb.size);
#endif
      if (hb.type == 0) {
        const uint8_t* s;
        if (int r = in.slice(hb.size, &s)) return fail(r, bi, PS_STRUCT);
      } else if (hb.type == 1) {
        if (int r = in.u8(&hb.rle)) return fail(r, bi, PS_STRUCT);
      } else if (hb.type == 2) {
        const uint8_t* s;
        if (int r = in.slice(hb.size, &s)) return fail(r, bi, PS_STRUCT);
        CompBlock& cb = hb.cb;
        cb.src = hb.src;
        cb.size = hb.size;
        cb.block_in_frame = bi;
        cb.host_stage = PS_ALL;
        WalkErr e;
        int r = parse_compressed(base, hb.src, hb.size, &cb, &e);
        if (r) {
          cb.host_stage = (uint8_t)e.stage;
          push(hb);
          return fail(r, bi, e.stage);
        }
      } else {
        return fail(ZD_E_RESERVED_BLOCK_TYPE, bi, PS_STRUCT);
      }
      push(hb);
      if (hb.last) break;
    }
    if (f.has_checksum) {
      uint64_t cs;
      if (in.le(4, &cs)) return fail(ZD_E_MISSING_CHECKSUM, hf->nb, PS_STRUCT);
      f.checksum = (uint32_t)cs;
    }
  } else if ((f.magic ^ MAGIC_SKIP) <= 0x0F) {
    f.kind = ZD_FRAME_SKIPPABLE;
    uint64_t len;
    if (int r = in.le(4, &len)) return fail(r, 0, PS_STRUCT);
    const uint8_t* s;
    HostBlock hb;
    zero_bytes(&hb, sizeof hb);
    hb.src = (uint64_t)(in.p - base);
    if (int r = in.slice((size_t)len, &s)) return fail(r, 0, PS_STRUCT);
    hb.type = 4;
    hb.size = (uint32_t)len;
    hb.last = 1;
    push(hb);
  } else {
    return fail(ZD_E_UNRECOGNIZED_MAGIC, 0, PS_STRUCT);
  }
  f.src_size = (uint64_t)(in.p - base) - f.src_offset;
  return 0;
}

ZD_HD inline bool magic_word(uint32_t m) { return m == MAGIC_ZSTD || (m ^ MAGIC_SKIP) <= 0x0F; }

// The device walk's per-range summary (zd_k_walk, count pass): where the
// range's chain starts and ends, its status and sizes; the fill pass writes
// the range's frames and blocks at f_off / b_off.
struct WalkRange {
  uint64_t p0;          // first frame start of the chain (a magic number in the range), or the range end
  uint64_t end;         // where the chain stopped (first frame start >= range end, or past a failing frame)
  uint64_t f_off, b_off;
  uint32_t nframes, nblocks;
  int32_t status;
  uint32_t pad;
};

}  // namespace zd
