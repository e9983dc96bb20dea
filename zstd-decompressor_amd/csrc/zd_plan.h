// zd_plan.h — the per-frame descriptor pass of the planner, shared by the
// host planner (zd_host.cpp build_plan, per part on the worker threads) and the
// device planner (zd_kernels.hip zd_k_plan_count / zd_k_plan_fill, one lane per
// frame, zd_plan_create_device): one source, so the two plans cannot drift.
#pragma once
#include <stdint.h>

#include "../../include/zd.h"
#include "zd_common.h"
#include "zd_walk.h"

namespace zd {

constexpr uint32_t K4F_CAP_BYTES = 128u << 10;   // frames up to this output size execute in LDS (K4F)

template <typename T>
ZD_HD inline T plan_min(T a, T b) { return a < b ? a : b; }
ZD_HD inline uint64_t plan_align(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// K4J (block-parallel execute, pointer jumping) takes the frames of at least
// K4J_MIN_BLOCKS compressed blocks: the streaming K4 runs a frame's blocks one
// after another on one wave, which a frame of many blocks cannot hide behind
// other frames unless the plan holds thousands of them
// (K4J_MAX_FRAMES).  ZD_K4J=1 / 0 forces it on (every frame with a
// compressed block) / off.
constexpr uint32_t K4J_MIN_BLOCKS = 16;
constexpr uint64_t K4J_MAX_FRAMES = 1024;
// A plan of few frames leaves the GPU nearly idle with one wave per frame on
// the streaming K4 (the reference's moby-dick sample: one frame of 10 blocks,
// 159k sequences on one wave): there K4J takes every frame of 2 or more
// compressed blocks.
constexpr uint64_t K4J_FEW_FRAMES = 64;
constexpr uint32_t K4J_MIN_BLOCKS_FEW = 2;

// Running indices of build_plan: every array it fills grows frame by frame,
// so a frame's entries start at the counts of the frames before it.
// (all u64, so that the device build scans them as PLAN_FIELDS words)
struct PlanCounts {
  uint64_t frames = 0, blocks = 0, comps = 0, luts = 0, fses = 0, lits = 0, nrec = 0, nseq = 0, out = 0;
  uint64_t tables = 0, huf = 0, seq = 0, k4f = 0, copies = 0;
  uint64_t jframes = 0, jblk = 0, jseg = 0;
  uint64_t inexact = 0;          // frames whose capacity is an upper bound (no usable FCS)
  uint64_t jwords = 0;           // K4J state words: a frame's region starts a 16-word piece, 16 words of slack after
  uint64_t jpieces = 0;          // K4J 16-byte pieces over the frames' regions
  uint64_t k0only = 0;           // frames K0 copies whole (every block raw / RLE): no K4 for them
  ZD_HD bool exact() const { return inexact == 0; }
  ZD_HD void add(const PlanCounts& o) {
    frames += o.frames; blocks += o.blocks; comps += o.comps; luts += o.luts; fses += o.fses; lits += o.lits;
    nrec += o.nrec; nseq += o.nseq; out += o.out; tables += o.tables; huf += o.huf; seq += o.seq; k4f += o.k4f;
    copies += o.copies; jframes += o.jframes; jblk += o.jblk; jseg += o.jseg; inexact += o.inexact;
    jwords += o.jwords; jpieces += o.jpieces; k0only += o.k0only;
  }
};
constexpr int PLAN_FIELDS = 21;
static_assert(sizeof(PlanCounts) == PLAN_FIELDS * 8, "PlanCounts: u64 fields only");

// Plan-wide inputs of the per-frame pass.  `prev_*` seed the Treeless/Repeat
// resolution (context API), -1 when absent.
struct PlanCtx {
  int32_t prev_huf;
  int32_t prev_tab[3];
  uint64_t out_len0, fixed_cap, cap0;
  const HostFrame* cap0_frame;   // the plan's first frame (cap0 applies to it)
  uint64_t rep0[3];
  uint32_t flags;
  bool k4f_on, k4j_auto;
  bool fused;              // zd_k_fused plan: no K4F, 128-byte aligned literal and record slots
  int k4j_mode;
  uint32_t k4j_min;        // compressed blocks a frame needs for K4J (automatic mode)
};

// Where the filling pass writes: the plan's host vectors (small plans, the
// context API) or the pinned upload staging at the workspace offsets.
struct Sink {
  CompBlock* comps;
  BlockRec* blocks;
  FrameDesc* fdesc;
  FrameState* fstate0;
  uint32_t *list_tables, *list_huf, *list_seq, *list_k4f;
  CopyDesc* copies;
  JFrame* jframes;
  JBlkDesc* jblkd;
  JSegDesc* jsegd;
  uint64_t *frame_out, *frame_cap;
};

// One frame's descriptors at the running indices c (build_plan).  FILL: the
// entries are written to S; otherwise c only advances (the counting pass).
// A K4J frame's descriptors (JFrame, its JBlkDesc and JSegDesc entries) are
// written here too, at the running K4J indices, so the host and the device
// build them alike; jm->note(n) gets each K4J frame's sequence count (the
// plan's pointer-jumping rounds follow the largest).
template <bool FILL, typename JOUT>
ZD_HD void plan_frame(const PlanCtx& X, const HostFrame& hf, const HostBlock* hblocks, PlanCounts& c, const Sink& S,
                      JOUT* jm) {
  const uint32_t fi = (uint32_t)c.frames;
  FrameDesc fd{};
  FrameState fs{};
  fs.key = hf.key;
  fs.rep[0] = X.rep0[0]; fs.rep[1] = X.rep0[1]; fs.rep[2] = X.rep0[2];
  fd.first_block = (uint32_t)c.blocks;
  fd.out_len0 = X.out_len0;
  int32_t huf_prev = X.prev_huf;
  int32_t tab_prev[3] = {X.prev_tab[0], X.prev_tab[1], X.prev_tab[2]};
  uint64_t bound = 0;
  bool seqs_in_frame = false;
  const bool frame_failed_host = hf.key != KEY_NONE;
  uint64_t jseg = 0;
  // a re-plan of a frame that overran (zd_plan_decompress): by identity, the
  // counting pass numbers each part's frames from 0
  const bool replanned = X.cap0 && &hf == X.cap0_frame && hf.d.kind == ZD_FRAME_ZSTD;
  for (uint32_t bi = 0; bi < hf.nb; bi++) {
    const HostBlock& hb = hblocks[hf.b0 + bi];
    BlockRec br{};
    br.src = hb.src; br.size = hb.size; br.type = hb.type; br.last = hb.last; br.rle = hb.rle; br.comp = -1;
    if (hb.type == 2) {
      CompBlock cb = hb.cb;
      cb.frame = fi;
      cb.block_in_frame = bi;
      cb.prebuilt = 0;
      cb.huf_src = -1;
      cb.tab_src[0] = cb.tab_src[1] = cb.tab_src[2] = -1;
      const uint32_t ci = (uint32_t)c.comps;
      const bool failing = cb.host_stage != PS_ALL;
      // literals: Treeless resolution (literals.rs:59-66)
      if (!failing && (cb.lit_type == LIT_COMPRESSED || cb.lit_type == LIT_TREELESS)) {
        if (cb.lit_type == LIT_COMPRESSED) { cb.huf_src = (int32_t)ci; huf_prev = (int32_t)ci; }
        else cb.huf_src = huf_prev;
        if (cb.huf_src < 0)
          fs.key = plan_min(fs.key, make_key(PH_DECODE, bi, DS_LITERALS, 0, ZD_E_HUFFMAN_DECODER_MISSING));
      }
      if (cb.lit_type == LIT_COMPRESSED && cb.host_stage > PS_HUF_DESC) cb.lut_slot = (uint32_t)c.luts++;
      // sequences: Repeat resolution (sequences.rs:147-187, 232-234)
      if (!failing) {
        if (cb.nseq == 0) {
          int code = ZD_E_EMPTY_INPUT_DATA;
          for (int k = 0; k < 3; k++) if (tab_prev[k] < 0) { code = ZD_E_NO_PREVIOUS_DECODER; break; }
          fs.key = plan_min(fs.key, make_key(PH_DECODE, bi, DS_SEQUENCES, 0, code));
        } else {
          cb.fse_slot = (uint32_t)c.fses++;
          bool miss = false;
          for (int k = 0; k < 3; k++) {
            if (cb.modes[k] == M_REPEAT) {
              if (tab_prev[k] < 0) { miss = true; break; }
              cb.tab_src[k] = tab_prev[k];
            } else {
              cb.tab_src[k] = (int32_t)ci;
            }
          }
          if (miss) fs.key = plan_min(fs.key, make_key(PH_DECODE, bi, DS_SEQUENCES, 0, ZD_E_NO_PREVIOUS_DECODER));
          else for (int k = 0; k < 3; k++) tab_prev[k] = cb.tab_src[k];
        }
      } else if (cb.nseq) {
        cb.fse_slot = (uint32_t)c.fses++;
      }
      // workspace
      if (cb.lit_type == LIT_COMPRESSED || cb.lit_type == LIT_TREELESS) {
        cb.lit_extra = 0;
        if (replanned) {             // a symbol is at least one bit: <= 8 literals per stream byte
          uint64_t most = 0;
          for (int k = 0; k < cb.nstreams; k++) most += 8ull * cb.stream_size[k];
          if (most > cb.lit_regen) cb.lit_extra = (uint32_t)(most - cb.lit_regen);
        }
        cb.lit_out = c.lits;
        c.lits += plan_align((uint64_t)cb.lit_regen + 32 + cb.lit_extra, X.fused ? 128 : 16);   // + K2's 16-byte slack
      }
      if (X.fused) c.nrec = plan_align(c.nrec, 16);   // a block's records start a 128-byte line
      cb.seq_out = c.nrec;
      c.nseq += cb.nseq;
      c.nrec += rec_slots(cb.nseq);              // record pairs, a spare pair past the block's last
      seqs_in_frame |= cb.nseq > 0;
      br.comp = (int32_t)ci;
      jseg += cb.nseq > J_SEG ? (cb.nseq + J_SEG - 1) / J_SEG : 1;
      const bool needs_tables = (cb.lit_type == LIT_COMPRESSED && cb.host_stage > PS_HUF_DESC) ||
                                (cb.nseq > 0 && cb.host_stage > PS_SEQ_TABLES);
      if (needs_tables) { if (FILL) S.list_tables[c.tables] = ci; c.tables++; }
      if (!frame_failed_host) {
        if ((cb.lit_type == LIT_COMPRESSED || cb.lit_type == LIT_TREELESS) && cb.nstreams && cb.huf_src >= 0) {
          if (FILL) S.list_huf[c.huf] = ci;
          c.huf++;
        }
        if (cb.nseq > 0 && cb.tab_src[0] >= 0 && cb.tab_src[1] >= 0 && cb.tab_src[2] >= 0) {
          if (FILL) S.list_seq[c.seq] = ci;
          c.seq++;
        }
      }
      if (FILL) S.comps[ci] = cb;
      c.comps++;
      bound += MAX_BLOCK_OUT;
    } else {
      bound += hb.size;
      jseg += 1;
    }
    if (FILL) S.blocks[c.blocks] = br;
    c.blocks++;
  }
  if (X.fused) c.nrec = plan_align(c.nrec, 16);   // (the next frame's records start a line: per-frame counts scan)
  fd.nblocks = hf.nb;
  uint64_t cap;
  if (hf.d.kind == ZD_FRAME_SKIPPABLE) {
    // a truncated skippable frame fails to index and keeps no payload block
    cap = ((X.flags & ZD_F_SKIPPABLE) && hf.nb) ? hblocks[hf.b0].size : 0;
    if (!(X.flags & ZD_F_SKIPPABLE)) fd.nblocks = 0;
  } else if (hf.d.content_size != UINT64_MAX && hf.d.content_size <= bound) {
    cap = hf.d.content_size;
  } else {
    cap = bound;
    c.inexact = 1;
  }
  if (frame_failed_host) fd.nblocks = 0;
  if (X.fixed_cap) cap = X.fixed_cap;
  if (replanned) {
    cap = X.cap0;
    c.inexact = 1;
  }
  fd.out = c.out;
  fd.out_cap = cap;
  // K4J: frames of many compressed blocks, and any frame past the streaming
  // K4's int32 positions (distances, zd_common.h)
  const bool to_j = X.out_len0 == 0 && !frame_failed_host && fd.nblocks && hf.ncomp && hf.d.kind == ZD_FRAME_ZSTD &&
                    cap <= K4J_MAX_FRAME_OUT &&
                    (X.k4j_mode >= 0 ? X.k4j_mode == 1
                                     : ((X.k4j_auto && hf.ncomp >= X.k4j_min) || cap > K4_MAX_FRAME_OUT));
  // larger frames with sequences that K4J does not take (forced off, or past
  // its 32 GiB) are outside the GPU path's domain
  if (!to_j && cap > K4_MAX_FRAME_OUT && seqs_in_frame)
    fs.key = plan_min(fs.key, make_key(PH_LIMIT, 0, 0, 0, ZD_E_OUT_OF_DOMAIN));
  if (to_j) {
    fd.lds = 2;
    uint64_t nseq = 0;
    uint32_t njs = (uint32_t)c.jseg;
    for (uint32_t k = 0; k < fd.nblocks; k++) {
      const HostBlock& hb = hblocks[hf.b0 + k];
      const uint32_t bn = hb.type == 2 ? hb.cb.nseq : 0u;
      nseq += bn;
      if (FILL) {
        JBlkDesc d{};
        d.block = fd.first_block + k;
        d.jframe = (uint32_t)c.jframes;
        d.j = k;
        d.seg0 = njs;
        for (uint32_t g = 0; g == 0 || g * J_SEG < bn; g++) S.jsegd[njs++] = JSegDesc{(uint32_t)c.jblk + k, g};
        S.jblkd[c.jblk + k] = d;
      }
    }
    if (FILL) {
      JFrame jf{};
      jf.base = c.jwords;                      // word index: frame pieces of 16 words are 64-byte lines
      jf.cap = cap;
      jf.piece0 = c.jpieces;
      jf.frame = fi;
      jf.jb0 = (uint32_t)c.jblk;
      jf.njb = fd.nblocks;
      S.jframes[c.jframes] = jf;
    }
    if (jm) jm->note(nseq);
    c.jframes++;
    c.jblk += fd.nblocks;
    c.jseg += jseg;
    c.jwords += plan_align(cap + 16, 16);
    c.jpieces += (cap + 15) / 16;
  } else {
    // K4F (whole frame resident in LDS, one 1024-thread workgroup per frame)
    // executes the frames that fit it in plans of 256-768 frames, where the
    // streaming K4 runs one round at its batch latency (C3: 0.64 vs 0.75 ms);
    // it is slower on C4 (EXPERIMENTS.md).  ZD_K4F=1 / 0 forces it on / off.
    fd.lds = (X.k4f_on && X.out_len0 == 0 && cap <= K4F_CAP_BYTES) ? 1u : 0u;
  }
  if (fd.lds == 1) { if (FILL) S.list_k4f[c.k4f] = fi; c.k4f++; }
  // Leading raw / RLE blocks (skippable payloads too) have output offsets
  // known here: K0 copies them in parallel pieces, the streaming K4 starts
  // after them (a frame of raw/RLE blocks only never reaches K4's loop).
  if (!fd.lds && fd.nblocks && cap < 0x7FF00000ull) {
    uint64_t pre = 0;
    uint32_t k = 0;
    for (; k < fd.nblocks; k++) {
      const HostBlock& hb = hblocks[hf.b0 + k];
      if (hb.type != 0 && hb.type != 1 && hb.type != 4) break;
      if (X.out_len0 + pre + hb.size > cap) break;
      for (uint64_t x = 0; x < hb.size; x += COPY_PIECE) {
        if (FILL) {
          CopyDesc cd{};
          cd.src = hb.src + (hb.type == 1 ? 0 : x);
          cd.dst = c.out + X.out_len0 + pre + x;
          cd.size = (uint32_t)plan_min<uint64_t>(COPY_PIECE, hb.size - x);
          cd.fill = hb.type == 1 ? (0x100u | hb.rle) : 0u;
          S.copies[c.copies] = cd;
        }
        c.copies++;
      }
      pre += hb.size;
    }
    fd.skip = k;
    fd.skip_bytes = pre;
    // every block copied by K0: the frame's length is known here, and no
    // executor runs it (a launch less when no frame needs the streaming K4)
    if (k == fd.nblocks && fs.key == KEY_NONE) {
      fd.lds = 3;
      fs.out_len = X.out_len0 + pre;
      c.k0only++;
    }
  }
  if (FILL) {
    S.frame_out[fi] = c.out;
    S.frame_cap[fi] = cap;
    S.fdesc[fi] = fd;
    S.fstate0[fi] = fs;
  }
  c.out += cap;
  c.frames++;
}


}  // namespace zd
