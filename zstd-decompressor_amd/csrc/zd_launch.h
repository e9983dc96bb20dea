// zd_launch.h — host-side entry points of the gfx950 kernels (zd_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zd_common.h"
#include "zd_plan.h"

namespace zd {

struct LaunchArgs {
  const uint8_t* src;      // d_src
  uint64_t src_size;
  uint8_t* out;            // output base (d_dst or the plan's staging buffer)
  uint8_t* ws;             // workspace base
  Workspace W;
  uint32_t n_tables, n_huf, n_seq, n_frames, n_k4f, n_copies;
  hipStream_t stream;
  hipEvent_t* events;      // optional: N_KERNELS + 1 events recorded around the kernels
  hipStream_t aux = nullptr;   // optional second stream: K2 beside K3
  hipEvent_t fork = nullptr, join = nullptr;
  uint32_t n_jframes = 0, n_jblk = 0, n_jseg = 0;   // K4J frames / their blocks / scatter segments
  uint32_t n_k0only = 0;                   // frames K0 copies whole (FrameDesc::lds 3)
  uint32_t j_rounds = 0;                   // K4J pointer-jumping rounds launched
  uint64_t j_pieces = 0;                   // 16-byte pieces over the K4J frames' regions
  bool k3_lat = false;     // K3 as one block per wave (zd_k_sequences_l), few-block plans
  bool k3_quad = true;     // K3 as four lanes per block (zd_k_sequences_q); false: one lane per block
  uint32_t j_hops = 6;                     // K4J: hops per pending word and round (ZD_J_HOPS)
  uint32_t j_hops2 = 12;                   // K4J: the same in the sweeps after round 1 (ZD_J_HOPS2)
  uint32_t cus = 256;                      // compute units of the device (K4J rounds' grid)
  bool fused = false;                      // K3 + K4 as zd_k_fused, then the redo pass
  bool k1_seq_waves = false;               // K1's sequence half one wave per block (zd_k_tables_seqw)
  bool k1_fork = false;                    // no K2 | K3 fork: K1's halves on the two streams (aux, fork, join)
  // optional (zd_plan_set_profiling mode 2): an event pair recorded on
  // `stream` around each launch group that can carry a plan's work -- K0,
  // zd_k_fused, K4, K4F, the K4J kernels (kDomNames) -- with the fork and
  // fusion kept; bit g of *dom_used is set when group g launched
  hipEvent_t* dom_events = nullptr;
  uint32_t* dom_used = nullptr;
};

// K1 table parse/build -> K2 Huffman literals -> K3 FSE sequences -> K4 execute.
hipError_t launch_pipeline(const LaunchArgs& a);

// zd_decode_async's state reset (frame / block states, K1 and K4J counters, K4J done flags).
hipError_t launch_reset(uint8_t* ws, const Workspace& W, uint64_t n_frames, uint64_t n_comps, bool k4j,
                        uint64_t j_pieces, hipStream_t s);

// Copies frame outputs from staging (at cap offsets) to exact offsets.
hipError_t launch_compact(const uint8_t* staging, uint8_t* dst, const uint64_t* d_from,
                          const uint64_t* d_to, const uint64_t* d_len, uint32_t n, hipStream_t s);

// XXH64 of n byte ranges [base + off[i], + len[i]) -> hash[i] (device arrays)
hipError_t launch_xxh64(const uint8_t* base, const uint64_t* d_off, const uint64_t* d_len, uint32_t n,
                        uint64_t* d_hash, hipStream_t s);

// Device header walk (zd_walk.h): ranges [first + k chunk, + chunk) of src[0, n),
// count pass (fill = false: WalkRange summaries) or fill pass (frames/blocks at
// the summaries' f_off / b_off).
struct WalkRange;
struct HostFrame;
struct HostBlock;
hipError_t launch_walk(const uint8_t* src, uint64_t n, uint64_t first, uint64_t chunk, uint32_t nranges, WalkRange* wr,
                       HostFrame* frames, HostBlock* blocks, bool fill, hipStream_t s);

// Device descriptors (zd_plan_create_device): the shape pass (PlanShape
// zeroed first), the count pass + exclusive scan (cnt: nf x PLAN_FIELDS
// words, scanned within 256-frame tiles; tot: (tiles + 1) x PLAN_FIELDS
// words, the tiles' starts and then the plan's totals), the fill pass.
struct PlanShape { uint32_t multi, jcand; uint64_t jmaxseq; };
hipError_t launch_plan_shape(const HostFrame* frames, uint64_t nf, uint32_t k4j_min, PlanShape* out, hipStream_t s);
hipError_t launch_plan_count(const PlanCtx& X, const HostFrame* frames, const HostBlock* blocks, uint64_t nf,
                             uint64_t* cnt, uint64_t* tot, PlanShape* shape, hipStream_t s);
hipError_t launch_plan_fill(const PlanCtx& X, const HostFrame* frames, const HostBlock* blocks, uint64_t nf,
                            const uint64_t* cnt, const uint64_t* tot, const Sink& S, hipStream_t s);

constexpr int N_KERNELS = 6;
// mode-2 launch groups (LaunchArgs::dom_events: events 2g, 2g + 1)
constexpr int N_DOM = 5;
enum { DOM_K0 = 0, DOM_FUSED = 1, DOM_K4 = 2, DOM_K4F = 3, DOM_K4J = 4 };
extern const char* const kDomNames[N_DOM];
constexpr uint32_t K4F_CAP = K4F_CAP_BYTES;   // frames up to this output size execute in LDS (K4F)
extern const char* const kKernelNames[N_KERNELS];

}  // namespace zd
