// zd_host.cpp — host planner and C ABI (include/zd.h).
//
// The host does what the reference's parse phase does with headers only
// (FrameIterator / Frame::parse / Header::parse / Block::parse and the
// fixed-size parts of LiteralsSection::parse and Sequences::parse), resolves
// which block's Huffman/FSE tables every block uses (Treeless literals,
// Repeat_Mode) and carves the device workspace.  Everything that reads
// entropy-coded data — Huffman/FSE table descriptions, literal streams,
// sequence bitstreams, the LZ77 execute — runs in the HIP kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/zd.h"
#include "zd_common.h"
#include "zd_internal.h"
#include "zd_launch.h"
#include "zd_plan.h"
#include "zd_walk.h"

using namespace zd;

namespace {

// Frames indexed by one thread of the host walk: a contiguous run of the
// input's frames and their blocks, stored flat.
struct HostPart {
  std::vector<HostFrame> frames;
  std::vector<HostBlock> blocks;
};

// The host walk's block sink: a part's block vector
struct VecSink {
  std::vector<HostBlock>& v;
  size_t size() const { return v.size(); }
  void push(const HostBlock& b) { v.push_back(b); }
};

#define HIPCHK(x) do { hipError_t _e = (x); if (_e != hipSuccess) { \
  fprintf(stderr, "zd: %s failed: %s\n", #x, hipGetErrorString(_e)); return ZD_E_HIP; } } while (0)

}  // namespace

// ===========================================================================
// Plan
// ===========================================================================
struct zd_plan {
  uint32_t flags = 0;
  std::vector<HostPart> parts;          // the host walk's frames, in input order
  std::vector<size_t> part_f0;          // plan frame index of each part's first frame
  size_t nframes = 0;
  std::vector<CompBlock> comps;
  std::vector<BlockRec> blocks;
  std::vector<FrameDesc> fdesc;
  std::vector<FrameState> fstate0;
  std::vector<uint32_t> list_tables, list_huf, list_seq, list_k4f;
  std::vector<CopyDesc> copies;         // K0 pieces
  std::vector<JFrame> jframes;          // K4J frames, their blocks and the scatter's segments
  std::vector<JBlkDesc> jblkd;
  std::vector<JSegDesc> jsegd;
  uint64_t j_bytes = 0, j_pieces = 0;
  uint32_t j_rounds = 0;
  // counts of the descriptor arrays (large plans keep their descriptors only
  // in the pinned staging until the upload: the vectors above stay empty)
  uint64_t n_comps = 0, n_blocks = 0, n_frames = 0, n_tables = 0, n_huf = 0, n_seq = 0, n_k4f = 0, n_copies = 0;
  uint64_t n_jframes = 0, n_jblk = 0, n_jseg = 0, n_k0only = 0;
  bool fused = false;                           // zd_k_fused plan (build_plan fuse_plan)
  bool last_fused = false;                      // the last zd_decode_async launched zd_k_fused
  std::vector<uint64_t> frame_out, frame_cap;   // output offset and capacity per frame
  bool staged = false;
  std::unique_lock<std::mutex> stage_lock;      // the pinned staging, from build_plan to upload_plan
  zd_plan_info info{};
  Workspace W{};
  uint8_t* d_ws = nullptr;
  uint64_t ws_bytes = 0;                 // size of the d_ws allocation (>= W.total: a cached block)
  int dev = -1;                          // the device d_ws and the aux stream belong to (upload_plan)
  uint64_t desc_bytes = 0;               // the host-filled head of the workspace (one upload)
  uint8_t* d_staging = nullptr;          // the output of a non-exact layout, or the copy an exact one is compacted from
  uint64_t staging_bytes = 0;
  int index_status = 0;
  uint64_t cap0 = 0;                     // capacity of frame 0 instead of its own (a re-plan, zd_plan_decompress)
  // the first failing frame of the last zd_plan_results when its failure is
  // a limit of the GPU path the host can lift (LS_CAPACITY, LS_JROUNDS)
  int64_t limit_frame = -1;
  uint32_t limit_stage = 0;
  size_t index_stop = 0;                 // frame index that failed to index (== nframes - 1) or nframes
  // a plan whose descriptors the GPU built (zd_plan_create_device): its
  // frame index stays in the workspace (W.hframes) until a caller needs it
  bool dev_built = false;
  zd::FrameOuts io_fo;                   // per-frame outcome of the last zd_plan_decompress
  mutable std::vector<HostFrame> dev_frames;
  // the frame index on the host (a device-built plan's comes back once);
  // false when it cannot be read -- nothing is kept then, a later call retries
  bool frames_ready() const {
    if (!dev_built || dev_frames.size() == nframes) return true;
    std::vector<HostFrame> v(nframes);
    if (nframes && hipMemcpy(v.data(), d_ws + W.hframes, nframes * sizeof(HostFrame), hipMemcpyDeviceToHost) !=
                       hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    dev_frames = std::move(v);
    return true;
  }
  // (callers check frames_ready() first)
  const HostFrame& frame(size_t f) const {
    if (dev_built) return dev_frames[f];
    const size_t k = (size_t)(std::upper_bound(part_f0.begin(), part_f0.end(), f) - part_f0.begin()) - 1;
    return parts[k].frames[f - part_f0[k]];
  }
  void set_parts(std::vector<HostPart>&& p) {
    parts = std::move(p);
    part_f0.clear();
    nframes = 0;
    for (const HostPart& hp : parts) { part_f0.push_back(nframes); nframes += hp.frames.size(); }
  }
  bool profile = false;                  // mode 1: every kernel timed, one after another
  bool profile_dom = false;              // mode 2: the launch groups that carry work, timed in the pipeline as it runs
  uint32_t dom_used = 0;                 // the groups (kDomNames) the last mode-2 launch recorded
  hipEvent_t dom_ev[2 * N_DOM] = {};
  hipEvent_t ev[N_KERNELS + 1] = {};
  bool ev_made = false;
  bool launched = false;
  hipStream_t last_stream = nullptr;     // the stream of the last zd_decode_async
  // context API hook: comp 0 is a prebuilt "previous block" carrying tables
  bool has_prebuilt = false;
  // second stream for K2 beside K3 (created on first launch)
  hipStream_t aux = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  // output layout of the last zd_plan_results (frames before the first failure)
  std::vector<uint64_t> res_off, res_len;
  uint64_t* d_meta = nullptr;            // zd_plan_results' compaction / zd_plan_checksums' arrays
  uint64_t meta_cap = 0;                 // (u64 entries)
  // zd_plan_decompress (host in, host out): device buffers kept between calls
  uint8_t* io_src = nullptr;
  uint64_t io_src_cap = 0;
  uint8_t* io_dst = nullptr;
  uint64_t io_dst_cap = 0;
};

namespace {

uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// Executor routing (zd_route, a pure function of the plan's shape and the
// device's CU count; every bound below is in units of the CU count, measured
// on the 256-CU MI355X):
// * K4F takes one workgroup per CU: rounds of one frame per CU at ~0.21 ms
//   each against the streaming K4's one round (~0.75 ms) of up to 16 frames
//   per CU, so it pays for up to three rounds (scripts/exp_thresholds.sh:
//   8192 frames 12.1 vs 7.7 ms per step): plans of 1-3 frames per CU.
// * zd_k_fused holds four frames per workgroup and at most one workgroup per
//   CU beside K2 (which its K4 waves wait for): plans of 1-4 single-block
//   frames per CU (C3: 763 frames).
// * K1's sequence half one wave per block (zd_k_tables_seqw) while the plan
//   fits one round of 64 tables per CU (scripts/r3_k1wmax.sh: one rank's C4
//   share at 8 GPUs, 10,240 blocks, +1 %; full C4, 81,920 blocks, -1 %).
// * K2 beside K3 (the fork) where K3's last round of chains (64 per CU)
//   leaves LDS for K2: the round's fill f = (blocks mod 64 CUs) / (64 CUs),
//   measured with K3Q on C4-shaped plans (value, no fork -> fork): 10,240
//   blocks (f 0.63) 194 -> 221 GB/s, 20,480 (0.25) 211 -> 234, 40,960 (0.5)
//   247 -> 253; 12,288 (0.75) 221 -> 210, 16,384 (0) 251 -> 214, 32,768 (0)
//   266 -> 250, 81,920 (0) 273 -> 268; 763 (C3) and 8,192 (0.5) fork.  So
//   fork when 0 < f <= 0.65 (and at least one block per CU).
// * Without the fork, K1's two halves on the two streams (C4 273.3 -> 274.0).
// The ZD_FUSE / ZD_K4F / ZD_FORK / ZD_K1FORK / ZD_K1W_MAX environment
// variables are experiment overrides read once per process (route_env);
// nothing reads them unless they are set.
struct RouteIn {
  uint32_t cus;
  uint64_t nframes, n_tables, n_seq, n_huf;
  bool single_block_frames;      // every frame a zstd frame of one compressed block, no host-found error
  bool context;                  // a DecodingContext plan (existing output or prebuilt tables)
  uint32_t flags;                // ZD_F_*
};
struct Route {
  bool fused = false, k4f = false, k1_seq_waves = false, fork = false, k1_fork = false, k3_lat = false;
};
constexpr uint32_t K4F_MIN_PER_CU = 1, K4F_MAX_PER_CU = 3;
constexpr uint32_t FUSE_MIN_PER_CU = 1, FUSE_MAX_PER_CU = 4;
constexpr uint32_t K1W_MAX_PER_CU = 64;
constexpr uint32_t K3_CHAINS_PER_CU = 64;
// K3L (one chain per wave, latency-first) while its waves fit two a SIMD:
// beyond that K3Q's 16 chains a wave win on issue
constexpr uint32_t K3L_MAX_PER_CU = 8;
constexpr double FORK_MAX_FILL = 0.65;
Route route_plan(const RouteIn& in) {
  Route r;
  const uint64_t cus = std::max<uint32_t>(in.cus, 1);
  r.fused = !(in.flags & (ZD_F_NO_FUSE | ZD_F_SEQ_ONE_LANE | ZD_F_BLOCK_PARALLEL)) && !in.context &&
            in.single_block_frames && in.nframes >= FUSE_MIN_PER_CU * cus && in.nframes <= FUSE_MAX_PER_CU * cus;
  r.k4f = !r.fused && in.nframes >= K4F_MIN_PER_CU * cus && in.nframes <= K4F_MAX_PER_CU * cus;
  r.k1_seq_waves = in.n_tables <= K1W_MAX_PER_CU * cus && !(in.flags & ZD_F_K1_LANES);
  const uint64_t slots = K3_CHAINS_PER_CU * cus, rem = in.n_seq % slots;
  r.fork = in.n_seq >= cus && rem != 0 && (double)rem <= FORK_MAX_FILL * (double)slots;
  r.k1_fork = !r.fork && in.n_huf && in.n_seq;
  r.k3_lat = in.n_seq <= K3L_MAX_PER_CU * cus && !(in.flags & (ZD_F_SEQ_ONE_LANE | ZD_F_SEQ_NO_LATENCY));
  return r;
}
// The environment overrides (experiments only), read once
struct RouteEnv {
  int fuse = -1, k4f = -1, fork = -1, k1fork = -1, k3l = -1;
  int64_t k1w_max = -1;
  RouteEnv() {
    auto get = [](const char* n) { const char* e = getenv(n); return e ? atoi(e) : -1; };
    fuse = get("ZD_FUSE"); k4f = get("ZD_K4F"); fork = get("ZD_FORK"); k1fork = get("ZD_K1FORK"); k3l = get("ZD_K3L");
    if (const char* e = getenv("ZD_K1W_MAX")) k1w_max = atoll(e);
  }
};
const RouteEnv& route_env() {
  static const RouteEnv e;
  return e;
}
constexpr size_t PAR_INDEX_MIN_BYTES = 4u << 20;    // the host walk in parallel from 4 MiB of input (>= 512 frames)
constexpr size_t FRAMES_INDEX_SERIAL_MAX = 4096;     // zd_frames_index asked for at most this many frames: walk only them

// A process-wide pool of host worker threads (created on first use, kept:
// spawning 15 threads per planner pass cost ~0.3 ms each time).
class WorkerPool {
 public:
  static WorkerPool& get() {
    static WorkerPool* p = new WorkerPool();   // never destroyed: workers idle on the cv at exit
    return *p;
  }
  // f(k) for k in [0, n): k = 0 on the calling thread, the rest on the
  // workers (n - 1 <= size()); returns when all ran.  Not reentrant from f.
  void run(size_t n, const std::function<void(size_t)>& f) {
    std::unique_lock<std::mutex> lk(m_);
    while (busy_) idle_.wait(lk);              // one job at a time
    busy_ = true;
    job_ = &f;
    next_ = 1;
    end_ = n;
    left_ = n - 1;
    gen_++;
    go_.notify_all();
    lk.unlock();
    f(0);
    lk.lock();
    done_.wait(lk, [&] { return left_ == 0; });
    job_ = nullptr;
    busy_ = false;
    idle_.notify_one();
  }
  size_t size() const { return th_.size(); }

 private:
  WorkerPool() {
    const unsigned n = std::max(1u, std::min(16u, std::thread::hardware_concurrency())) - 1;
    for (unsigned i = 0; i < n; i++) th_.emplace_back([this] { loop(); });
    for (auto& t : th_) t.detach();
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
      go_.wait(lk, [&] { return gen_ != seen && job_ && next_ < end_; });
      seen = gen_;
      while (job_ && next_ < end_) {
        const size_t k = next_++;
        const std::function<void(size_t)>* f = job_;
        lk.unlock();
        (*f)(k);
        lk.lock();
        if (--left_ == 0) done_.notify_all();
      }
    }
  }
  std::mutex m_;
  std::condition_variable go_, done_, idle_;
  std::vector<std::thread> th_;
  const std::function<void(size_t)>* job_ = nullptr;
  size_t next_ = 0, end_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool busy_ = false;
};

// Runs f(k) for k in [0, n) in parallel (the calling thread takes k = 0;
// n - 1 must not exceed the pool's workers, else the rest run inline).
template <typename F>
void run_parts(size_t n, F f) {
  if (n <= 1) { if (n) f(0); return; }
  WorkerPool& pool = WorkerPool::get();
  const size_t par = std::min(n, pool.size() + 1);
  const std::function<void(size_t)> g = [&](size_t k) { for (size_t j = k; j < n; j += par) f(j); };
  pool.run(par, g);
}

// Pinned host staging for the descriptor upload, kept between plans: large
// plans write their descriptors straight into it at the workspace offsets
// (pinned pages never fault) and upload them with one DMA.
struct HostStage {
  std::mutex m;
  uint8_t* p = nullptr;
  size_t cap = 0;
  bool pinned = false;     // hipHostMalloc (else malloc: no device to pin for)
  void release() {
    if (p) { if (pinned) (void)hipHostFree(p); else free(p); }
    p = nullptr;
    cap = 0;
  }
};
HostStage& host_stage() {
  static HostStage h;
  return h;
}
constexpr uint64_t STAGE_MIN_BYTES = 1u << 20;     // smaller plans fill host vectors

// K3's chains in flight on the current device: 64 per CU (LDS-bound)
// (the CU count of each device, cached under a lock: plans are made and
// launched from several threads)
size_t k3_slots() {
  static std::mutex m;
  static std::vector<int> cus_of;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) { (void)hipGetLastError(); return 64 * 256; }
  std::lock_guard<std::mutex> g(m);
  if ((size_t)dev >= cus_of.size()) cus_of.resize((size_t)dev + 1, 0);
  if (!cus_of[(size_t)dev]) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
      (void)hipGetLastError();
      cus = 256;
    }
    cus_of[(size_t)dev] = cus;
  }
  return 64 * (size_t)cus_of[(size_t)dev];
}

// K4J's mode from the plan flags (ZD_K4J=1 / 0, read once, forces it on / off)
int k4j_mode_of(uint32_t flags) {
  static const char* k4j_env = getenv("ZD_K4J");
  return (flags & ZD_F_BLOCK_PARALLEL) ? 1 : (flags & ZD_F_FRAME_SERIAL) ? 0 : (k4j_env ? atoi(k4j_env) : -1);
}

// Every frame of the host walk a zstd frame of one compressed block, with no
// walk-found error (the fused kernel's plans)
bool host_single_block_frames(const zd_plan* P) {
  for (const HostPart& hp : P->parts)
    for (const HostFrame& hf : hp.frames)
      if (hf.d.kind != ZD_FRAME_ZSTD || hf.key != KEY_NONE || hf.nb != 1) return false;
  return true;
}

// The per-frame pass's plan-wide inputs (routing included): `single` =
// every frame a single-block zstd frame, `j_candidates` = frames K4J would
// take in automatic mode (frames without a walk-found error and with at
// least k4j_min compressed blocks; counted only when the mode is automatic).
PlanCtx plan_ctx(const zd_plan* P, int32_t prev_huf, const int32_t prev_tab[3], uint64_t out_len0,
                 const uint64_t rep0[3], uint64_t fixed_cap, bool single, uint64_t j_candidates) {
  PlanCtx X{};
  X.prev_huf = prev_huf;
  for (int k = 0; k < 3; k++) { X.prev_tab[k] = prev_tab[k]; X.rep0[k] = rep0[k]; }
  X.out_len0 = out_len0;
  X.fixed_cap = fixed_cap;
  X.cap0 = P->cap0;
  X.cap0_frame = nullptr;
  for (const HostPart& hp : P->parts)
    if (!hp.frames.empty()) { X.cap0_frame = hp.frames.data(); break; }
  X.flags = P->flags;
  RouteIn in{};
  in.cus = (uint32_t)(k3_slots() / 64);
  in.nframes = P->nframes;
  in.context = out_len0 != 0 || P->has_prebuilt;
  in.flags = P->flags;
  in.single_block_frames = single;
  const Route r = route_plan(in);
  const RouteEnv& E = route_env();
  X.fused = r.fused;
  // ZD_FUSE=1 forces the fused kernel on any plan of single-block frames
  // (its K2 then runs before it, not beside it, zd_decode_async); 0 off
  if (E.fuse == 0) X.fused = false;
  if (E.fuse == 1) X.fused = !(P->flags & (ZD_F_NO_FUSE | ZD_F_SEQ_ONE_LANE | ZD_F_BLOCK_PARALLEL)) && !in.context &&
                             single && P->nframes >= 1;
  X.k4f_on = E.k4f >= 0 ? E.k4f == 1 : r.k4f;
  if (X.fused) X.k4f_on = false;
  X.k4j_mode = k4j_mode_of(P->flags);
  X.k4j_min = P->nframes <= K4J_FEW_FRAMES ? K4J_MIN_BLOCKS_FEW : K4J_MIN_BLOCKS;
  X.k4j_auto = X.k4j_mode < 0 && out_len0 == 0 && j_candidates > 0 && j_candidates <= K4J_MAX_FRAMES;
  return X;
}

// The descriptor arrays at the head of the workspace (a host-filled plan
// uploads them at once)
void carve_head(Workspace& W, const PlanCounts& T, uint64_t& o) {
  auto carve = [&](uint64_t bytes) { uint64_t r = o; o = align_up(o + bytes, 256); return r; };
  W.comp = carve(sizeof(CompBlock) * std::max<uint64_t>(T.comps, 1));
  W.blocks = carve(sizeof(BlockRec) * std::max<uint64_t>(T.blocks, 1));
  W.frames = carve(sizeof(FrameDesc) * std::max<uint64_t>(T.frames, 1));
  W.frame_state0 = carve(sizeof(FrameState) * std::max<uint64_t>(T.frames, 1));
  W.list_tables = carve(4 * std::max<uint64_t>(T.tables, 1));
  W.list_huf = carve(4 * std::max<uint64_t>(T.huf, 1));
  W.list_seq = carve(4 * std::max<uint64_t>(T.seq, 1));
  W.list_k4f = carve(4 * std::max<uint64_t>(T.k4f, 1));
  W.copies = carve(sizeof(CopyDesc) * std::max<uint64_t>(T.copies, 1));
  W.jframes = carve(sizeof(JFrame) * std::max<uint64_t>(T.jframes, 1));
  W.jblkd = carve(sizeof(JBlkDesc) * std::max<uint64_t>(T.jblk, 1));
  W.jsegd = carve(sizeof(JSegDesc) * std::max<uint64_t>(T.jseg, 1));
}
// The device-only arrays after them (K4J's sizes from its descriptors)
void carve_tail(zd_plan* P, Workspace& W, const PlanCounts& T, uint64_t& o, uint64_t j_base, uint64_t j_pieces,
                uint64_t j_maxseq) {
  auto carve = [&](uint64_t bytes) { uint64_t r = o; o = align_up(o + bytes, 256); return r; };
  W.comp_state = carve(sizeof(CompState) * std::max<uint64_t>(T.comps, 1));
  W.huge = carve(4 * (std::max<uint64_t>(T.tables, 1) + 1));
  W.deep = carve(16 + (T.luts ? DEEP_POOL_BYTES : 0));
  W.frame_state = carve(sizeof(FrameState) * std::max<uint64_t>(T.frames, 1));
  W.lits = carve(T.lits + 64);
  W.seqs = carve(8 * T.nrec + 64);
  W.luts = carve((uint64_t)LUT_ENTRIES * 2 * std::max<uint64_t>(T.luts, 1));
  W.fses = carve((uint64_t)FSE_SLOT * 2 * std::max<uint64_t>(T.fses, 1));
  // K4J: pointer jumping resolves every match byte within ceil(log2(matches
  // + 1)) rounds (each pointer chain ends at a literal after at most one hop
  // per earlier match; each round halves the hops left)
  P->j_bytes = T.jframes ? j_base + 16 : 0;
  P->j_pieces = j_pieces;
  P->j_rounds = 0;
  if (T.jframes) {
    uint32_t r = 1;
    while (r < (uint32_t)J_MAX_ROUNDS - 1 && (1ull << r) <= j_maxseq + 1) r++;
    // a hop whose composed distance would reach 2^31 (J_FINAL) keeps its
    // word until its source is final, so a chain spanning k windows of
    // 2 GiB resolves within k times the rounds of one (by induction on k:
    // the bytes of the windows below are final by then, and the rest of
    // the chain is one window of hops ending at them); j_base (the plan's
    // K4J words) bounds the largest frame.  Rounds past the first are
    // sweeps that stop when nothing is pending: the bound costs nothing
    // on frames that converge sooner.
    const uint64_t k = std::max<uint64_t>(1, (j_base + (1ull << 31) - 1) >> 31);
    P->j_rounds = (uint32_t)((r + 1) * k);
  }
  W.jblk = carve(sizeof(JBlk) * std::max<uint64_t>(T.jblk, 1));
  W.jseg = carve(sizeof(JSeg) * std::max<uint64_t>(T.jseg, 1));
  W.jpend = carve(4 * (J_MAX_ROUNDS + 1));
  W.jdone = carve(std::max<uint64_t>(j_pieces, 1));
  W.jst = carve(4 * P->j_bytes + 64);
  W.redo = carve(std::max<uint64_t>(T.frames, 1));
  W.k2done = carve(4);
}
// The plan's array counts from the totals
void plan_totals(zd_plan* P, const PlanCounts& T, bool fused) {
  P->n_comps = T.comps; P->n_blocks = T.blocks; P->n_frames = T.frames;
  P->n_tables = T.tables; P->n_huf = T.huf; P->n_seq = T.seq; P->n_k4f = T.k4f; P->n_copies = T.copies;
  P->n_jframes = T.jframes; P->n_jblk = T.jblk; P->n_jseg = T.jseg; P->n_k0only = T.k0only;
  P->fused = fused && T.jframes == 0 && T.k4f == 0;
}
void plan_info(zd_plan* P, const PlanCounts& T) {
  zd_plan_info& I = P->info;
  I.nframes = T.frames;
  I.nblocks = T.blocks;
  I.ncompressed = T.comps;
  I.out_bytes = T.out;
  I.out_exact = T.exact();
  I.workspace_bytes = P->W.total;
  I.nsequences = T.nseq;
  I.nliterals = T.lits;
  I.index_status = P->index_status;
  I.executors = (P->fused ? ZD_EXEC_FUSED : 0u) | (P->n_k4f ? ZD_EXEC_K4F : 0u) | (P->n_jframes ? ZD_EXEC_K4J : 0u);
}

// The largest K4J frame's sequence count (plan_frame's jm)
struct JMax {
  uint64_t m = 0;
  void note(uint64_t n) { m = std::max(m, n); }
};

// Builds device-side descriptors from the host frames: one counting pass and
// one filling pass over the parts in parallel (each part's entries start at
// the counts of the parts before it), then the K4J descriptors in frame order.
// `staged`: a large plan may fill the pinned staging (zd_plan_create); the
// context API keeps host vectors it edits afterwards.
int build_plan(zd_plan* P, int32_t prev_huf, const int32_t prev_tab[3], uint64_t out_len0,
               const uint64_t rep0[3], uint64_t fixed_cap, bool staged = false) {
  uint64_t j_candidates = 0;
  if (k4j_mode_of(P->flags) < 0 && out_len0 == 0) {
    const uint32_t k4j_min = P->nframes <= K4J_FEW_FRAMES ? K4J_MIN_BLOCKS_FEW : K4J_MIN_BLOCKS;
    for (const HostPart& hp : P->parts)
      for (const HostFrame& hf : hp.frames) j_candidates += hf.key == KEY_NONE && hf.ncomp >= k4j_min;
  }
  const PlanCtx X = plan_ctx(P, prev_huf, prev_tab, out_len0, rep0, fixed_cap, host_single_block_frames(P),
                             j_candidates);

  const size_t np = P->parts.size();
  std::vector<PlanCounts> cnt(np + 1);
  const Sink none{};
  run_parts(np, [&](size_t k) {
    const HostPart& hp = P->parts[k];
    PlanCounts c;
    for (const HostFrame& hf : hp.frames) plan_frame<false, JMax>(X, hf, hp.blocks.data(), c, none, nullptr);
    if (X.fused) {          // parts start aligned, so the filling pass pads exactly as this count did
      c.lits = align_up(c.lits, 128);
      c.nrec = align_up(c.nrec, 16);
    }
    cnt[k + 1] = c;
  });
  for (size_t k = 1; k <= np; k++) { PlanCounts t = cnt[k - 1]; t.add(cnt[k]); cnt[k] = t; }
  const PlanCounts T = cnt[np];

  // workspace carve-up: the arrays the host fills first (one upload), then
  // the device-only ones
  Workspace& W = P->W;
  W = Workspace{};
  uint64_t o = 0;
  carve_head(W, T, o);
  P->desc_bytes = o;
  plan_totals(P, T, X.fused);
  P->frame_out.resize(T.frames);
  P->frame_cap.resize(T.frames);
  Sink S{};
  P->staged = staged && P->desc_bytes >= STAGE_MIN_BYTES;
  if (P->staged) {
    // held until upload_plan has copied the staging out
    P->stage_lock = std::unique_lock<std::mutex>(host_stage().m);
    HostStage& H = host_stage();
    if (H.cap < P->desc_bytes) {
      H.release();
      const size_t want = P->desc_bytes + (P->desc_bytes >> 2);
      H.pinned = hipHostMalloc((void**)&H.p, want, hipHostMallocDefault) == hipSuccess;
      if (!H.pinned) {
        (void)hipGetLastError();
        H.p = (uint8_t*)aligned_alloc(4096, align_up(want, 4096));
      }
      if (!H.p) return ZD_E_NO_MEMORY;
      H.cap = want;
    }
    uint8_t* b = H.p;
    S = Sink{(CompBlock*)(b + W.comp), (BlockRec*)(b + W.blocks), (FrameDesc*)(b + W.frames),
             (FrameState*)(b + W.frame_state0), (uint32_t*)(b + W.list_tables), (uint32_t*)(b + W.list_huf),
             (uint32_t*)(b + W.list_seq), (uint32_t*)(b + W.list_k4f), (CopyDesc*)(b + W.copies),
             (JFrame*)(b + W.jframes), (JBlkDesc*)(b + W.jblkd), (JSegDesc*)(b + W.jsegd), nullptr, nullptr};
    P->comps.clear(); P->blocks.clear(); P->fdesc.clear(); P->fstate0.clear();
    P->list_tables.clear(); P->list_huf.clear(); P->list_seq.clear(); P->list_k4f.clear(); P->copies.clear();
    P->jframes.clear(); P->jblkd.clear(); P->jsegd.clear();
  } else {
    P->comps.assign(T.comps, CompBlock{});
    P->blocks.assign(T.blocks, BlockRec{});
    P->fdesc.assign(T.frames, FrameDesc{});
    P->fstate0.assign(T.frames, FrameState{});
    P->list_tables.assign(T.tables, 0);
    P->list_huf.assign(T.huf, 0);
    P->list_seq.assign(T.seq, 0);
    P->list_k4f.assign(T.k4f, 0);
    P->copies.assign(T.copies, CopyDesc{});
    P->jframes.assign(T.jframes, JFrame{});
    P->jblkd.assign(T.jblk, JBlkDesc{});
    P->jsegd.assign(T.jseg, JSegDesc{});
    S = Sink{P->comps.data(), P->blocks.data(), P->fdesc.data(), P->fstate0.data(), P->list_tables.data(),
             P->list_huf.data(), P->list_seq.data(), P->list_k4f.data(), P->copies.data(), P->jframes.data(),
             P->jblkd.data(), P->jsegd.data(), nullptr, nullptr};
  }
  S.frame_out = P->frame_out.data();
  S.frame_cap = P->frame_cap.data();
  // (the K4J descriptors are written by plan_frame at the running K4J indices)
  std::vector<JMax> jm(np);
  run_parts(np, [&](size_t k) {
    const HostPart& hp = P->parts[k];
    PlanCounts c = cnt[k];
    for (const HostFrame& hf : hp.frames) plan_frame<true, JMax>(X, hf, hp.blocks.data(), c, S, &jm[k]);
  });
  uint64_t j_maxseq = 0;
  for (const JMax& m : jm) j_maxseq = std::max(j_maxseq, m.m);
  carve_tail(P, W, T, o, T.jwords, T.jpieces, j_maxseq);
  W.total = o;

  plan_info(P, T);
  return 0;
}

// Device workspaces of destroyed plans, kept for the next plans of this
// process (a plan's workspace is up to ~1.2x its decoded bytes: K3's
// records, the literals, the tables).  A plan takes a cached block of at
// least its size and at most 1.25x + 64 MiB; zd_trim_cache() frees them all,
// and so does a failed allocation before its retry.  ZD_WS_CACHE_MB caps
// the bytes held (default 8 GiB, at most 4 blocks; 0 disables the cache).
// The cache is invisible to PyTorch's allocator: a torch user that needs the
// memory back calls zd_trim_cache.
struct WsCache {
  struct E { int dev; uint8_t* p; uint64_t bytes; };
  std::mutex m;
  std::vector<E> free;
  uint64_t held = 0;
};
WsCache& ws_cache() {
  static WsCache c;
  return c;
}
uint64_t ws_cache_limit() {
  static const uint64_t lim = getenv("ZD_WS_CACHE_MB") ? strtoull(getenv("ZD_WS_CACHE_MB"), nullptr, 0) << 20
                                                       : 8ull << 30;
  return lim;
}
void ws_trim(int dev) {           // dev < 0: every device
  WsCache& C = ws_cache();
  std::lock_guard<std::mutex> g(C.m);
  for (size_t i = 0; i < C.free.size();) {
    if (dev < 0 || C.free[i].dev == dev) {
      (void)hipFree(C.free[i].p);
      C.held -= C.free[i].bytes;
      C.free.erase(C.free.begin() + (long)i);
    } else {
      i++;
    }
  }
}
hipError_t ws_alloc(int dev, uint64_t bytes, uint8_t** p, uint64_t* got) {
  {
    WsCache& C = ws_cache();
    std::lock_guard<std::mutex> g(C.m);
    size_t best = SIZE_MAX;
    for (size_t i = 0; i < C.free.size(); i++) {
      const WsCache::E& e = C.free[i];
      if (e.dev == dev && e.bytes >= bytes && e.bytes <= bytes + bytes / 4 + (64ull << 20) &&
          (best == SIZE_MAX || e.bytes < C.free[best].bytes))
        best = i;
    }
    if (best != SIZE_MAX) {
      *p = C.free[best].p;
      *got = C.free[best].bytes;
      C.held -= *got;
      C.free.erase(C.free.begin() + (long)best);
      return hipSuccess;
    }
  }
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    ws_trim(dev);
    e = hipMalloc(p, bytes);
  }
  *got = bytes;
  return e;
}
// (dev: the device p was allocated on, whatever device is current now)
void ws_release(uint8_t* p, uint64_t bytes, int dev) {
  if (!p) return;
  const uint64_t lim = ws_cache_limit();
  if (dev < 0 || bytes > lim) { (void)hipFree(p); return; }
  WsCache& C = ws_cache();
  std::lock_guard<std::mutex> g(C.m);
  C.free.push_back(WsCache::E{dev, p, bytes});
  C.held += bytes;
  while (C.held > lim || C.free.size() > 4) {        // oldest first
    (void)hipFree(C.free.front().p);
    C.held -= C.free.front().bytes;
    C.free.erase(C.free.begin());
  }
}

// the output staging of a plan whose frames' sizes are bounds
int upload_staging(zd_plan* P) {
  if (!P->info.out_exact) {
    P->staging_bytes = P->info.out_bytes;
    HIPCHK(hipMalloc(&P->d_staging, std::max<uint64_t>(P->staging_bytes, 16)));
  }
  return 0;
}

int upload_plan(zd_plan* P) {
  HIPCHK(hipGetDevice(&P->dev));
  HIPCHK(ws_alloc(P->dev, P->W.total, &P->d_ws, &P->ws_bytes));
  if (P->staged) {
    // the descriptors are in the pinned staging at their workspace offsets
    const hipError_t e = hipMemcpy(P->d_ws, host_stage().p, P->desc_bytes, hipMemcpyHostToDevice);
    P->stage_lock = std::unique_lock<std::mutex>();
    HIPCHK(e);
  } else {
    const Workspace& W = P->W;
    struct Piece { uint64_t off; const void* p; size_t bytes; };
    const Piece pieces[] = {
        {W.comp, P->comps.data(), P->comps.size() * sizeof(CompBlock)},
        {W.blocks, P->blocks.data(), P->blocks.size() * sizeof(BlockRec)},
        {W.frames, P->fdesc.data(), P->fdesc.size() * sizeof(FrameDesc)},
        {W.frame_state0, P->fstate0.data(), P->fstate0.size() * sizeof(FrameState)},
        {W.list_tables, P->list_tables.data(), P->list_tables.size() * 4},
        {W.list_huf, P->list_huf.data(), P->list_huf.size() * 4},
        {W.list_seq, P->list_seq.data(), P->list_seq.size() * 4},
        {W.list_k4f, P->list_k4f.data(), P->list_k4f.size() * 4},
        {W.copies, P->copies.data(), P->copies.size() * sizeof(CopyDesc)},
        {W.jframes, P->jframes.data(), P->jframes.size() * sizeof(JFrame)},
        {W.jblkd, P->jblkd.data(), P->jblkd.size() * sizeof(JBlkDesc)},
        {W.jsegd, P->jsegd.data(), P->jsegd.size() * sizeof(JSegDesc)},
    };
    for (const Piece& q : pieces)
      if (q.bytes) HIPCHK(hipMemcpy(P->d_ws + q.off, q.p, q.bytes, hipMemcpyHostToDevice));
  }
  return upload_staging(P);
}

// A plan's second stream and its fork/join events, kept for the next plans
// of the process (creating them took ~0.25 ms per plan).
struct AuxSet { int dev; hipStream_t s; hipEvent_t fork, join; };
std::mutex& aux_mutex() {
  static std::mutex m;
  return m;
}
std::vector<AuxSet>& aux_free() {
  static std::vector<AuxSet>* v = new std::vector<AuxSet>();   // never destroyed (no HIP calls at exit)
  return *v;
}
bool aux_take(zd_plan* P) {
  const int dev = P->dev;                 // upload_plan's device (current here)
  if (dev < 0) return false;
  {
    std::lock_guard<std::mutex> g(aux_mutex());
    auto& v = aux_free();
    for (size_t i = 0; i < v.size(); i++) {
      if (v[i].dev != dev) continue;
      P->aux = v[i].s; P->fork = v[i].fork; P->join = v[i].join;
      v.erase(v.begin() + (long)i);
      return true;
    }
  }
  return hipStreamCreateWithFlags(&P->aux, hipStreamNonBlocking) == hipSuccess &&
         hipEventCreateWithFlags(&P->fork, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&P->join, hipEventDisableTiming) == hipSuccess;
}
void aux_give(zd_plan* P) {
  const int dev = P->dev;                 // the plan's device, not the current one
  if (P->aux && P->fork && P->join && dev >= 0) {
    std::lock_guard<std::mutex> g(aux_mutex());
    if (aux_free().size() < 8) {
      aux_free().push_back(AuxSet{dev, P->aux, P->fork, P->join});
      P->aux = nullptr; P->fork = P->join = nullptr;
      return;
    }
  }
  if (P->fork) (void)hipEventDestroy(P->fork);
  if (P->join) (void)hipEventDestroy(P->join);
  if (P->aux) (void)hipStreamDestroy(P->aux);
  P->aux = nullptr; P->fork = P->join = nullptr;
}

// Frames from in (FrameIterator::next, frame.rs:94-99) into `part` until the
// input ends, a frame starting at or past `stop` comes up, or one fails (kept,
// with its status).
int index_frames(const uint8_t* src, Bytes& in, size_t stop, HostPart& part) {
  while (in.n && (size_t)(in.p - src) < stop) {
    HostFrame hf;
    VecSink sink{part.blocks};
    int r = index_frame(src, in, &hf, sink);
    part.frames.push_back(hf);
    if (r) return r;
  }
  return 0;
}

// Index of the frame of a chain (frames in input order) that starts at byte
// `at`, or SIZE_MAX.
template <typename FR>
size_t chain_start(const FR& frames, size_t at, size_t count = SIZE_MAX) {
  size_t lo = 0, hi = std::min(count, (size_t)frames.size());
  while (lo < hi) {
    const size_t m = lo + (hi - lo) / 2;
    if (frames[m].d.src_offset < at) lo = m + 1; else hi = m;
  }
  return (lo < std::min(count, (size_t)frames.size()) && frames[lo].d.src_offset == at) ? lo : SIZE_MAX;
}

inline bool magic_at(const uint8_t* p) {
  uint32_t m;
  memcpy(&m, p, 4);
  return magic_word(m);
}

// The host walk (FrameIterator over the whole input).  Large inputs are cut
// into T byte ranges; thread k finds the first frame magic in its range and
// indexes the chain of frames from there while they start inside the range.
// Each frame's start follows from the one before it, so a chain that reaches
// a position of the true chain (the one from offset 0) is the true chain
// from there on.  The stitch checks exactly that: range k's frames are kept
// from the frame that starts where the kept frames before it end; a range
// whose chain never meets that position (a magic number inside data, or a
// frame longer than a range) is dropped and the walk continues serially.
// The result is the serial walk's, first failing frame included.
int plan_index(zd_plan* P, const uint8_t* src, size_t n) {
  static const char* wt = getenv("ZD_WALK_THREADS");   // experiments
  const unsigned hw = wt ? (unsigned)std::max(1, atoi(wt)) : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const size_t T = n >= PAR_INDEX_MIN_BYTES ? std::min<size_t>(hw, n >> 20) : 1;
  std::vector<HostPart> part(T);
  std::vector<int> st(T, 0);
  std::vector<size_t> end(T, 0), cut(T + 1);
  for (size_t k = 0; k <= T; k++) cut[k] = (size_t)((unsigned __int128)n * k / T);
  std::vector<double> tms(T, 0.0);
  const auto tw0 = std::chrono::steady_clock::now();
  run_parts(T, [&](size_t k) {
    const auto tk0 = std::chrono::steady_clock::now();
    struct Stamp {
      double& out; std::chrono::steady_clock::time_point t0;
      ~Stamp() { out = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
    } stamp{tms[k], tk0};
    size_t p = cut[k];
    for (;;) {
      if (k) {                                   // the first candidate frame start in the range
        while (p < cut[k + 1] && (p + 4 > n || !magic_at(src + p))) p++;
        if (p >= cut[k + 1]) { end[k] = p; return; }
      }
      part[k].blocks.reserve((cut[k + 1] - cut[k]) / (16u << 10) + 16);
      Bytes in{src + p, n - p};
      st[k] = index_frames(src, in, cut[k + 1], part[k]);
      end[k] = (size_t)(in.p - src);
      // a candidate that fails at once was a magic inside data: look further
      if (k && st[k] && part[k].frames.size() == 1) {
        part[k].frames.clear();
        part[k].blocks.clear();
        st[k] = 0;
        p++;
        continue;
      }
      return;
    }
  });
  std::vector<HostPart> keep;
  int status = 0;
  size_t cur = 0;                                // where the kept frames end
  uint64_t serial = 0;                           // bytes the stitch walked itself
  for (size_t k = 0; k < T && !status;) {
    if (k && cur >= cut[k + 1]) { k++; continue; }   // the range lies inside a kept frame
    const size_t i = k ? chain_start(part[k].frames, cur) : 0;
    if (i != SIZE_MAX) {
      HostPart& hp = part[k];
      if (i) hp.frames.erase(hp.frames.begin(), hp.frames.begin() + (long)i);   // their blocks stay unreferenced
      status = st[k];
      cur = end[k];
      keep.push_back(std::move(hp));
      k++;
      continue;
    }
    // The chains do not meet (range k's walk started at a magic number
    // inside data, or its first frame starts in an earlier range): walk on
    // from cur frame by frame, only until a frame ends where a later range's
    // chain has a frame start, then stitch on from that range.  One planted
    // magic number costs at most the ranges it spoils, never the rest of the
    // input (the walks from a given position are identical).
    HostPart tail;
    Bytes in{src + cur, n - cur};
    size_t kk = k;
    while (in.n) {
      HostFrame hf;
      VecSink sink{tail.blocks};
      const int r = index_frame(src, in, &hf, sink);
      tail.frames.push_back(hf);
      const size_t p = (size_t)(in.p - src);
      serial += p - cur;
      cur = p;
      if (r) { status = r; break; }
      while (kk + 1 < T && cur >= cut[kk + 1]) kk++;
      if (kk > k && chain_start(part[kk].frames, cur) != SIZE_MAX) break;
    }
    keep.push_back(std::move(tail));
    k = kk > k ? kk : T;
  }
  const auto tw1 = std::chrono::steady_clock::now();
  P->set_parts(std::move(keep));
  if (getenv("ZD_PLAN_TIMES")) {
    fprintf(stderr, "zd walk: %zu threads, threads", T);
    for (double t : tms) fprintf(stderr, " %.1f", t);
    fprintf(stderr, " ms; walk %.2f ms, stitch %.2f ms, serial %llu bytes\n",
            std::chrono::duration<double, std::milli>(tw1 - tw0).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw1).count(),
            (unsigned long long)serial);
  }
  P->index_status = status;
  P->index_stop = P->nframes;
  P->info.walk_serial_bytes = serial;
  return 0;
}

// The device walk (zd_kernels.hip zd_k_walk): plan_index for an input that
// is resident in HBM.  Byte ranges of >= 256 KiB (at most 16384 of them),
// one wave each; the count pass gives every range's chain (WalkRange), the
// fill pass writes their frames and blocks into one array each, which come
// back to the host through pinned staging.  The stitch is plan_index's, over
// the ranges; where two chains do not meet, the rest of the input is walked
// serially on the device (one range from there to the end).  The kept frames
// are then cut into parts for the parallel descriptor build.
struct DevWalkBufs {                      // device and pinned buffers, kept between plans
  std::mutex m;
  int dev = -1;
  WalkRange* d_wr = nullptr;
  size_t cap_wr = 0;
  uint8_t* d_out = nullptr;              // frames | blocks
  size_t cap_out = 0;
  uint8_t* h_out = nullptr;              // pinned
  size_t cap_h = 0;
  WalkRange* h_wr = nullptr;             // pinned
  size_t cap_hwr = 0;
  size_t fb = 0, bytes = 0;              // the last fill pass: frames | blocks layout in d_out
  // the device descriptor build (build_plan_device): per-frame counts and
  // tile sums, the frames' output offsets and capacities, the shape
  uint64_t* d_cnt = nullptr;
  size_t cap_cnt = 0;
  uint64_t* d_tot = nullptr;
  size_t cap_tot = 0;
  uint64_t* d_fo = nullptr;
  size_t cap_fo = 0;
  PlanShape* d_shape = nullptr;
  uint64_t* h_small = nullptr;           // pinned: shape, totals
};
DevWalkBufs& dev_walk_bufs() {
  static DevWalkBufs* b = new DevWalkBufs();
  return *b;
}

template <typename T>
bool grow_dev(T*& p, size_t& cap, size_t need) {
  if (need <= cap) return true;
  const size_t n = need;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  if (hipMalloc(&p, n * sizeof(T)) != hipSuccess) { (void)hipGetLastError(); return false; }
  cap = n;
  return true;
}
template <typename T>
bool grow_pinned(T*& p, size_t& cap, size_t need) {
  if (need <= cap) return true;
  const size_t n = need;
  if (p) (void)hipHostFree(p);
  p = nullptr;
  cap = 0;
  if (hipHostMalloc(&p, n * sizeof(T), hipHostMallocDefault) != hipSuccess) return false;
  cap = n;
  return true;
}

// zd_plan_decompress's host <-> device path: a process-wide ring of two
// pinned chunks.  H2D: chunk k is copied into its pinned slot by the worker
// pool while chunk k - 1's DMA runs; D2H: chunk k + 1's DMA runs while chunk
// k is copied out.  (A pageable hipMemcpy stages through the runtime's own
// buffers with one thread.)  Without pinned memory it falls back to that.
constexpr uint64_t IO_CHUNK = 32ull << 20;
struct IoRing {
  std::mutex m;
  uint8_t* p[2] = {nullptr, nullptr};
  bool tried = false;
  bool ok() {
    if (!tried) {
      tried = true;
      for (auto& b : p)
        if (hipHostMalloc((void**)&b, IO_CHUNK, hipHostMallocDefault) != hipSuccess) { (void)hipGetLastError(); b = nullptr; }
      if (!p[0] || !p[1]) {
        for (auto& b : p) if (b) (void)hipHostFree(b);
        p[0] = p[1] = nullptr;
      }
    }
    return p[0] != nullptr;
  }
};
IoRing& io_ring() {
  static IoRing* r = new IoRing();   // never destroyed (no HIP calls at exit)
  return *r;
}
struct IoEvents {
  hipEvent_t e[2] = {nullptr, nullptr};
  bool ok = true;
  IoEvents() {
    for (auto& x : e) ok = ok && hipEventCreateWithFlags(&x, hipEventDisableTiming) == hipSuccess;
  }
  ~IoEvents() { for (auto& x : e) if (x) (void)hipEventDestroy(x); }
};
void par_memcpy(uint8_t* d, const uint8_t* s, size_t n) {
  const size_t T = std::min<size_t>(16, std::max<size_t>(1, n >> 21));   // >= 2 MiB a thread
  run_parts(T, [&](size_t k) {
    const size_t a = n * k / T, b = n * (k + 1) / T;
    memcpy(d + a, s + a, b - a);
  });
}
// The ring is held only while its slots are in use: the H2D copy returns
// after its last DMA (the stream synchronised), the D2H copy after its last
// host copy, so decodes on other plans or devices run beside it.
int io_h2d(uint8_t* d, const uint8_t* h, size_t n, hipStream_t s, IoRing& R, hipEvent_t ev[2]) {
  if (!n) return 0;
  std::lock_guard<std::mutex> lk(R.m);
  if (!R.ok()) { HIPCHK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s)); HIPCHK(hipStreamSynchronize(s)); return 0; }
  for (size_t o = 0, k = 0; o < n; o += IO_CHUNK, k++) {
    const size_t c = std::min<size_t>(IO_CHUNK, n - o);
    if (k >= 2) HIPCHK(hipEventSynchronize(ev[k & 1]));   // chunk k - 2's DMA out of this slot
    par_memcpy(R.p[k & 1], h + o, c);
    HIPCHK(hipMemcpyAsync(d + o, R.p[k & 1], c, hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(ev[k & 1], s));
  }
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}
int io_d2h(uint8_t* h, const uint8_t* d, size_t n, hipStream_t s, IoRing& R, hipEvent_t ev[2]) {
  if (!n) return 0;
  std::lock_guard<std::mutex> lk(R.m);
  if (!R.ok()) { HIPCHK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s)); HIPCHK(hipStreamSynchronize(s)); return 0; }
  const size_t nk = (n + IO_CHUNK - 1) / IO_CHUNK;
  auto chunk = [&](size_t k) { return std::min<size_t>(IO_CHUNK, n - k * IO_CHUNK); };
  auto issue = [&](size_t k) -> int {
    HIPCHK(hipMemcpyAsync(R.p[k & 1], d + k * IO_CHUNK, chunk(k), hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(ev[k & 1], s));
    return 0;
  };
  if (int r = issue(0)) return r;
  for (size_t k = 0; k < nk; k++) {
    if (k + 1 < nk) if (int r = issue(k + 1)) return r;
    HIPCHK(hipEventSynchronize(ev[k & 1]));
    par_memcpy(h + k * IO_CHUNK, R.p[k & 1], chunk(k));
  }
  return 0;
}

// The fill pass's index (in B.d_out) -> the pinned copy
int dev_walk_download(DevWalkBufs& B, hipStream_t s, const HostFrame** frames, const HostBlock** blocks) {
  if (hipMemcpyAsync(B.h_out, B.d_out, B.bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return ZD_E_HIP;
  *frames = (const HostFrame*)B.h_out;
  *blocks = (const HostBlock*)(B.h_out + B.fb);
  return 0;
}

// Walks `nranges` ranges from `first`; on return wr (pinned) holds the
// summaries with f_off / b_off, frames / blocks (pinned) the fill pass.
int dev_walk(DevWalkBufs& B, const uint8_t* d_src, uint64_t n, uint64_t first, uint64_t chunk, uint32_t nranges,
             hipStream_t s, uint64_t* F_out, uint64_t* B_out, const HostFrame** frames, const HostBlock** blocks,
             bool download = true) {
  if (!grow_dev(B.d_wr, B.cap_wr, nranges) || !grow_pinned(B.h_wr, B.cap_hwr, nranges)) return ZD_E_HIP;
  if (launch_walk(d_src, n, first, chunk, nranges, B.d_wr, nullptr, nullptr, false, s) != hipSuccess ||
      hipMemcpyAsync(B.h_wr, B.d_wr, nranges * sizeof(WalkRange), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return ZD_E_HIP;
  uint64_t F = 0, NB = 0;
  for (uint32_t k = 0; k < nranges; k++) {
    B.h_wr[k].f_off = F; B.h_wr[k].b_off = NB;
    F += B.h_wr[k].nframes; NB += B.h_wr[k].nblocks;
  }
  const size_t fb = align_up(F * sizeof(HostFrame), 256), bytes = fb + NB * sizeof(HostBlock);
  *F_out = F;
  *B_out = NB;
  if (!F) return 0;
  if (!grow_dev(B.d_out, B.cap_out, bytes) || !grow_pinned(B.h_out, B.cap_h, bytes)) return ZD_E_HIP;
  HostFrame* d_frames = (HostFrame*)B.d_out;
  HostBlock* d_blocks = (HostBlock*)(B.d_out + fb);
  if (hipMemcpyAsync(B.d_wr, B.h_wr, nranges * sizeof(WalkRange), hipMemcpyHostToDevice, s) != hipSuccess ||
      launch_walk(d_src, n, first, chunk, nranges, B.d_wr, d_frames, d_blocks, true, s) != hipSuccess)
    return ZD_E_HIP;
  B.fb = fb;
  B.bytes = bytes;
  if (download) return dev_walk_download(B, s, frames, blocks);
  return hipStreamSynchronize(s) != hipSuccess ? ZD_E_HIP : 0;
}

// Frames fr[i] (i in the kept list) with their blocks (global indices into
// bl) -> parts of about equal frame counts, built in parallel, b0 rebased.
void parts_from(const std::vector<const HostFrame*>& kept, const HostBlock* bl, std::vector<HostPart>& out) {
  const size_t nf = kept.size();
  const size_t T = std::max<size_t>(1, std::min<size_t>(16, nf / 512));
  const size_t base = out.size();
  out.resize(base + T);
  run_parts(T, [&](size_t t) {
    const size_t a = nf * t / T, e = nf * (t + 1) / T;
    HostPart& hp = out[base + t];
    size_t nb = 0;
    for (size_t i = a; i < e; i++) nb += kept[i]->nb;
    hp.frames.resize(e - a);
    hp.blocks.resize(nb);
    size_t b = 0;
    for (size_t i = a; i < e; i++) {
      HostFrame f = *kept[i];
      memcpy(hp.blocks.data() + b, bl + f.b0, f.nb * sizeof(HostBlock));
      f.b0 = (uint32_t)b;
      b += f.nb;
      hp.frames[i - a] = f;
    }
  });
}

// The descriptors of a device-walked plan built on the GPU:
// frames [0, F) of the walk's index in B.d_out (block indices global) are the
// plan's frames.  The host reads back the routing shape (two counters), the
// plan's totals (PLAN_FIELDS words) and the frames' output offsets and
// capacities (16 bytes a frame); everything else is written in place in the
// workspace by the planner's own per-frame pass (zd_plan.h plan_frame).
// K4J frames included: plan_frame writes their descriptors at the scanned
// K4J indices, and the count pass reports the largest K4J frame's sequence
// count (the rounds), so no plan falls back to the host build.
int build_plan_device(zd_plan* P, DevWalkBufs& B, uint64_t F, hipStream_t s) {
  const HostFrame* d_frames = (const HostFrame*)B.d_out;
  const HostBlock* d_blocks = (const HostBlock*)(B.d_out + B.fb);
  P->nframes = F;
  const uint32_t k4j_min = F <= K4J_FEW_FRAMES ? K4J_MIN_BLOCKS_FEW : K4J_MIN_BLOCKS;
  const uint64_t nt = (F + 255) / 256;
  if (!B.d_shape && hipMalloc(&B.d_shape, sizeof(PlanShape)) != hipSuccess) return ZD_E_HIP;
  if (!B.h_small && hipHostMalloc((void**)&B.h_small, 64 * 8, hipHostMallocDefault) != hipSuccess) return ZD_E_HIP;
  if (!grow_dev(B.d_cnt, B.cap_cnt, std::max<uint64_t>(F, 1) * PLAN_FIELDS) ||
      !grow_dev(B.d_tot, B.cap_tot, (nt + 1) * PLAN_FIELDS) || !grow_dev(B.d_fo, B.cap_fo, 2 * std::max<uint64_t>(F, 1)))
    return ZD_E_HIP;
  HIPCHK(launch_plan_shape(d_frames, F, k4j_min, B.d_shape, s));
  HIPCHK(hipMemcpyAsync(B.h_small, B.d_shape, sizeof(PlanShape), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  PlanShape shape;
  memcpy(&shape, B.h_small, sizeof shape);
  const int32_t none[3] = {-1, -1, -1};
  const uint64_t rep0[3] = {1, 4, 8};
  const PlanCtx X = plan_ctx(P, -1, none, 0, rep0, 0, shape.multi == 0, k4j_mode_of(P->flags) < 0 ? shape.jcand : 0);
  HIPCHK(launch_plan_count(X, d_frames, d_blocks, F, B.d_cnt, B.d_tot, B.d_shape, s));
  HIPCHK(hipMemcpyAsync(B.h_small, B.d_tot + nt * PLAN_FIELDS, PLAN_FIELDS * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(B.h_small + PLAN_FIELDS, B.d_shape, sizeof(PlanShape), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  PlanCounts T;
  memcpy(&T, B.h_small, sizeof T);
  memcpy(&shape, B.h_small + PLAN_FIELDS, sizeof shape);
  Workspace& W = P->W;
  W = Workspace{};
  uint64_t o = 0;
  carve_head(W, T, o);
  P->desc_bytes = o;
  plan_totals(P, T, X.fused);
  carve_tail(P, W, T, o, T.jwords, T.jpieces, shape.jmaxseq);
  W.hframes = o;
  o = align_up(o + sizeof(HostFrame) * std::max<uint64_t>(F, 1), 256);
  W.total = o;
  HIPCHK(hipGetDevice(&P->dev));
  HIPCHK(ws_alloc(P->dev, W.total, &P->d_ws, &P->ws_bytes));
  uint8_t* b = P->d_ws;
  uint64_t* d_fout = B.d_fo;
  uint64_t* d_fcap = B.d_fo + std::max<uint64_t>(F, 1);
  const Sink S{(CompBlock*)(b + W.comp), (BlockRec*)(b + W.blocks), (FrameDesc*)(b + W.frames),
               (FrameState*)(b + W.frame_state0), (uint32_t*)(b + W.list_tables), (uint32_t*)(b + W.list_huf),
               (uint32_t*)(b + W.list_seq), (uint32_t*)(b + W.list_k4f), (CopyDesc*)(b + W.copies),
               (JFrame*)(b + W.jframes), (JBlkDesc*)(b + W.jblkd), (JSegDesc*)(b + W.jsegd), d_fout, d_fcap};
  HIPCHK(launch_plan_fill(X, d_frames, d_blocks, F, B.d_cnt, B.d_tot, S, s));
  if (F) HIPCHK(hipMemcpyAsync(b + W.hframes, d_frames, F * sizeof(HostFrame), hipMemcpyDeviceToDevice, s));
  P->frame_out.resize(F);
  P->frame_cap.resize(F);
  if (F) {
    HIPCHK(hipMemcpyAsync(P->frame_out.data(), d_fout, F * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(P->frame_cap.data(), d_fcap, F * 8, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  P->dev_built = true;
  P->staged = false;
  plan_info(P, T);
  P->info.device_descriptors = 1;
  return 0;
}

// ZD_DEV_DESC=0 (read once): device-walked plans take the host's descriptor
// build (the comparison leg of tests/test_gpu_walk.py)
bool dev_host_descriptors() {
  static const bool off = getenv("ZD_DEV_DESC") && atoi(getenv("ZD_DEV_DESC")) == 0;
  return off;
}

int plan_index_dev(zd_plan* P, const uint8_t* d_src, size_t n, hipStream_t s) {
  const auto tw0 = std::chrono::steady_clock::now();
  std::vector<HostPart> keep;
  int status = 0;
  double t_walk = 0, t_tail = 0;
  uint64_t serial_dev = 0;                    // bytes the stitch walked itself (tail walks)
  if (n) {
    DevWalkBufs& B = dev_walk_bufs();
    std::lock_guard<std::mutex> lk(B.m);
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (B.dev != dev) {                      // buffers of another device: start over
      if (B.d_wr) (void)hipFree(B.d_wr);
      if (B.d_out) (void)hipFree(B.d_out);
      B.d_wr = nullptr; B.cap_wr = 0; B.d_out = nullptr; B.cap_out = 0;
      B.dev = dev;
    }
    const uint64_t chunk = std::max<uint64_t>(256u << 10, (n + 16383) / 16384);
    const uint32_t T = (uint32_t)((n + chunk - 1) / chunk);
    uint64_t F = 0, NB = 0;
    const HostFrame* fr = nullptr;
    const HostBlock* bl = nullptr;
    if (int r = dev_walk(B, d_src, n, 0, chunk, T, s, &F, &NB, &fr, &bl, false)) return r;
    t_walk = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw0).count();
    const auto cut = [&](size_t k) { return std::min<uint64_t>((uint64_t)k * chunk, n); };
    // The common case from the range summaries alone: every range's chain
    // starts where the kept frames before it end (or the range lies inside a
    // kept frame and found none), so the plan's frames are a prefix of the
    // walk's index, and its descriptors are built where the index is
    // (build_plan_device); otherwise the index comes back for the host stitch.
    if (F && !dev_host_descriptors()) {
      uint64_t cur = 0, kept_end = 0;
      int st = 0;
      bool ok = true;
      for (size_t k = 0; k < T && !st && ok; k++) {
        const WalkRange& R = B.h_wr[k];
        if (k && cur >= cut(k + 1)) { ok = R.nframes == 0; continue; }
        if (k && !(R.nframes && R.p0 == cur)) { ok = false; break; }
        kept_end = R.f_off + R.nframes;
        st = R.status;
        cur = R.end;
      }
      if (ok) {
        const int r = build_plan_device(P, B, kept_end, s);
        if (r < 0) return r;
        if (r == 0) {
          P->index_status = st;
          P->info.index_status = st;
          P->info.walk_serial_bytes = 0;
          P->index_stop = P->nframes;
          if (getenv("ZD_PLAN_TIMES"))
            fprintf(stderr, "zd device walk + descriptors: %.2f ms (walk %.2f)\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw0).count(), t_walk);
          return 0;
        }
      }
    }
    if (F)
      if (int r = dev_walk_download(B, s, &fr, &bl)) return r;
    struct Chain {                                   // one range's frames
      const HostFrame* p; size_t n;
      size_t size() const { return n; }
      const HostFrame& operator[](size_t i) const { return p[i]; }
    };
    // the walk's results stay in the pinned buffers unless a tail walk (which
    // reuses them) is needed: then they move to host vectors first
    std::vector<WalkRange> wr_keep;
    std::vector<HostFrame> fr_keep;
    std::vector<HostBlock> bl_keep;
    const WalkRange* wr = B.h_wr;
    auto chain = [&](size_t k) { return Chain{fr + wr[k].f_off, wr[k].nframes}; };
    std::vector<const HostFrame*> kept;
    kept.reserve(F);
    size_t cur = 0;
    for (size_t k = 0; k < T && !status;) {
      const WalkRange& R = wr[k];
      if (k && cur >= cut(k + 1)) { k++; continue; } // the range lies inside a kept frame
      const Chain c = chain(k);
      const size_t i0 = k ? chain_start(c, cur) : 0;
      if (i0 != SIZE_MAX) {
        for (size_t i = i0; i < c.n; i++) kept.push_back(c.p + i);
        status = R.status;
        cur = R.end;
        k++;
        continue;
      }
      // the chains do not meet: walk on from cur one range at a time on the
      // device (frames that start before the range's end), until the chain
      // reaches a frame start of a later range's chain (plan_index's rule)
      const auto tt = std::chrono::steady_clock::now();
      if (wr_keep.empty()) {
        wr_keep.assign(B.h_wr, B.h_wr + T);
        fr_keep.assign(fr, fr + F);
        bl_keep.assign(bl, bl + NB);
        wr = wr_keep.data(); fr = fr_keep.data(); bl = bl_keep.data();
      }
      parts_from(kept, bl, keep);                    // (kept may point into the pinned copy: same bytes)
      kept.clear();
      size_t kk = k;
      for (;;) {
        uint64_t F2 = 0, NB2 = 0;
        const HostFrame* fr2 = nullptr;
        const HostBlock* bl2 = nullptr;
        const uint64_t hi = std::max<uint64_t>(cut(kk + 1), cur + 1);
        if (int r = dev_walk(B, d_src, n, cur, hi - cur, 1, s, &F2, &NB2, &fr2, &bl2)) return r;
        std::vector<const HostFrame*> t2;
        for (uint64_t i = 0; i < F2; i++) t2.push_back(fr2 + i);
        parts_from(t2, bl2, keep);
        status = B.h_wr[0].status;
        serial_dev += B.h_wr[0].end - cur;
        cur = B.h_wr[0].end;
        if (status || !F2 || cur >= n) break;
        while (kk + 1 < T && cur >= cut(kk + 1)) kk++;
        if (kk > k && chain_start(chain(kk), cur) != SIZE_MAX) break;
      }
      t_tail += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tt).count();
      k = (kk > k && !status && cur < n) ? kk : T;
    }
    parts_from(kept, bl, keep);
  }
  P->set_parts(std::move(keep));
  if (getenv("ZD_PLAN_TIMES"))
    fprintf(stderr, "zd device walk: %.2f ms (kernels + index download %.2f, serial tail %.2f)\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw0).count(), t_walk, t_tail);
  P->index_status = status;
  P->info.walk_serial_bytes = serial_dev;
  P->index_stop = P->nframes;
  return 0;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
// Diagnostics (ZD_PLAN_DUMP=path): the plan's descriptor arrays, for
// comparing planner revisions byte for byte.
static void dump_plan_desc(const zd_plan* P) {
  const char* path = getenv("ZD_PLAN_DUMP");
  if (!path) return;
  FILE* f = fopen(path, "wb");
  if (!f) return;
  auto w = [&](const void* p, size_t bytes) { uint64_t b = bytes; fwrite(&b, 8, 1, f); if (bytes) fwrite(p, 1, bytes, f); };
  const Workspace& W = P->W;
  std::vector<uint8_t> dev_head;               // a device-built plan's descriptors, read back
  if (P->dev_built) {
    dev_head.resize(P->desc_bytes);
    if (P->desc_bytes && hipMemcpy(dev_head.data(), P->d_ws, P->desc_bytes, hipMemcpyDeviceToHost) != hipSuccess)
      (void)hipGetLastError();
  }
  auto at = [&](uint64_t off, const void* vec) -> const void* {
    if (P->dev_built) return (const void*)(dev_head.data() + off);
    return P->staged ? (const void*)(host_stage().p + off) : vec;
  };
  w(at(W.comp, P->comps.data()), P->n_comps * sizeof(CompBlock));
  w(at(W.blocks, P->blocks.data()), P->n_blocks * sizeof(BlockRec));
  w(at(W.frames, P->fdesc.data()), P->n_frames * sizeof(FrameDesc));
  w(at(W.frame_state0, P->fstate0.data()), P->n_frames * sizeof(FrameState));
  w(at(W.list_tables, P->list_tables.data()), P->n_tables * 4);
  w(at(W.list_huf, P->list_huf.data()), P->n_huf * 4);
  w(at(W.list_seq, P->list_seq.data()), P->n_seq * 4);
  w(at(W.list_k4f, P->list_k4f.data()), P->n_k4f * 4);
  w(at(W.copies, P->copies.data()), P->n_copies * sizeof(CopyDesc));
  w(at(W.jframes, P->jframes.data()), P->n_jframes * sizeof(JFrame));
  w(at(W.jblkd, P->jblkd.data()), P->n_jblk * sizeof(JBlkDesc));
  w(at(W.jsegd, P->jsegd.data()), P->n_jseg * sizeof(JSegDesc));
  w(P->frame_out.data(), P->frame_out.size() * 8);
  zd_plan_info I = P->info; I.workspace_bytes = 0; I.host_ns = I.device_ns = 0; I.walk_serial_bytes = 0;
  I.device_descriptors = 0;
  w(&I, sizeof I);
  uint64_t x[4] = {P->j_bytes, P->j_pieces, P->j_rounds, (uint64_t)(int64_t)P->index_status};
  w(x, sizeof x);
  fclose(f);
}

extern "C" {

int zd_abi_version(void) { return ZD_ABI_VERSION; }

int zd_route(uint32_t cus, uint64_t nframes, uint64_t n_tables, uint64_t n_seq_blocks, uint64_t n_huf_blocks,
             int single_block_frames, uint32_t flags, uint32_t* route) {
  if (!route || !cus) return ZD_E_INVALID_ARG;
  RouteIn in{};
  in.cus = cus; in.nframes = nframes; in.n_tables = n_tables; in.n_seq = n_seq_blocks; in.n_huf = n_huf_blocks;
  in.single_block_frames = single_block_frames != 0;
  in.flags = flags;
  const Route r = route_plan(in);
  *route = (r.fused ? ZD_ROUTE_FUSED : 0u) | (r.k4f ? ZD_ROUTE_K4F : 0u) | (r.k1_seq_waves ? ZD_ROUTE_K1_SEQ_WAVES : 0u) |
           (r.fork ? ZD_ROUTE_FORK : 0u) | (r.k1_fork ? ZD_ROUTE_K1_FORK : 0u);
  return ZD_OK;
}

void zd_trim_cache(void) { ws_trim(-1); }

const char* zd_status_name(int s) {
  switch (s) {
    case ZD_OK: return "Ok";
    case ZD_E_NOT_ENOUGH_BYTES: return "NotEnoughBytes";
    case ZD_E_NOT_ENOUGH_BITS: return "NotEnoughBits";
    case ZD_E_MAX_READABLE_BITS_EXCEEDED: return "MaximumReadableBitsExceeded";
    case ZD_E_EMPTY_INPUT_DATA: return "EmptyInputData";
    case ZD_E_NULL_BYTE: return "NullByte";
    case ZD_E_EMPTY_SLICE: return "EmptySliceError";
    case ZD_E_LARGE_ACCURACY_LOG: return "LargeAccuracyLog";
    case ZD_E_CORRUPTED_TABLE: return "CorruptedTable";
    case ZD_E_SEQUENCE_CODE_MAX_EXCEEDED: return "SequenceCodeMaxValueExceeded";
    case ZD_E_HUFFMAN_DECODER_MISSING: return "HuffmanDecoderMissing";
    case ZD_E_CORRUPTED_STREAMS_SIZE: return "CorruptedStreamsSizeTooBig";
    case ZD_E_SEQ_RESERVED_SET: return "ReservedSet(sequences)";
    case ZD_E_NO_PREVIOUS_DECODER: return "NoPreviousDecoder";
    case ZD_E_CTX_WINDOW_SIZE_TOO_BIG: return "WindowSizeTooBig(context)";
    case ZD_E_NULL_OFFSET: return "NullOffsetError";
    case ZD_E_IMPOSSIBLE_VALUE: return "ImpossibleValue";
    case ZD_E_RESERVED_BLOCK_TYPE: return "ReservedBlockType";
    case ZD_E_UNRECOGNIZED_MAGIC: return "UnrecognizedMagic";
    case ZD_E_FRAME_RESERVED_SET: return "ReservedSet(frame)";
    case ZD_E_MISSING_CHECKSUM: return "MissingChecksum";
    case ZD_E_WINDOW_SIZE_TOO_BIG: return "WindowSizeTooBig";
    case ZD_E_REF_PANIC: return "ReferencePanic";
    case ZD_E_OUT_OF_DOMAIN: return "OutOfDomain";
    case ZD_E_DST_TOO_SMALL: return "DstTooSmall";
    case ZD_E_INVALID_ARG: return "InvalidArgument";
    case ZD_E_HIP: return "HipError";
    case ZD_E_NO_MEMORY: return "NoMemory";
    case ZD_E_NOT_DECODED: return "NotDecoded";
    case ZD_E_COMM: return "CommError";
    default: return "Unknown";
  }
}

int zd_frames_index(const uint8_t* src, size_t n, zd_frame_desc* frames, size_t cap_frames, size_t* nframes,
                    zd_block_desc* blocks, size_t cap_blocks, size_t* nblocks, size_t* consumed) {
  if (!src && n) return ZD_E_INVALID_ARG;
  zd_plan W;                                     // the host walk only (no device state)
  if (frames && cap_frames && cap_frames <= FRAMES_INDEX_SERIAL_MAX) {
    // a few frames asked for: walk only those (serially), not the whole input
    HostPart hp;
    Bytes in{src, n};
    for (size_t f = 0; f <= cap_frames && in.n; f++) {
      HostFrame hf;
      VecSink sink{hp.blocks};
      const int r = index_frame(src, in, &hf, sink);
      hp.frames.push_back(hf);
      if (r) break;
    }
    std::vector<HostPart> v;
    v.push_back(std::move(hp));
    W.set_parts(std::move(v));
  } else {
    plan_index(&W, src, n);
  }
  size_t nf = 0, nb = 0;
  int status = 0;
  size_t stop = n;
  for (const HostPart& hp : W.parts) {
    for (const HostFrame& hf : hp.frames) {
      if (frames && cap_frames && nf >= cap_frames) { stop = (size_t)hf.d.src_offset; goto done; }
      if (hf.status) { status = hf.status; stop = (size_t)hf.d.src_offset; goto done; }
      if (frames && nf < cap_frames) {
        frames[nf] = hf.d;
        frames[nf].first_block = (uint32_t)nb;
        frames[nf].num_blocks = hf.nb;
      }
      for (uint32_t k = 0; k < hf.nb; k++) {
        const HostBlock& b = hp.blocks[hf.b0 + k];
        if (blocks && nb < cap_blocks) {
          zd_block_desc& d = blocks[nb];
          d.src_offset = b.src; d.block_size = b.size; d.type = b.type == 4 ? 0 : b.type;
          d.last = b.last; d.rle_byte = b.rle; d._pad = 0;
        }
        nb++;
      }
      nf++;
    }
  }
done:
  if (nframes) *nframes = nf;
  if (nblocks) *nblocks = nb;
  if (consumed) *consumed = stop;
  return status;
}

}  // extern "C"

int zd::frame_spans(const uint8_t* src, size_t n, std::vector<uint64_t>& off, std::vector<uint64_t>& size,
                    size_t* consumed) {
  zd_plan W;
  plan_index(&W, src, n);
  off.clear();
  size.clear();
  off.reserve(W.nframes);
  size.reserve(W.nframes);
  size_t stop = n;
  int status = 0;
  for (const HostPart& hp : W.parts) {
    for (const HostFrame& hf : hp.frames) {
      if (hf.status) { status = hf.status; stop = (size_t)hf.d.src_offset; goto done; }
      off.push_back(hf.d.src_offset);
      size.push_back(hf.d.src_size);
    }
  }
done:
  if (consumed) *consumed = stop;
  return status;
}

extern "C" {

// zd_plan_create / zd_plan_create_device: the walk (host or device), then
// the descriptors, the workspace and the upload.
static int plan_create(const uint8_t* src, const uint8_t* d_src, size_t n, uint32_t flags, hipStream_t s,
                       zd_plan** out, uint64_t cap0) {
  zd_plan* P = new (std::nothrow) zd_plan();
  if (!P) return ZD_E_NO_MEMORY;
  P->flags = flags;
  P->cap0 = cap0;
  const auto t0 = std::chrono::steady_clock::now();
  if (d_src) {
    if (int r = plan_index_dev(P, d_src, n, s)) { zd_plan_destroy(P); return r; }
  } else {
    plan_index(P, src, n);
  }
  const auto ti = std::chrono::steady_clock::now();
  int32_t none[3] = {-1, -1, -1};
  uint64_t rep0[3] = {1, 4, 8};
  if (!P->dev_built)
    if (int r = build_plan(P, -1, none, 0, rep0, 0, true)) { zd_plan_destroy(P); return r; }
  P->info.src_bytes = n;
  const auto t1 = std::chrono::steady_clock::now();
  dump_plan_desc(P);
  if (getenv("ZD_PLAN_TIMES"))
    fprintf(stderr, "zd plan: index %.2f ms, descriptors %.2f ms\n",
            std::chrono::duration<double, std::milli>(ti - t0).count(),
            std::chrono::duration<double, std::milli>(t1 - ti).count());
  int r = P->dev_built ? upload_staging(P) : upload_plan(P);
  const auto tu = std::chrono::steady_clock::now();
  // the second stream and its events (K2 beside K3) exist
  // from here on, so zd_decode_async creates nothing
  if (!r && !aux_take(P)) r = ZD_E_HIP;
  if (r) { zd_plan_destroy(P); return r; }
  const auto t2 = std::chrono::steady_clock::now();
  if (getenv("ZD_PLAN_TIMES"))
    fprintf(stderr, "zd plan: workspace + upload %.2f ms, streams %.2f ms\n",
            std::chrono::duration<double, std::milli>(tu - t1).count(),
            std::chrono::duration<double, std::milli>(t2 - tu).count());
  P->info.host_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
  P->info.device_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
  *out = P;
  return ZD_OK;
}

int zd_plan_create(const uint8_t* src, size_t n, uint32_t flags, zd_plan** out) {
  if (!out || (!src && n)) return ZD_E_INVALID_ARG;
  return plan_create(src, nullptr, n, flags, nullptr, out, 0);
}

int zd_plan_create_device(const uint8_t* d_src, size_t n, uint32_t flags, void* stream, zd_plan** out) {
  if (!out || (!d_src && n)) return ZD_E_INVALID_ARG;
  static const uint8_t none = 0;
  return plan_create(nullptr, d_src ? d_src : &none, n, flags, (hipStream_t)stream, out, 0);
}

int zd_plan_info_get(const zd_plan* P, zd_plan_info* info) {
  if (!P || !info) return ZD_E_INVALID_ARG;
  *info = P->info;
  return ZD_OK;
}

void zd_plan_destroy(zd_plan* P) {
  if (!P) return;
  // the workspace and the second stream go back to process caches: work the
  // plan launched must be done with them first (hipFree used to imply that)
  if (P->launched) {
    (void)hipStreamSynchronize(P->last_stream);
    if (P->aux) (void)hipStreamSynchronize(P->aux);
  }
  ws_release(P->d_ws, P->ws_bytes, P->dev);
  if (P->d_staging) (void)hipFree(P->d_staging);
  if (P->d_meta) (void)hipFree(P->d_meta);
  if (P->io_src) (void)hipFree(P->io_src);
  if (P->io_dst) (void)hipFree(P->io_dst);
  if (P->ev_made) {
    for (auto& e : P->ev) (void)hipEventDestroy(e);
    for (auto& e : P->dom_ev) (void)hipEventDestroy(e);
  }
  aux_give(P);
  delete P;
}

int zd_plan_set_profiling(zd_plan* P, int enable) {
  if (!P || enable < 0 || enable > 2) return ZD_E_INVALID_ARG;
  if (enable && !P->ev_made) {
    for (auto& e : P->ev) HIPCHK(hipEventCreate(&e));
    for (auto& e : P->dom_ev) HIPCHK(hipEventCreate(&e));
    P->ev_made = true;
  }
  P->profile = enable == 1;
  P->profile_dom = enable == 2;
  return ZD_OK;
}

int zd_plan_kernel_times(zd_plan* P, const char** names, float* ms, int cap, int* n) {
  if (!P || !P->launched || !(P->profile || P->profile_dom)) return ZD_E_INVALID_ARG;
  if (P->profile_dom) {
    int k = 0;
    for (int g = 0; g < N_DOM && k < cap; g++) {
      if (!(P->dom_used >> g & 1)) continue;
      HIPCHK(hipEventSynchronize(P->dom_ev[2 * g + 1]));
      float t = 0;
      HIPCHK(hipEventElapsedTime(&t, P->dom_ev[2 * g], P->dom_ev[2 * g + 1]));
      if (names) names[k] = kDomNames[g];
      if (ms) ms[k] = t;
      k++;
    }
    if (n) *n = k;
    return ZD_OK;
  }
  HIPCHK(hipEventSynchronize(P->ev[N_KERNELS]));
  int k = 0;
  for (; k < N_KERNELS && k < cap; k++) {
    if (names) names[k] = kKernelNames[k];
    float t = 0;
    HIPCHK(hipEventElapsedTime(&t, P->ev[k], P->ev[k + 1]));
    if (ms) ms[k] = t;
  }
  if (n) *n = k;
  return ZD_OK;
}

int zd_decode_async(zd_plan* P, const uint8_t* d_src, uint8_t* d_dst, size_t dst_cap, void* stream) {
  if (!P) return ZD_E_INVALID_ARG;
  // out_bytes bounds the output in both layouts (the staging layout is
  // compacted into d_dst by zd_plan_results)
  if (dst_cap < P->info.out_bytes) return ZD_E_DST_TOO_SMALL;
  hipStream_t s = (hipStream_t)stream;
  // frame and block states are reset every launch (keys, lengths, repeat
  // offsets, flags) from device-resident copies: no host memory is read, so
  // a graph captured around this call replays the reset
  // (one launch, zd_k_reset: frame states, block states, K1's tree list and
  // deep pool counters, K4J's round counters and done flags; ZD_RESET_COPIES
  // builds keep the six copy / fill launches it replaced)
#ifndef ZD_RESET_COPIES
  HIPCHK(launch_reset(P->d_ws, P->W, P->n_frames, P->n_comps, P->n_jframes != 0, P->j_pieces, s));
#else
  HIPCHK(hipMemcpyAsync(P->d_ws + P->W.frame_state, P->d_ws + P->W.frame_state0,
                        P->n_frames * sizeof(FrameState), hipMemcpyDeviceToDevice, s));
  HIPCHK(hipMemsetAsync(P->d_ws + P->W.comp_state, 0, std::max<uint64_t>(P->n_comps, 1) * sizeof(CompState), s));
  HIPCHK(hipMemsetAsync(P->d_ws + P->W.huge, 0, 4, s));
  HIPCHK(hipMemsetAsync(P->d_ws + P->W.deep, 0, 4, s));
  if (P->n_jframes) {
    HIPCHK(hipMemsetAsync(P->d_ws + P->W.jpend, 0, 4 * (J_MAX_ROUNDS + 1), s));
    HIPCHK(hipMemsetAsync(P->d_ws + P->W.jdone, 0, std::max<uint64_t>(P->j_pieces, 1), s));
  }
#endif
  LaunchArgs a{};
  a.src = d_src;
  a.src_size = P->info.src_bytes;
  a.out = P->info.out_exact ? d_dst : P->d_staging;
  a.ws = P->d_ws;
  a.W = P->W;
  a.n_tables = (uint32_t)P->n_tables;
  a.n_huf = (uint32_t)P->n_huf;
  a.n_seq = (uint32_t)P->n_seq;
  a.n_frames = (uint32_t)P->n_frames;
  a.n_k4f = (uint32_t)P->n_k4f;
  a.n_copies = (uint32_t)P->n_copies;
  a.n_jframes = (uint32_t)P->n_jframes;
  a.n_k0only = (uint32_t)P->n_k0only;
  a.n_jblk = (uint32_t)P->n_jblk;
  a.n_jseg = (uint32_t)P->n_jseg;
  // ZD_F_J_ONE_ROUND (a test switch, set per plan) cuts the rounds to one
  // of one hop: the path that re-plans a frame whose pointer jumping did not
  // converge, on the streaming executor
  const bool one_round = (P->flags & ZD_F_J_ONE_ROUND) != 0;
  a.j_rounds = one_round && P->j_rounds ? 1u : P->j_rounds;
  a.j_pieces = P->j_pieces;
  // hops per pending word and K4J round (c3s, scripts/exp_jhops.sh, K4J ms
  // with the word-per-lane rounds, round 5: 4 hops 1.91, 5 1.85, 6 1.75-1.77,
  // 7 1.76, 8 1.78-1.79, 12 1.85, 16 1.90); ZD_J_HOPS overrides
  static const char* hops_env = getenv("ZD_J_HOPS");
  a.j_hops = one_round ? 1u : hops_env ? (uint32_t)std::max(1, atoi(hops_env)) : 6u;
  // the sweeps after round 1 (c3s, round 6: 4 / 6 / 8 / 12 hops 3.19 /
  // 3.09 / 3.08 / 3.06 ms a step, profiles/r6_graph_replay_ab.txt); ZD_J_HOPS2 overrides
  static const char* hops2_env = getenv("ZD_J_HOPS2");
  a.j_hops2 = one_round ? 1u : hops2_env ? (uint32_t)std::max(1, atoi(hops2_env)) : 12u;
  a.cus = (uint32_t)(k3_slots() / 64);
  a.stream = s;
  // K3 as four lanes per block (K3Q, default): C3 (763 blocks) 2.89 -> 2.31
  // ms, a forked 8,192-block plan 4.24 -> 2.48, full C4 13.88 -> 13.80; the
  // plan flag ZD_F_SEQ_ONE_LANE keeps the one-lane chain (same records)
  a.k3_quad = !(P->flags & ZD_F_SEQ_ONE_LANE);
  a.events = P->profile ? P->ev : nullptr;
  // routing (route_plan): K2 beside K3 on a second stream, K1's halves on
  // the two streams, K1's sequence half one wave per block
  RouteIn in{};
  in.cus = (uint32_t)(k3_slots() / 64);
  in.nframes = P->n_frames; in.n_tables = P->n_tables; in.n_seq = P->n_seq; in.n_huf = P->n_huf;
  in.flags = P->flags;
  const Route r = route_plan(in);
  const RouteEnv& E = route_env();
  // (a forced fused plan past FUSE_MAX_PER_CU frames per CU: K2 before it, its
  // workgroups could not find room beside the fused ones)
  const bool big_fused = P->fused && P->n_frames > FUSE_MAX_PER_CU * (uint64_t)in.cus;
  const bool fork = E.fork >= 0 ? E.fork == 1 && !big_fused : r.fork && !big_fused;
  if (fork) { a.aux = P->aux; a.fork = P->fork; a.join = P->join; }
  if (!fork && !P->profile && (E.k1fork >= 0 ? E.k1fork == 1 && P->n_huf && P->n_seq : r.k1_fork)) {
    a.aux = P->aux; a.fork = P->fork; a.join = P->join;
    a.k1_fork = true;
  }
  a.k1_seq_waves = E.k1w_max >= 0 ? P->n_tables <= (uint64_t)E.k1w_max && !(P->flags & ZD_F_K1_LANES) : r.k1_seq_waves;
  a.k3_lat = E.k3l >= 0 ? E.k3l == 1 && !(P->flags & (ZD_F_SEQ_ONE_LANE | ZD_F_SEQ_NO_LATENCY)) : r.k3_lat;
  P->last_fused = P->fused && !P->profile;
  if (P->last_fused) {
    a.fused = true;
    HIPCHK(hipMemsetAsync(P->d_ws + P->W.redo, 0, std::max<uint64_t>(P->n_frames, 1), s));
    HIPCHK(hipMemsetAsync(P->d_ws + P->W.k2done, 0, 4, s));
  }
  if (P->profile_dom) {
    a.dom_events = P->dom_ev;
    P->dom_used = 0;
    a.dom_used = &P->dom_used;
  }
  HIPCHK(launch_pipeline(a));
  P->launched = true;
  P->last_stream = s;
  return ZD_OK;
}

int zd_plan_results(zd_plan* P, uint8_t* d_dst, void* stream, int32_t* frame_status, uint64_t* frame_len,
                    uint64_t* total_len, int32_t* first_error_frame) {
  if (!P || !P->launched) return ZD_E_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipStreamSynchronize(s));
  size_t nf = P->n_frames;
  std::vector<FrameState> st(nf);
  if (nf) HIPCHK(hipMemcpy(st.data(), P->d_ws + P->W.frame_state, nf * sizeof(FrameState), hipMemcpyDeviceToHost));
  int first = -1;
  int overall = 0;
  uint64_t total = 0;
  P->limit_frame = -1;
  P->limit_stage = 0;
  P->info.error_key = KEY_NONE;
  std::vector<uint64_t> from, to, len;
  bool need_compact = !P->info.out_exact;
  for (size_t f = 0; f < nf; f++) {
    int code = key_code(st[f].key);
    uint64_t l = st[f].out_len;
    if (first >= 0) code = ZD_E_NOT_DECODED;
    if (frame_status) frame_status[f] = code;
    if (frame_len) frame_len[f] = code ? 0 : l;
    if (code && first < 0) {
      first = (int)f;
      overall = code;
      const uint64_t k = st[f].key;
      P->info.error_key = k;
      if (code == ZD_E_OUT_OF_DOMAIN && key_phase(k) == PH_LIMIT &&
          (key_stage(k) == LS_CAPACITY || key_stage(k) == LS_JROUNDS)) {
        P->limit_frame = (int64_t)f;
        P->limit_stage = key_stage(k);
      }
      if (code == ZD_E_OUT_OF_DOMAIN && key_phase(k) == PH_DECODE && key_stage(k) == DS_LITERALS &&
          ((k >> 8) & 0xFFFFF) == DS_LIT_OVERFLOW_SUB) {
        P->limit_frame = (int64_t)f;
        P->limit_stage = LS_CAPACITY;          // a re-plan gives its blocks room for every literal
      }
    }
    if (first < 0) {
      if (P->info.out_exact && l != P->frame_cap[f]) need_compact = true;
      from.push_back(P->frame_out[f]);
      to.push_back(total);
      len.push_back(l);
      total += l;
    }
  }
  if (need_compact && !from.empty()) {
    // exact layout but a frame came out shorter than its FCS: move through a staging copy
    const uint8_t* stage = P->d_staging;
    if (P->info.out_exact) {
      // the plan's staging buffer, made on the first such call and kept
      if (!P->d_staging) {
        P->staging_bytes = P->info.out_bytes;
        HIPCHK(hipMalloc(&P->d_staging, std::max<uint64_t>(P->staging_bytes, 16)));
      }
      HIPCHK(hipMemcpyAsync(P->d_staging, d_dst, P->info.out_bytes, hipMemcpyDeviceToDevice, s));
      stage = P->d_staging;
    }
    size_t m = from.size();
    if (!grow_dev(P->d_meta, P->meta_cap, 3 * m)) return ZD_E_HIP;
    uint64_t* d_meta = P->d_meta;
    HIPCHK(hipMemcpy(d_meta, from.data(), m * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_meta + m, to.data(), m * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_meta + 2 * m, len.data(), m * 8, hipMemcpyHostToDevice));
    HIPCHK(launch_compact(stage, d_dst, d_meta, d_meta + m, d_meta + 2 * m, (uint32_t)m, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  if (first < 0 && P->index_status) { first = (int)nf; overall = P->index_status; }
  // frames zd_k_fused handed to its redo pass (a fast-chain reject, or a wait
  // past its bound: a slowdown, never a different output)
  P->info.fused_redo_frames = 0;
  if (P->last_fused && nf) {
    std::vector<uint8_t> redo(nf);
    HIPCHK(hipMemcpy(redo.data(), P->d_ws + P->W.redo, nf, hipMemcpyDeviceToHost));
    for (uint8_t r : redo) P->info.fused_redo_frames += r != 0;
  }
  P->res_off = to;
  P->res_len = len;
  if (total_len) *total_len = total;
  if (first_error_frame) *first_error_frame = first;
  return overall;
}

int zd_plan_checksums(zd_plan* P, const uint8_t* d_dst, void* stream, int32_t* ok, uint64_t* hash) {
  if (!P || !P->launched) return ZD_E_INVALID_ARG;
  hipStream_t s = (hipStream_t)stream;
  const size_t nf = P->n_frames, m = P->res_off.size();   // frames 0..m-1 were decoded
  std::vector<uint64_t> h(m, 0);
  if (m) {
    if (!grow_dev(P->d_meta, P->meta_cap, 3 * m)) return ZD_E_HIP;
    uint64_t* d = P->d_meta;
    hipError_t e = hipMemcpy(d, P->res_off.data(), m * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + m, P->res_len.data(), m * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_xxh64(d_dst, d, d + m, (uint32_t)m, d + 2 * m, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) e = hipMemcpy(h.data(), d + 2 * m, m * 8, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return ZD_E_HIP;
  }
  if (!P->frames_ready()) return ZD_E_HIP;
  for (size_t f = 0; f < nf; f++) {
    const zd_frame_desc& d = P->frame(f).d;
    const bool have = f < m && d.kind == ZD_FRAME_ZSTD && d.has_checksum;
    if (ok) ok[f] = have ? ((uint32_t)h[f] == d.checksum ? 1 : 0) : -1;
    if (hash) hash[f] = f < m ? h[f] : 0;
  }
  return ZD_OK;
}

}  // extern "C"

namespace {

// Makes o hold `need` bytes, keeping its first `keep`.  When o.p is the
// caller's own allocation (*o.own) it grows by half at least; when o.p is a
// buffer the caller lent (rank 0's gather buffer in zd_decode_sharded) the
// kept allocation *o.own is reused if it holds `need`, else replaced by one of
// `need` bytes (half again over its old size at most) -- never sized from the
// lent buffer.
int devout_reserve(DevOut& o, uint64_t need, uint64_t keep, hipStream_t s) {
  if (need <= o.cap) return 0;
  const bool lent = o.p != *o.own;
  if (lent && *o.own && *o.own_cap >= need) {
    if (keep) HIPCHK(hipMemcpyAsync(*o.own, o.p, keep, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    o.p = *o.own;
    o.cap = *o.own_cap;
    return 0;
  }
  const uint64_t base = lent ? (*o.own ? *o.own_cap : 0) : o.cap;
  const uint64_t want = std::max<uint64_t>(need, base + base / 2);
  uint8_t* q = nullptr;
  if (hipMalloc(&q, want) != hipSuccess) {
    (void)hipGetLastError();
    ws_trim(-1);
    HIPCHK(hipMalloc(&q, want));
  }
  if (keep) HIPCHK(hipMemcpyAsync(q, o.p, keep, hipMemcpyDeviceToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  if (*o.own) (void)hipFree(*o.own);        // the old kept allocation (o.p or unused)
  *o.own = q;
  *o.own_cap = want;
  o.p = q;
  o.cap = want;
  return 0;
}

bool call_failed(int st) { return st == ZD_E_HIP || st == ZD_E_INVALID_ARG || st == ZD_E_DST_TOO_SMALL; }

}  // namespace

// Re-plans past a frame that reached a limit the host can lift: a frame that
// decodes past the capacity its plan reserved (its Frame_Content_Size, or
// 128 KiB per block -- the reference checks neither, decoding_context.rs:
// 29-47, block.rs:50) is planned again from its own start with four times the
// capacity (K4_MAX_FRAME_OUT at most); a K4J frame whose pointer jumping did
// not converge is planned again on the streaming executor.  Each re-plan
// covers the input from that frame on (the same resident input, from that
// frame's offset); its output follows the frames before in `out`.
constexpr int LIMIT_RETRIES = 12;

int zd::decode_resident(zd_plan* P, const uint8_t* src, size_t n, const uint8_t* d_src, DevOut& out, void* stream,
                        uint64_t* total_out, int64_t* first_out, uint64_t* replans, FrameOuts* fo) {
  const hipStream_t s = (hipStream_t)stream;
  *total_out = 0;
  *first_out = -1;
  const uint64_t ob = std::max<uint64_t>(P->info.out_bytes, 16);
  if (int r = devout_reserve(out, ob, 0, s)) return r;
  int st = zd_decode_async(P, d_src, out.p, out.cap, s);
  if (st) return st;
  uint64_t produced = 0;
  int32_t first = -1;
  // per-frame outcomes: the current plan's, written into fo from frame fbase on
  std::vector<int32_t> fs;
  std::vector<uint64_t> fl;
  auto want = [&](zd_plan* Q) {
    if (!fo) return;
    fs.assign(Q->n_frames, 0);
    fl.assign(Q->n_frames, 0);
  };
  auto keep = [&](zd_plan* Q, int64_t fb, uint64_t at) {
    if (!fo) return;
    uint64_t o = at;
    for (size_t f = 0; f < Q->n_frames && fb + (int64_t)f < (int64_t)fo->status.size(); f++) {
      fo->status[fb + f] = fs[f];
      fo->off[fb + f] = o;
      fo->len[fb + f] = fl[f];
      o += fl[f];
    }
  };
  if (fo) {
    fo->status.assign(P->n_frames, ZD_E_NOT_DECODED);
    fo->off.assign(P->n_frames, 0);
    fo->len.assign(P->n_frames, 0);
  }
  want(P);
  st = zd_plan_results(P, out.p, s, fo ? fs.data() : nullptr, fo ? fl.data() : nullptr, &produced, &first);
  if (call_failed(st)) return st;
  keep(P, 0, 0);
  zd_plan* cur = P;
  size_t base = 0;                                 // cur's input starts at src + base
  int64_t fbase = 0;                               // and its frame 0 is P's frame fbase
  for (int k = 0; k < LIMIT_RETRIES && st == ZD_E_OUT_OF_DOMAIN && cur->limit_frame >= 0; k++) {
    const size_t f = (size_t)cur->limit_frame;
    const uint64_t old_cap = cur->frame_cap[f];
    uint32_t flags = cur->flags;
    uint64_t cap0 = 0;
    if (cur->limit_stage == LS_CAPACITY) {
      // past K4J's 32 GiB, or with K4J forced off the streaming K4's int32
      // positions (plan_frame keys a larger frame out of domain): stop
      const uint64_t lim = k4j_mode_of(flags) == 0 ? K4_MAX_FRAME_OUT : K4J_MAX_FRAME_OUT;
      if (old_cap >= lim) break;
      cap0 = std::min<uint64_t>(lim, std::max<uint64_t>(4 * old_cap, old_cap + (1u << 20)));
    } else {
      flags = (flags & ~ZD_F_BLOCK_PARALLEL) | ZD_F_FRAME_SERIAL;
      cap0 = old_cap;
    }
    if (!cur->frames_ready()) { st = ZD_E_HIP; break; }
    const size_t at = base + (size_t)cur->frame(f).d.src_offset;
    zd_plan* Q = nullptr;
    const int r = plan_create(src + at, nullptr, n - at, flags, nullptr, &Q, cap0);
    if (r) { st = r; break; }
    if (replans) (*replans)++;
    const uint64_t qob = std::max<uint64_t>(Q->info.out_bytes, 16);
    uint64_t t2 = 0;
    int32_t qfirst = -1;
    st = devout_reserve(out, produced + qob, produced, s);
    if (!st) st = zd_decode_async(Q, d_src + at, out.p + produced, qob, s);
    want(Q);
    if (!st) st = zd_plan_results(Q, out.p + produced, s, fo ? fs.data() : nullptr, fo ? fl.data() : nullptr, &t2, &qfirst);
    if (cur != P) zd_plan_destroy(cur);
    cur = Q;
    base = at;
    fbase += (int64_t)f;
    first = qfirst;
    if (call_failed(st)) break;
    keep(Q, fbase, produced);
    produced += t2;
  }
  if (cur != P) {
    P->info.error_key = cur->info.error_key;
    zd_plan_destroy(cur);
  }
  if (call_failed(st)) return st;
  *total_out = produced;
  *first_out = first >= 0 ? fbase + first : -1;
  return st;
}

extern "C" {

int zd_plan_decompress(zd_plan* P, const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
  if (!P || (!src && n) || n != P->info.src_bytes) return ZD_E_INVALID_ARG;
  // device buffers owned by the plan (kept for the next call), the input and
  // output through the pinned ring (chunked, the host copies on the worker
  // pool overlapping the DMA), everything on one stream
  if (!grow_dev(P->io_src, P->io_src_cap, n + ZD_SRC_PADDING)) return ZD_E_HIP;
  const hipStream_t s = nullptr;
  IoEvents ev;
  if (!ev.ok) return ZD_E_HIP;
  const auto t0 = std::chrono::steady_clock::now();
  if (int r = io_h2d(P->io_src, src, n, s, io_ring(), ev.e)) return r;
  const auto t1 = std::chrono::steady_clock::now();
  DevOut o{P->io_dst, P->io_dst_cap, &P->io_dst, &P->io_dst_cap};
  uint64_t produced = 0;
  int64_t first = -1;
  P->info.replans = 0;
  const int st = decode_resident(P, src, n, P->io_src, o, s, &produced, &first, &P->info.replans, &P->io_fo);
  if (call_failed(st)) return st;
  const auto t2 = std::chrono::steady_clock::now();
  const size_t copy = (size_t)std::min<uint64_t>(produced, cap);
  if (copy && dst)
    if (int e = io_d2h(dst, o.p, copy, s, io_ring(), ev.e)) return e;
  const auto t3 = std::chrono::steady_clock::now();
  auto ns = [](auto a, auto b) { return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count(); };
  P->info.io_h2d_ns = ns(t0, t1);
  P->info.io_decode_ns = ns(t1, t2);
  P->info.io_d2h_ns = ns(t2, t3);
  if (out_len) *out_len = (size_t)produced;
  if (!st && produced > cap) return ZD_E_DST_TOO_SMALL;
  return st;
}

int zd_plan_frame_outputs(const zd_plan* P, int32_t* status, uint64_t* offset, uint64_t* length, size_t cap,
                          size_t* n) {
  if (!P) return ZD_E_INVALID_ARG;
  const size_t m = P->io_fo.status.size();
  for (size_t f = 0; f < m && f < cap; f++) {
    if (status) status[f] = P->io_fo.status[f];
    if (offset) offset[f] = P->io_fo.off[f];
    if (length) length[f] = P->io_fo.len[f];
  }
  if (n) *n = m;
  return ZD_OK;
}

int zd_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len, uint32_t flags) {
  zd_plan* P = nullptr;
  int r = zd_plan_create(src, n, flags, &P);
  if (r) return r;
  r = zd_plan_decompress(P, src, n, dst, cap, out_len);
  zd_plan_destroy(P);
  return r;
}

// ===========================================================================
// DecodingContext mirror
// ===========================================================================
}  // extern "C"

struct zd_context {
  uint64_t window = 0;
  uint8_t* d_out = nullptr;     // decoded (capacity d_cap)
  uint64_t d_cap = 0;
  uint64_t len = 0;
  uint64_t rep[3] = {1, 4, 8};
  // persisted tables of the previous blocks (one virtual comp block)
  uint16_t* d_lut = nullptr;    // LUT_ENTRIES
  uint16_t* d_fse = nullptr;    // FSE_SLOT entries
  uint8_t huf_bits = 0;
  uint8_t al[3] = {0, 0, 0};
  bool has_huf = false;
  bool has_tab[3] = {false, false, false};
  // the persisted Huffman table's deep-tree pool (a tree with more leaves
  // than a LUT slot holds keeps its symbols there): the pool's counter and
  // bytes as the plan that built it left them, deep_used bytes
  uint8_t* d_deep = nullptr;
  uint32_t deep_used = 0;
  // kept between calls: the stream every block runs on (one synchronisation
  // per block) and the block-input buffer (grown, never freed per call)
  hipStream_t s = nullptr;
  uint8_t* d_in = nullptr;
  uint64_t in_cap = 0;
};

namespace {

// The caller's bytes in the context's input buffer (async on its stream).
int ctx_input(zd_context* c, const uint8_t* src, size_t n) {
  if (n + ZD_SRC_PADDING > c->in_cap) {
    if (c->d_in) (void)hipFree(c->d_in);
    c->d_in = nullptr;
    c->in_cap = 0;
    const uint64_t nc = std::max<uint64_t>(n + ZD_SRC_PADDING, 256u << 10);
    HIPCHK(hipMalloc(&c->d_in, nc));
    c->in_cap = nc;
  }
  if (n) HIPCHK(hipMemcpyAsync(c->d_in, src, n, hipMemcpyHostToDevice, c->s));
  return 0;
}

int ctx_reserve(zd_context* c, uint64_t need) {
  if (need <= c->d_cap) return 0;
  uint64_t nc = std::max<uint64_t>(c->d_cap ? c->d_cap * 2 : (1 << 20), need);
  uint8_t* nd = nullptr;
  HIPCHK(hipMalloc(&nd, nc));
  if (c->len) HIPCHK(hipMemcpy(nd, c->d_out, c->len, hipMemcpyDeviceToDevice));
  if (c->d_out) (void)hipFree(c->d_out);
  c->d_out = nd;
  c->d_cap = nc;
  return 0;
}

}  // namespace

extern "C" {

int zd_context_new(uint64_t window_size, zd_context** out) {
  if (!out) return ZD_E_INVALID_ARG;
  if (window_size > MAX_WIN_SIZE) return ZD_E_CTX_WINDOW_SIZE_TOO_BIG;   // decoding_context.rs:29-35
  zd_context* c = new (std::nothrow) zd_context();
  if (!c) return ZD_E_NO_MEMORY;
  c->window = window_size;
  if (hipMalloc(&c->d_lut, LUT_ENTRIES * 2) != hipSuccess || hipMalloc(&c->d_fse, FSE_SLOT * 2) != hipSuccess ||
      hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) != hipSuccess) {
    zd_context_free(c);
    return ZD_E_HIP;
  }
  *out = c;
  return ZD_OK;
}

void zd_context_free(zd_context* c) {
  if (!c) return;
  if (c->d_out) (void)hipFree(c->d_out);
  if (c->d_lut) (void)hipFree(c->d_lut);
  if (c->d_fse) (void)hipFree(c->d_fse);
  if (c->d_deep) (void)hipFree(c->d_deep);
  if (c->d_in) (void)hipFree(c->d_in);
  if (c->s) { (void)hipStreamSynchronize(c->s); (void)hipStreamDestroy(c->s); }
  delete c;
}

int zd_context_decoded(const zd_context* c, uint8_t* dst, size_t cap, size_t* len) {
  if (!c) return ZD_E_INVALID_ARG;
  if (len) *len = c->len;
  size_t k = (size_t)std::min<uint64_t>(cap, c->len);
  if (k && dst) HIPCHK(hipMemcpy(dst, c->d_out, k, hipMemcpyDeviceToHost));
  return cap < c->len ? ZD_E_DST_TOO_SMALL : ZD_OK;
}

int zd_context_offsets(const zd_context* c, uint64_t offsets[3]) {
  if (!c || !offsets) return ZD_E_INVALID_ARG;
  for (int i = 0; i < 3; i++) offsets[i] = c->rep[i];
  return ZD_OK;
}

// Runs a one-frame plan whose output continues the context's decoded buffer:
// copies and kernels on the context's stream, one synchronisation (for the
// frame state and the block's table state).
static int ctx_run(zd_context* c, zd_plan* P, const uint8_t* src, size_t n) {
  if (int r = upload_plan(P)) return r;
  if (int r = ctx_input(c, src, n)) return r;
  const hipStream_t s = c->s;
  HIPCHK(hipMemsetAsync(P->d_ws + P->W.comp_state, 0, std::max<size_t>(P->comps.size(), 1) * sizeof(CompState), s));
  HIPCHK(hipMemsetAsync(P->d_ws + P->W.huge, 0, 4, s));
  HIPCHK(hipMemsetAsync(P->d_ws + P->W.deep, 0, 4, s));
  // prebuilt comp 0 carries the context's tables
  CompState pcs{};
  if (P->has_prebuilt) {
    const CompBlock& pb = P->comps[0];
    uint8_t* luts = P->d_ws + P->W.luts + (uint64_t)pb.lut_slot * LUT_ENTRIES * 2;
    uint8_t* fses = P->d_ws + P->W.fses + (uint64_t)pb.fse_slot * FSE_SLOT * 2;
    HIPCHK(hipMemcpyAsync(luts, c->d_lut, LUT_ENTRIES * 2, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(fses, c->d_fse, FSE_SLOT * 2, hipMemcpyDeviceToDevice, s));
    pcs.huf_bits = c->huf_bits;
    for (int k = 0; k < 3; k++) pcs.al[k] = c->al[k];
    HIPCHK(hipMemcpyAsync(P->d_ws + P->W.comp_state, &pcs, sizeof pcs, hipMemcpyHostToDevice, s));
    // a Treeless block reuses the persisted tree: when its symbols live in
    // the deep pool, the pool comes back too, at the offsets the LUT slot's
    // DEEP_POOL_AT word names (its counter included, so nothing new lands on it)
    if (P->comps.size() > 1 && P->comps[1].lit_type == LIT_TREELESS && c->has_huf && c->deep_used)
      HIPCHK(hipMemcpyAsync(P->d_ws + P->W.deep, c->d_deep, 16 + (size_t)c->deep_used, hipMemcpyDeviceToDevice, s));
  }
  P->info.out_exact = 1;    // output goes straight into the context buffer
  P->fdesc[0].out = 0;
  HIPCHK(hipMemcpyAsync(P->d_ws + P->W.frames, P->fdesc.data(), sizeof(FrameDesc), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(P->d_ws + P->W.frame_state, P->fstate0.data(), sizeof(FrameState), hipMemcpyHostToDevice, s));
  LaunchArgs a{};
  a.src = c->d_in; a.src_size = n; a.out = c->d_out; a.ws = P->d_ws; a.W = P->W;
  a.n_tables = (uint32_t)P->list_tables.size();
  a.n_huf = (uint32_t)P->list_huf.size();
  a.n_seq = (uint32_t)P->list_seq.size();
  a.n_frames = 1;
  a.n_k4f = (uint32_t)P->list_k4f.size();
  a.n_copies = (uint32_t)P->copies.size();
  a.stream = s;
  if (launch_pipeline(a) != hipSuccess) return ZD_E_HIP;
  // the frame state and every block's table state in one synchronisation
  const size_t nc = P->comps.size();
  std::vector<CompState> cst(std::max<size_t>(nc, 1));
  FrameState st{};
  uint32_t deep_used = 0;
  HIPCHK(hipMemcpyAsync(&st, P->d_ws + P->W.frame_state, sizeof st, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(&deep_used, P->d_ws + P->W.deep, 4, hipMemcpyDeviceToHost, s));
  if (nc) HIPCHK(hipMemcpyAsync(cst.data(), P->d_ws + P->W.comp_state, nc * sizeof(CompState), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  int code = key_code(st.key);
  if (code) return code;
  c->len = st.out_len;
  for (int i = 0; i < 3; i++) c->rep[i] = st.rep[i];
  // persist tables defined by the real block (comp index 1 when prebuilt, else 0);
  // the device copies stay on the stream, ahead of the next block's work
  size_t ci = P->has_prebuilt ? 1 : 0;
  if (ci < nc) {
    const CompBlock& cb = P->comps[ci];
    const CompState& cs = cst[ci];
    if (cb.lit_type == LIT_COMPRESSED) {
      HIPCHK(hipMemcpyAsync(c->d_lut, P->d_ws + P->W.luts + (uint64_t)cb.lut_slot * LUT_ENTRIES * 2, LUT_ENTRIES * 2,
                            hipMemcpyDeviceToDevice, s));
      c->huf_bits = cs.huf_bits;
      c->has_huf = true;
      c->deep_used = 0;
      if (deep_used) {             // the new tree's symbols are in the plan's pool
        if (!c->d_deep && hipMalloc(&c->d_deep, 16 + (size_t)DEEP_POOL_BYTES) != hipSuccess) {
          c->d_deep = nullptr;
          c->has_huf = false;
          return ZD_E_NO_MEMORY;
        }
        HIPCHK(hipMemcpyAsync(c->d_deep, P->d_ws + P->W.deep, 16 + (size_t)deep_used, hipMemcpyDeviceToDevice, s));
        c->deep_used = deep_used;
      }
    }
    for (int k = 0; k < 3 && cb.nseq; k++) {
      int32_t srcc = cb.tab_src[k];
      if (srcc < 0) continue;
      const CompBlock& sb = P->comps[(size_t)srcc];
      if ((size_t)srcc == ci) {
        HIPCHK(hipMemcpyAsync(c->d_fse + k * FSE_TAB,
                              P->d_ws + P->W.fses + ((uint64_t)sb.fse_slot * FSE_SLOT + k * FSE_TAB) * 2, FSE_TAB * 2,
                              hipMemcpyDeviceToDevice, s));
        c->al[k] = cst[(size_t)srcc].al[k];
      }
      c->has_tab[k] = true;
    }
    // the plan's workspace is released after this call: the copies out of it first
    HIPCHK(hipStreamSynchronize(s));
  }
  return ZD_OK;
}

int zd_block_decode(zd_context* c, const uint8_t* src, size_t n, size_t* consumed, int* last) {
  if (!c || (!src && n)) return ZD_E_INVALID_ARG;
  // Block::parse (block.rs:43-72) on the host side
  Bytes in{src, n};
  const uint8_t* h;
  if (int r = in.slice(3, &h)) return r;
  uint32_t x = h[0] | (h[1] << 8) | ((uint32_t)h[2] << 16);
  HostBlock hb;
  memset(&hb, 0, sizeof hb);
  hb.last = x & 1; hb.type = (x >> 1) & 3; hb.size = x >> 3; hb.src = 3;
  if (hb.type == 0) { const uint8_t* s; if (int r = in.slice(hb.size, &s)) return r; }
  else if (hb.type == 1) { if (int r = in.u8(&hb.rle)) return r; }
  else if (hb.type == 2) {
    const uint8_t* s;
    if (int r = in.slice(hb.size, &s)) return r;
    hb.cb.src = 3; hb.cb.size = hb.size; hb.cb.host_stage = PS_ALL;
    WalkErr e;
    if (int r = parse_compressed(src, 3, hb.size, &hb.cb, &e)) return r;
  } else return ZD_E_RESERVED_BLOCK_TYPE;
  size_t used = n - in.n;
  if (consumed) *consumed = used;
  if (last) *last = hb.last;

  zd_plan P;
  HostPart part;
  HostFrame hf;
  memset(&hf.d, 0, sizeof hf.d);
  hf.d.kind = ZD_FRAME_ZSTD;
  hf.d.content_size = UINT64_MAX;
  int32_t prev_huf = -1, prev_tab[3] = {-1, -1, -1};
  bool need_pre = c->has_huf || c->has_tab[0] || c->has_tab[1] || c->has_tab[2];
  if (need_pre) {
    // virtual previous block: a compressed block that is never decoded
    HostBlock pre;
    memset(&pre, 0, sizeof pre);
    pre.type = 2;
    pre.cb.lit_type = LIT_COMPRESSED;
    pre.cb.host_stage = PS_ALL;
    pre.cb.nseq = 1;
    pre.cb.modes[0] = pre.cb.modes[1] = pre.cb.modes[2] = M_FSE;
    part.blocks.push_back(pre);
    P.has_prebuilt = true;
    if (c->has_huf) prev_huf = 0;
    for (int k = 0; k < 3; k++) if (c->has_tab[k]) prev_tab[k] = 0;
  }
  part.blocks.push_back(hb);
  hf.nb = (uint32_t)part.blocks.size();
  for (const HostBlock& b : part.blocks) hf.ncomp += b.type == 2;
  part.frames.push_back(hf);
  {
    std::vector<HostPart> one;
    one.push_back(std::move(part));
    P.set_parts(std::move(one));
  }
  // resolve with the prebuilt block as "previous": build_plan walks the blocks in
  // order, so the virtual block seeds Treeless/Repeat through prev_huf/prev_tab.
  uint64_t cap = c->len + (hb.type == 2 ? (uint64_t)MAX_BLOCK_OUT : (uint64_t)hb.size);
  if (int r = ctx_reserve(c, cap + 16)) return r;
  uint64_t rep0[3] = {c->rep[0], c->rep[1], c->rep[2]};
  build_plan(&P, prev_huf, prev_tab, c->len, rep0, c->d_cap);
  if (P.has_prebuilt) {
    // the virtual block: prebuilt, never executed, tables self-referencing
    CompBlock& pb = P.comps[0];
    pb.prebuilt = 1;
    pb.huf_src = 0;
    for (int k = 0; k < 3; k++) pb.tab_src[k] = 0;
    P.list_tables.erase(std::remove(P.list_tables.begin(), P.list_tables.end(), 0u), P.list_tables.end());
    P.list_huf.erase(std::remove(P.list_huf.begin(), P.list_huf.end(), 0u), P.list_huf.end());
    P.list_seq.erase(std::remove(P.list_seq.begin(), P.list_seq.end(), 0u), P.list_seq.end());
    // the real block resolves Treeless/Repeat against comp 0 (build_plan already
    // chained them through the virtual block's own FSE/Compressed modes)
    P.blocks[0].type = 5;    // skip in execute
    FrameState& fs = P.fstate0[0];
    // build_plan's keys came from the virtual block; keep only a capacity
    // limit (PH_LIMIT: the context past the streaming K4's int32 positions)
    if (fs.key != KEY_NONE && key_phase(fs.key) != PH_LIMIT) fs.key = KEY_NONE;
    // re-derive host decode errors for the real block only
    CompBlock& cb = P.comps[1];
    if (cb.lit_type == LIT_TREELESS && !c->has_huf)
      fs.key = std::min(fs.key, make_key(PH_DECODE, 1, DS_LITERALS, 0, ZD_E_HUFFMAN_DECODER_MISSING));
    if (cb.nseq == 0) {
      int code = ZD_E_EMPTY_INPUT_DATA;
      for (int k = 0; k < 3; k++) if (!c->has_tab[k]) { code = ZD_E_NO_PREVIOUS_DECODER; break; }
      fs.key = std::min(fs.key, make_key(PH_DECODE, 1, DS_SEQUENCES, 0, code));
    } else {
      for (int k = 0; k < 3; k++) {
        if (cb.modes[k] == M_REPEAT) {
          if (!c->has_tab[k]) {
            fs.key = std::min(fs.key, make_key(PH_DECODE, 1, DS_SEQUENCES, 0, ZD_E_NO_PREVIOUS_DECODER));
            cb.tab_src[k] = -1;
            break;
          }
          cb.tab_src[k] = 0;
        }
      }
      bool ok = cb.tab_src[0] >= 0 && cb.tab_src[1] >= 0 && cb.tab_src[2] >= 0;
      P.list_seq.erase(std::remove(P.list_seq.begin(), P.list_seq.end(), 1u), P.list_seq.end());
      if (ok) P.list_seq.push_back(1);
    }
    if (cb.lit_type == LIT_TREELESS) {
      cb.huf_src = c->has_huf ? 0 : -1;
      P.list_huf.erase(std::remove(P.list_huf.begin(), P.list_huf.end(), 1u), P.list_huf.end());
      if (cb.huf_src >= 0 && cb.nstreams) P.list_huf.push_back(1);
    }
  }
  P.info.src_bytes = n;
  int r = ctx_run(c, &P, src, n);
  ws_release(P.d_ws, P.ws_bytes, P.dev);
  P.d_ws = nullptr;
  if (P.d_staging) { (void)hipFree(P.d_staging); P.d_staging = nullptr; }
  return r;
}

int zd_execute_sequences(zd_context* c, const uint32_t* ll, const uint32_t* ofv, const uint32_t* ml, size_t nseq,
                         const uint8_t* lits, size_t nlits) {
  if (!c || (nseq && (!ll || !ofv || !ml)) || (nlits && !lits)) return ZD_E_INVALID_ARG;
  // One synthetic compressed block whose literals are raw (taken from `lits`)
  // and whose sequences are pre-decoded: only the execute kernel runs.
  uint64_t need = c->len + nlits;
  for (size_t i = 0; i < nseq; i++) need += ml[i];
  // the streaming K4's int32 positions bound the context's output
  if (need >= K4_MAX_FRAME_OUT) return ZD_E_OUT_OF_DOMAIN;
  if (int r = ctx_reserve(c, need + 16)) return r;
  zd_plan P;
  HostFrame hf;
  memset(&hf.d, 0, sizeof hf.d);
  hf.d.kind = ZD_FRAME_ZSTD;
  hf.d.content_size = UINT64_MAX;
  HostBlock hb;
  memset(&hb, 0, sizeof hb);
  hb.type = 2; hb.size = (uint32_t)nlits; hb.src = 0; hb.last = 1;
  hb.cb.lit_type = LIT_RAW; hb.cb.lit_regen = (uint32_t)nlits; hb.cb.lit_data = 0;
  hb.cb.nseq = (uint32_t)nseq; hb.cb.host_stage = PS_ALL; hb.cb.seq_direct = 1;
  hb.cb.modes[0] = hb.cb.modes[1] = hb.cb.modes[2] = M_RLE;
  HostPart part;
  part.blocks.push_back(hb);
  hf.nb = 1;
  hf.ncomp = 1;
  part.frames.push_back(hf);
  {
    std::vector<HostPart> one;
    one.push_back(std::move(part));
    P.set_parts(std::move(one));
  }
  int32_t none[3] = {-1, -1, -1};
  uint64_t rep0[3] = {c->rep[0], c->rep[1], c->rep[2]};
  P.flags |= ZD_F_FRAME_SERIAL;         // the streaming K4 (K4J reads no direct records)
  build_plan(&P, -1, none, c->len, rep0, c->d_cap);
  P.list_tables.clear();
  P.list_huf.clear();
  P.list_seq.clear();   // sequences come from the caller
  P.info.src_bytes = nlits;
  // the caller's triples as direct records (zd_common.h): a value past its
  // packed field is an escape with its exact triple in a DirectSide entry
  uint8_t* d_side = nullptr;
  auto fin = [&](int rr) {
    ws_release(P.d_ws, P.ws_bytes, P.dev);
    if (P.d_staging) (void)hipFree(P.d_staging);
    if (d_side) (void)hipFree(d_side);
    P.d_ws = nullptr; P.d_staging = nullptr; d_side = nullptr;
    return rr;
  };
  std::vector<uint64_t> rec(nseq);
  std::vector<DirectSide> side;
  if (nseq) {
    for (size_t i = 0; i < nseq; i++) {
      // K4's literal and offset checks run in 32 bits; a literals_length
      // past every literal the block holds is ImpossibleValue whatever its
      // size (decoding_context.rs:86-90), so it is clamped to nlits + 1:
      // the outcome is the reference's and no batch sum can wrap (nlits and
      // every match length are below K4_MAX_FRAME_OUT < 2^31)
      const uint32_t lli = (uint32_t)std::min<uint64_t>(ll[i], (uint64_t)nlits + 1);
      const bool esc = lli >= 0x1FFFF || ml[i] >= 0x3FFFF || ofv[i] >= DIRECT_GIANT;
      if (esc && side.empty()) side.assign(nseq, DirectSide{});
      if (esc) side[i] = DirectSide{lli, ml[i], ofv[i], 0};
      rec[i] = esc ? DIRECT_ESCAPE : seq_pack(lli, ml[i], ofv[i]);
    }
    if (!side.empty()) {
      if (hipMalloc(&d_side, side.size() * sizeof(DirectSide)) != hipSuccess) { d_side = nullptr; return fin(ZD_E_NO_MEMORY); }
      if (hipMemcpy(d_side, side.data(), side.size() * sizeof(DirectSide), hipMemcpyHostToDevice) != hipSuccess)
        return fin(ZD_E_HIP);
      P.comps[0].seq_side = (uint64_t)(uintptr_t)d_side;
    }
  }
  int r = upload_plan(&P);
  if (r) return fin(r);
  const hipStream_t s = c->s;
  if (int rr = ctx_input(c, lits, nlits)) return fin(rr);
  CompState cs{};
  cs.lit_count = (uint32_t)nlits;
  if (nseq && hipMemcpyAsync(P.d_ws + P.W.seqs, rec.data(), nseq * 8, hipMemcpyHostToDevice, s) != hipSuccess)
    return fin(ZD_E_HIP);
  P.fdesc[0].out = 0;
  if (hipMemcpyAsync(P.d_ws + P.W.comp_state, &cs, sizeof cs, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(P.d_ws + P.W.frames, P.fdesc.data(), sizeof(FrameDesc), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(P.d_ws + P.W.frame_state, P.fstate0.data(), sizeof(FrameState), hipMemcpyHostToDevice, s) != hipSuccess)
    return fin(ZD_E_HIP);
  LaunchArgs a{};
  a.src = c->d_in; a.src_size = nlits; a.out = c->d_out; a.ws = P.d_ws; a.W = P.W;
  a.n_frames = 1;
  a.n_k4f = (uint32_t)P.list_k4f.size();
  a.n_copies = (uint32_t)P.copies.size();
  a.stream = s;
  FrameState st{};
  if (launch_pipeline(a) != hipSuccess ||
      hipMemcpyAsync(&st, P.d_ws + P.W.frame_state, sizeof st, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fin(ZD_E_HIP);
  int code = key_code(st.key);
  if (code) return fin(code);
  c->len = st.out_len;
  for (int i = 0; i < 3; i++) c->rep[i] = st.rep[i];
  return fin(ZD_OK);
}

}  // extern "C"
