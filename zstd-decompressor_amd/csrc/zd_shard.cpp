// zd_shard.cpp — multi-GPU decode over frame ranges on the
// C ABI: the partition of a .zst input into contiguous frame ranges, a
// communicator over RCCL (xGMI on one node), and the gather of every rank's
// decoded range to rank 0.
//
// Frames are independent: each gets a fresh DecodingContext (frame.rs:232-237)
// and the CLI only concatenates frame outputs and stops at the first frame
// that fails (src/main.rs:43-53).  So a rank decodes its frame range on its
// own GPU with no collective on the data path; the only exchange is the
// outcome of every rank (status, first failing frame, length) and the
// point-to-point sends of decoded ranges to rank 0.
//
// RCCL is loaded at zd_comm_create (dlopen of librccl.so.1: the one PyTorch
// already loaded, or ROCm's), so libzd itself loads on hosts without it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/zd.h"
#include "zd_internal.h"
#include "zd_walk.h"

namespace {

// the slice of rccl.h used here (ABI-stable NCCL 2 interface)
typedef struct ncclComm* ncclComm_t;
typedef struct { char internal[ZD_COMM_ID_BYTES]; } ncclUniqueId;
typedef int ncclResult_t;
enum { ncclUint8 = 1, ncclInt64 = 4 };
struct Rccl {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl* rccl() {
  static Rccl R;
  static bool tried = false;
  if (tried) return R.h ? &R : nullptr;
  tried = true;
  const char* names[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
  for (const char* n : names)
    if ((R.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
  if (!R.h) return nullptr;
  bool ok = true;
  auto sym = [&](auto& f, const char* name) {
    f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(R.h, name));
    ok = ok && f;
  };
  sym(R.GetUniqueId, "ncclGetUniqueId");
  sym(R.CommInitRank, "ncclCommInitRank");
  sym(R.CommDestroy, "ncclCommDestroy");
  sym(R.AllGather, "ncclAllGather");
  sym(R.Send, "ncclSend");
  sym(R.Recv, "ncclRecv");
  sym(R.GroupStart, "ncclGroupStart");
  sym(R.GroupEnd, "ncclGroupEnd");
  sym(R.GetErrorString, "ncclGetErrorString");
  if (!ok) R.h = nullptr;
  return R.h ? &R : nullptr;
}

#define NCCLCHK(x) do { ncclResult_t _r = (x); if (_r != 0) { \
  fprintf(stderr, "zd: %s failed: %s\n", #x, R->GetErrorString ? R->GetErrorString(_r) : "?"); return ZD_E_COMM; } } while (0)
#define HIPCHK(x) do { hipError_t _e = (x); if (_e != hipSuccess) { \
  fprintf(stderr, "zd: %s failed: %s\n", #x, hipGetErrorString(_e)); return ZD_E_HIP; } } while (0)

}  // namespace

struct zd_comm {
  ncclComm_t nc = nullptr;
  int world = 0, rank = 0;
  int64_t* d_meta = nullptr;       // world x 4 int64: status, first error frame, length, root capacity
  // zd_decode_sharded's device buffers, grown as needed and kept between calls
  uint8_t* d_src = nullptr;
  uint64_t src_cap = 0;
  uint8_t* d_out = nullptr;
  uint64_t out_cap = 0;
};

namespace {

// *p holds at least `need` bytes afterwards (grown by hipMalloc, contents dropped)
bool grow(uint8_t*& p, uint64_t& cap, uint64_t need) {
  if (need <= cap) return true;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  if (hipMalloc(&p, need) != hipSuccess) { (void)hipGetLastError(); return false; }
  cap = need;
  return true;
}

// index_frame's block sink when only the frame walk matters
struct CountSink {
  size_t n = 0;
  size_t size() const { return n; }
  void push(const zd::HostBlock&) { n++; }
};

}  // namespace

extern "C" {

int zd_shard_partition(const uint64_t* frame_bytes, size_t n, int world, size_t* cuts) {
  if (world <= 0 || !cuts || (n && !frame_bytes)) return ZD_E_INVALID_ARG;
  std::vector<uint64_t> prefix(n + 1, 0);
  for (size_t i = 0; i < n; i++) prefix[i + 1] = prefix[i] + frame_bytes[i];
  const unsigned __int128 total = prefix[n];
  cuts[0] = 0;
  for (int k = 1; k < world; k++) {
    // first frame boundary whose prefix reaches k/world of the bytes
    size_t c = (size_t)(std::lower_bound(prefix.begin(), prefix.end(), (uint64_t)0,
                                         [&](uint64_t p, uint64_t) { return (unsigned __int128)p * world < total * k; }) -
                        prefix.begin());
    if (n >= (size_t)world) {                   // leave one frame for each remaining rank
      c = std::max(c, cuts[k - 1] + 1);
      c = std::min(c, n - (size_t)(world - k));
    }
    cuts[k] = std::min(std::max(c, cuts[k - 1]), n);
  }
  cuts[world] = n;
  return ZD_OK;
}

int zd_shard_cuts(const uint8_t* src, size_t n, int world, uint64_t* src_cuts, uint64_t* frame_cuts) {
  if (world <= 0 || (!src && n) || !src_cuts || !frame_cuts) return ZD_E_INVALID_ARG;
  // one walk of the input (zd_frames_index's): the frames before the first
  // that fails to index
  std::vector<uint64_t> off, sizes;
  size_t cons = 0;
  const int st = zd::frame_spans(src, n, off, sizes, &cons);
  const size_t nf = off.size();
  std::vector<size_t> cuts((size_t)world + 1);
  zd_shard_partition(sizes.data(), nf, world, cuts.data());
  auto off_of = [&](size_t f) -> uint64_t { return f < nf ? off[f] : (uint64_t)cons; };
  for (int k = 0; k <= world; k++) {
    frame_cuts[k] = cuts[(size_t)k];
    src_cuts[k] = off_of(cuts[(size_t)k]);
  }
  // a frame that fails to index, and everything after it, goes to the last
  // rank: its plan stops there with that frame's status (FrameIterator)
  if (st != 0) src_cuts[world] = n;
  return ZD_OK;
}

int zd_shard_range_at(const uint8_t* src, size_t n, const uint64_t* src_cuts, const uint64_t* frame_cuts, int rank,
                      int world, uint64_t* src_begin, uint64_t* src_end, uint64_t* frame_begin, uint64_t* frame_end) {
  if (world <= 0 || rank < 0 || rank >= world || (!src && n) || !src_cuts || !frame_cuts) return ZD_E_INVALID_ARG;
  const uint64_t sb = src_cuts[rank], se = src_cuts[rank + 1];
  const uint64_t fb = frame_cuts[rank], fe = frame_cuts[rank + 1];
  if (sb > se || se > n || fb > fe) return ZD_E_INVALID_ARG;
  // the rank's own frames only (FrameIterator::next from its first frame,
  // frame.rs:94-99): they must tile [sb, se) with fe - fb frames, except that
  // the last rank's range may end in a frame that fails to index (its plan
  // reports it); a range that is not such a tiling is not this input's cuts
  zd::Bytes in{src + sb, (size_t)(n - sb)};
  uint64_t count = 0;
  bool failed = false;
  while ((uint64_t)(in.p - src) < se) {
    zd::HostFrame hf;
    CountSink S;
    if (zd::index_frame(src, in, &hf, S)) { failed = true; break; }
    count++;
  }
  const bool tiles = failed ? (rank == world - 1 && se == n) : (uint64_t)(in.p - src) == se;
  if (!tiles || count != fe - fb) return ZD_E_INVALID_ARG;
  if (src_begin) *src_begin = sb;
  if (src_end) *src_end = se;
  if (frame_begin) *frame_begin = fb;
  if (frame_end) *frame_end = fe;
  return ZD_OK;
}

int zd_shard_range(const uint8_t* src, size_t n, int rank, int world, uint64_t* src_begin, uint64_t* src_end,
                   uint64_t* frame_begin, uint64_t* frame_end) {
  if (world <= 0 || rank < 0 || rank >= world || (!src && n)) return ZD_E_INVALID_ARG;
  std::vector<uint64_t> sc((size_t)world + 1), fc((size_t)world + 1);
  if (int r = zd_shard_cuts(src, n, world, sc.data(), fc.data())) return r;
  if (src_begin) *src_begin = sc[rank];
  if (src_end) *src_end = sc[rank + 1];
  if (frame_begin) *frame_begin = fc[rank];
  if (frame_end) *frame_end = fc[rank + 1];
  return ZD_OK;
}

int zd_comm_unique_id(uint8_t id[ZD_COMM_ID_BYTES]) {
  Rccl* R = rccl();
  if (!R) return ZD_E_COMM;
  ncclUniqueId u;
  NCCLCHK(R->GetUniqueId(&u));
  memcpy(id, u.internal, ZD_COMM_ID_BYTES);
  return ZD_OK;
}

int zd_comm_create(const uint8_t id[ZD_COMM_ID_BYTES], int world, int rank, zd_comm** out) {
  if (!out || world <= 0 || rank < 0 || rank >= world) return ZD_E_INVALID_ARG;
  Rccl* R = rccl();
  if (!R) return ZD_E_COMM;
  zd_comm* c = new (std::nothrow) zd_comm();
  if (!c) return ZD_E_NO_MEMORY;
  c->world = world;
  c->rank = rank;
  ncclUniqueId u;
  memcpy(u.internal, id, ZD_COMM_ID_BYTES);
  if (R->CommInitRank(&c->nc, world, u, rank) != 0 ||
      hipMalloc(&c->d_meta, sizeof(int64_t) * 4 * (size_t)world) != hipSuccess) {
    zd_comm_destroy(c);
    return ZD_E_COMM;
  }
  *out = c;
  return ZD_OK;
}

int zd_comm_buffers(const zd_comm* c, uint64_t* src_bytes, uint64_t* out_bytes) {
  if (!c) return ZD_E_INVALID_ARG;
  if (src_bytes) *src_bytes = c->src_cap;
  if (out_bytes) *out_bytes = c->out_cap;
  return ZD_OK;
}

void zd_comm_destroy(zd_comm* c) {
  if (!c) return;
  Rccl* R = rccl();
  if (c->nc && R) R->CommDestroy(c->nc);
  if (c->d_meta) (void)hipFree(c->d_meta);
  if (c->d_src) (void)hipFree(c->d_src);
  if (c->d_out) (void)hipFree(c->d_out);
  delete c;
}

int zd_gather_layout(const int64_t* meta, int world, uint64_t* off, uint64_t* len, zd_gather_result* res) {
  if (!meta || world <= 0 || !off || !len || !res) return ZD_E_INVALID_ARG;
  // the output stops at the first failing rank's failure (src/main.rs:43-53)
  int failed = world;
  for (int r = 0; r < world; r++)
    if (meta[4 * r] != 0) { failed = r; break; }
  uint64_t total = 0;
  for (int r = 0; r < world; r++) {
    len[r] = (r <= failed && meta[4 * r + 2] > 0) ? (uint64_t)meta[4 * r + 2] : 0;
    off[r] = total;
    total += len[r];
  }
  res->total_len = total;
  res->failed_rank = failed;
  res->status = failed < world ? (int32_t)meta[4 * failed] : ZD_OK;
  res->first_error_frame = failed < world ? meta[4 * failed + 1] : -1;
  if (total > (uint64_t)std::max<int64_t>(meta[3], 0)) {   // rank 0's capacity, known to all
    res->total_len = 0;
    return ZD_E_DST_TOO_SMALL;
  }
  return ZD_OK;
}

int zd_comm_gather(zd_comm* c, const uint8_t* d_local, uint64_t local_len, int32_t status, int64_t first_error_frame,
                   uint8_t* d_root_out, uint64_t root_cap, zd_gather_result* res, void* stream) {
  if (!c || !res || (local_len && !d_local) || (c->rank == 0 && root_cap && !d_root_out)) return ZD_E_INVALID_ARG;
  Rccl* R = rccl();
  if (!R) return ZD_E_COMM;
  hipStream_t s = (hipStream_t)stream;
  const int W = c->world;
  // every rank's outcome, on every rank
  const int64_t mine[4] = {status, status ? first_error_frame : -1, (int64_t)local_len,
                           c->rank == 0 ? (int64_t)root_cap : 0};
  HIPCHK(hipMemcpyAsync(c->d_meta + 4 * c->rank, mine, sizeof mine, hipMemcpyHostToDevice, s));
  NCCLCHK(R->AllGather(c->d_meta + 4 * c->rank, c->d_meta, 4, ncclInt64, c->nc, s));
  std::vector<int64_t> m(4 * (size_t)W);
  HIPCHK(hipMemcpyAsync(m.data(), c->d_meta, sizeof(int64_t) * m.size(), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  std::vector<uint64_t> len((size_t)W, 0), off((size_t)W, 0);
  if (int r = zd_gather_layout(m.data(), W, off.data(), len.data(), res)) return r;   // nobody sends
  if (c->rank == 0 && len[0] && d_local != d_root_out)
    HIPCHK(hipMemcpyAsync(d_root_out, d_local, len[0], hipMemcpyDeviceToDevice, s));
  // point-to-point over the peers' own xGMI links to GPU 0
  NCCLCHK(R->GroupStart());
  if (c->rank == 0) {
    for (int r = 1; r < W; r++)
      if (len[r]) NCCLCHK(R->Recv(d_root_out + off[r], len[r], ncclUint8, r, c->nc, s));
  } else if (len[c->rank]) {
    NCCLCHK(R->Send(d_local, len[c->rank], ncclUint8, 0, c->nc, s));
  }
  NCCLCHK(R->GroupEnd());
  return ZD_OK;
}

// zd_decode_sharded(_at) once the rank's range is known
static int decode_range(zd_comm* c, const uint8_t* src, uint64_t sb, uint64_t se, uint64_t fb, int32_t pre,
                        uint32_t flags, uint8_t* d_root_out, uint64_t root_cap, zd_gather_result* res, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int32_t status = pre;
  int64_t first = pre ? 0 : -1;
  uint64_t len = 0;
  uint8_t* d_out = nullptr;
  zd_plan* P = nullptr;
  // a local failure still takes part in the collective (as this rank's
  // status), so no rank is left waiting in it
  if (!pre && se > sb) {
    int err = 0;
    do {
      if ((err = zd_plan_create(src + sb, se - sb, flags, &P))) break;
      zd_plan_info info;
      zd_plan_info_get(P, &info);
      const uint64_t ob = std::max<uint64_t>(info.out_bytes, 16);
      if (!grow(c->d_src, c->src_cap, se - sb + ZD_SRC_PADDING)) { err = ZD_E_HIP; break; }
      if (hipMemcpyAsync(c->d_src, src + sb, se - sb, hipMemcpyHostToDevice, s) != hipSuccess) { err = ZD_E_HIP; break; }
      // rank 0's range comes first in the output: it decodes in place (until
      // a re-plan outgrows the root buffer: then into the communicator's own,
      // and the gather copies it over)
      zd::DevOut o = (c->rank == 0 && root_cap >= ob) ? zd::DevOut{d_root_out, root_cap, &c->d_out, &c->out_cap}
                                                     : zd::DevOut{c->d_out, c->out_cap, &c->d_out, &c->out_cap};
      // the same decode as zd_plan_decompress, re-plans past frames that
      // overran their reserved capacity included
      uint64_t replans = 0;
      const int r = zd::decode_resident(P, src + sb, se - sb, c->d_src, o, s, &len, &first, &replans);
      if (r == ZD_E_HIP || r == ZD_E_INVALID_ARG || r == ZD_E_DST_TOO_SMALL) { err = r; break; }
      d_out = o.p;
      status = r;
    } while (0);
    if (err) { status = err; len = 0; first = 0; }
  }
  auto fin = [&](int r) {
    zd_plan_destroy(P);
    return r;
  };
  const int g = zd_comm_gather(c, d_out, len, status, status ? (int64_t)fb + first : -1, d_root_out, root_cap, res, s);
  if (g == ZD_OK && hipStreamSynchronize(s) != hipSuccess) return fin(ZD_E_HIP);
  return fin(g);
}

int zd_decode_sharded(zd_comm* c, const uint8_t* src, size_t n, uint32_t flags, uint8_t* d_root_out, uint64_t root_cap,
                      zd_gather_result* res, void* stream) {
  if (!c || !res || (!src && n)) return ZD_E_INVALID_ARG;
  uint64_t sb = 0, se = 0, fb = 0, fe = 0;
  if (int r = zd_shard_range(src, n, c->rank, c->world, &sb, &se, &fb, &fe)) return r;
  return decode_range(c, src, sb, se, fb, ZD_OK, flags, d_root_out, root_cap, res, stream);
}

int zd_decode_sharded_at(zd_comm* c, const uint8_t* src, size_t n, const uint64_t* src_cuts, const uint64_t* frame_cuts,
                         uint32_t flags, uint8_t* d_root_out, uint64_t root_cap, zd_gather_result* res, void* stream) {
  if (!c || !res || (!src && n)) return ZD_E_INVALID_ARG;
  uint64_t sb = 0, se = 0, fb = 0, fe = 0;
  // cuts that do not fit this rank's range fail here but still join the
  // collective, so every rank sees ZD_E_INVALID_ARG in res->status
  const int pre = zd_shard_range_at(src, n, src_cuts, frame_cuts, c->rank, c->world, &sb, &se, &fb, &fe);
  return decode_range(c, src, sb, se, fb, pre, flags, d_root_out, root_cap, res, stream);
}

}  // extern "C"
