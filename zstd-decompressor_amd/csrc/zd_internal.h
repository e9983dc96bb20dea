// zd_internal.h — host-side helpers shared between the translation units of
// libzd (not part of the C ABI).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

struct zd_plan;

namespace zd {

// The frames of src[0, n) by zd_frames_index's walk, done once: offset and
// size of every frame before the first one that fails to index.  Returns
// that frame's status (0 if none) and sets *consumed to its offset (n when
// every frame indexed).
int frame_spans(const uint8_t* src, size_t n, std::vector<uint64_t>& off, std::vector<uint64_t>& size,
                size_t* consumed);

// A device output buffer a decode with re-plans may grow: p holds cap bytes.
// A growth allocates into *own / *own_cap (the caller's kept allocation) and
// keeps the bytes decoded so far; p may start out as a buffer the caller does
// not own (rank 0's output), which is never freed here.
struct DevOut {
  uint8_t* p;
  uint64_t cap;
  uint8_t** own;
  uint64_t* own_cap;
};

// Decodes plan P (made for src[0, n), resident at d_src with ZD_SRC_PADDING
// readable bytes after it) into out on `stream`, re-planning past a frame
// that reached a limit the host can lift (its reserved capacity, K4J rounds;
// zd_host.cpp decode_resident).  zd_plan_decompress and zd_decode_sharded
// both decode through it.  *total = bytes of the frames before the first
// failure, *first_frame = that frame's index in P (-1 if none), *replans =
// re-plans made.  Returns the input's status (ZD_E_HIP / ZD_E_INVALID_ARG /
// ZD_E_DST_TOO_SMALL: the call itself failed).
// Per-frame outcome of a decode_resident call (optional): frame f of P's
// status (ZD_OK, its error, ZD_E_NOT_DECODED after the first failure) and
// its bytes' offset and length in the output, re-plans included.
struct FrameOuts {
  std::vector<int32_t> status;
  std::vector<uint64_t> off, len;
};
int decode_resident(zd_plan* P, const uint8_t* src, size_t n, const uint8_t* d_src, DevOut& out, void* stream,
                    uint64_t* total, int64_t* first_frame, uint64_t* replans, FrameOuts* fo = nullptr);

}  // namespace zd
