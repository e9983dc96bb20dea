// zd_internal.h — host-side helpers shared between the translation units of
// libzd (not part of the C ABI).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace zd {

// The frames of src[0, n) by zd_frames_index's walk, done once: offset and
// size of every frame before the first one that fails to index.  Returns
// that frame's status (0 if none) and sets *consumed to its offset (n when
// every frame indexed).
int frame_spans(const uint8_t* src, size_t n, std::vector<uint64_t>& off, std::vector<uint64_t>& size,
                size_t* consumed);

}  // namespace zd
