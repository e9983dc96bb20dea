// fuzz_host.cpp -- sanitizer driver for libzd's host side and the oracle
// (ASan/UBSan/TSan on host code).  No GPU: it exercises what
// runs on the host -- the frame walk (zd_frames_index: the serial capped walk
// and the speculative parallel walk with its stitch), the shard partition and
// ranges, the gather layout -- and the oracle's decode (the test checker), on
// the given inputs and on seeded mutations of them (byte flips, truncations,
// planted frame magic numbers, splices).  Invariants are checked; the
// sanitizers check the memory and thread behaviour.
//
//   fuzz_host ITERATIONS SEED FILE...
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/zd.h"
#include "../../oracle/zd_oracle.h"

static uint64_t rs;
static uint64_t rnd() { rs ^= rs >> 12; rs ^= rs << 25; rs ^= rs >> 27; return rs * 0x2545F4914F6CDD1Dull; }
static size_t below(size_t n) { return n ? (size_t)(rnd() % n) : 0; }

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); fails++; } } while (0)

static std::vector<uint8_t> read_file(const char* p) {
  std::vector<uint8_t> v;
  FILE* f = fopen(p, "rb");
  if (!f) { perror(p); exit(2); }
  uint8_t b[1 << 16];
  size_t k;
  while ((k = fread(b, 1, sizeof b, f)) > 0) v.insert(v.end(), b, b + k);
  fclose(f);
  return v;
}

static void mutate(std::vector<uint8_t>& d, const std::vector<std::vector<uint8_t>>& pool) {
  static const uint8_t magic[4] = {0x28, 0xB5, 0x2F, 0xFD};
  switch (below(5)) {
    case 0:                                       // byte flips
      for (int k = 1 + (int)below(4); k > 0 && !d.empty(); k--) d[below(d.size())] = (uint8_t)rnd();
      break;
    case 1:                                       // truncation
      if (!d.empty()) d.resize(below(d.size()));
      break;
    case 2:                                       // planted magic numbers
      for (int k = 1 + (int)below(8); k > 0 && d.size() >= 4; k--) memcpy(&d[below(d.size() - 3)], magic, 4);
      break;
    case 3: {                                     // splice another input's bytes in
      const auto& o = pool[below(pool.size())];
      if (o.empty()) break;
      const size_t a = below(o.size()), len = below(std::min<size_t>(o.size() - a, 1 << 16)) + 1;
      const size_t at = below(d.size() + 1);
      d.insert(d.begin() + (long)at, o.begin() + (long)a, o.begin() + (long)(a + len));
      break;
    }
    default:                                      // a header byte of some frame region
      if (d.size() > 8) d[below(16) % d.size()] ^= (uint8_t)(1u << below(8));
  }
}

static void check_input(const std::vector<uint8_t>& d, bool oracle) {
  const uint8_t* src = d.empty() ? nullptr : d.data();
  size_t nf = 0, nb = 0, cons = 0;
  const int st = zd_frames_index(src, d.size(), nullptr, 0, &nf, nullptr, 0, &nb, &cons);
  std::vector<zd_frame_desc> fr(nf + 1);
  std::vector<zd_block_desc> bl(nb + 1);
  size_t nf2 = 0, nb2 = 0, cons2 = 0;
  const int st2 = zd_frames_index(src, d.size(), fr.data(), nf + 1, &nf2, bl.data(), nb + 1, &nb2, &cons2);
  CHECK(st == st2 && nf == nf2 && nb == nb2 && cons == cons2, "size query and fill disagree");
  CHECK(cons <= d.size(), "consumed past the input");
  uint64_t at = 0;
  for (size_t i = 0; i < nf2; i++) {
    CHECK(fr[i].src_offset == at, "frames not contiguous at %zu", i);
    at = fr[i].src_offset + fr[i].src_size;
    CHECK(fr[i].first_block + fr[i].num_blocks <= nb2, "frame blocks out of range");
  }
  CHECK(at == cons, "consumed %zu != end of frames %llu", cons, (unsigned long long)at);
  // the capped (serial) walk gives a prefix of the full walk
  const size_t cap = 1 + below(6);
  std::vector<zd_frame_desc> fc(cap);
  size_t nfc = 0, nbc = 0, consc = 0;
  zd_frames_index(src, d.size(), fc.data(), cap, &nfc, nullptr, 0, &nbc, &consc);
  CHECK(nfc == std::min(cap, nf2), "capped walk frame count %zu vs %zu", nfc, nf2);
  for (size_t i = 0; i < nfc && i < nf2; i++)
    CHECK(memcmp(&fc[i], &fr[i], sizeof fc[i]) == 0, "capped walk frame %zu differs", i);
  // shard ranges tile the indexed frames, every world
  for (int world = 1; world <= 8; world++) {
    uint64_t prev_end = 0, prev_fe = 0;
    for (int r = 0; r < world; r++) {
      uint64_t sb, se, fb, fe;
      CHECK(zd_shard_range(src, d.size(), r, world, &sb, &se, &fb, &fe) == ZD_OK, "zd_shard_range");
      CHECK(sb == prev_end && fb == prev_fe && se >= sb && fe >= fb, "ranges do not tile (world %d rank %d)", world, r);
      prev_end = se;
      prev_fe = fe;
    }
    CHECK(prev_fe == nf2, "frame ranges end at %llu, %zu frames", (unsigned long long)prev_fe, nf2);
    CHECK(prev_end == (st ? d.size() : cons), "byte ranges end at %llu", (unsigned long long)prev_end);
  }
  if (oracle) {
    uint8_t* out = nullptr;
    size_t ol = 0, of = 0;
    zdo_err e{};
    const int ost = zdo_decompress(src, d.size(), 0, &out, &ol, &of, &e);
    zdo_free(out);
    // a frame that fails the walk fails the oracle too, unless an earlier
    // failure (an entropy stage, found after the walk) stops the oracle first
    if (st) CHECK(ost != 0 && of <= nf2, "walk status %d at frame %zu, oracle %d after %zu frames", st, nf2, ost, of);
    else CHECK(ost == 0 || of <= nf2, "oracle fails past the walk's frames");
  }
}

static void check_layouts() {
  for (int t = 0; t < 200; t++) {
    const int world = 1 + (int)below(8);
    std::vector<int64_t> meta(4 * (size_t)world);
    for (int r = 0; r < world; r++) {
      meta[4 * r] = below(4) == 0 ? -(int64_t)(1 + below(95)) : 0;
      meta[4 * r + 1] = meta[4 * r] ? (int64_t)below(1000) : -1;
      meta[4 * r + 2] = (int64_t)below(1 << 20);
      meta[4 * r + 3] = r == 0 ? (int64_t)below(4 << 20) : 0;
    }
    std::vector<uint64_t> off(world), len(world);
    zd_gather_result res;
    const int s = zd_gather_layout(meta.data(), world, off.data(), len.data(), &res);
    CHECK(s == ZD_OK || s == ZD_E_DST_TOO_SMALL, "gather layout status %d", s);
    std::vector<uint64_t> sizes(below(40));
    for (auto& x : sizes) x = below(1 << 20);
    std::vector<size_t> cuts((size_t)world + 1);
    CHECK(zd_shard_partition(sizes.data(), sizes.size(), world, cuts.data()) == ZD_OK, "partition");
    for (int k = 0; k < world; k++) CHECK(cuts[k] <= cuts[k + 1], "cuts not ascending");
    CHECK(cuts[0] == 0 && cuts[world] == sizes.size(), "cuts do not cover");
  }
}

int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: %s ITERATIONS SEED FILE...\n", argv[0]); return 2; }
  const long iters = atol(argv[1]);
  rs = strtoull(argv[2], nullptr, 0) | 1;
  std::vector<std::vector<uint8_t>> pool;
  for (int i = 3; i < argc; i++) pool.push_back(read_file(argv[i]));
  const bool oracle = !getenv("FUZZ_NO_ORACLE");
  for (const auto& d : pool) check_input(d, oracle);
  check_layouts();
  for (long it = 0; it < iters; it++) {
    std::vector<uint8_t> d = pool[below(pool.size())];
    if (d.size() > (8u << 20) && (it % 8)) d.resize(below(1 << 20) + 1);   // big inputs whole now and then
    for (int k = 1 + (int)below(3); k > 0; k--) mutate(d, pool);
    check_input(d, oracle && d.size() < (4u << 20));
  }
  printf("fuzz_host: %ld iterations over %zu inputs, %d failures\n", iters, pool.size(), fails);
  return fails ? 1 : 0;
}
