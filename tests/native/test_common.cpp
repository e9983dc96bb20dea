// Host unit test of the arithmetic shared by the kernels and the host
// (zstd-decompressor_amd/csrc/zd_common.h): sequence-code baselines, the
// 16-bit FSE entry, K3's chain entries, direct sequence records, and K4's
// batch walk of the repeat offsets against a direct restatement of
// DecodingContext::decode_offset (decoding_context.rs:50-75).
#include <cstdio>
#include <cstdlib>
#include <random>
#include "../../zstd-decompressor_amd/csrc/zd_common.h"
using namespace zd;

static const uint32_t ML_BASE[53] = {3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,24,25,26,27,28,29,30,31,32,33,34,
  35,37,39,41,43,47,51,59,67,83,99,131,259,515,1027,2051,4099,8195,16387,32771,65539};
static const uint8_t ML_BITS[53] = {0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,
  1,1,1,1,2,2,3,3,4,4,5,7,8,9,10,11,12,13,14,15,16};
static const uint32_t LL_BASE[36] = {0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,18,20,22,24,28,32,40,48,64,128,256,512,1024,2048,4096,
  8192,16384,32768,65536};
static const uint8_t LL_BITS[36] = {0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,1,1,1,1,2,2,3,3,4,6,7,8,9,10,11,12,13,14,15,16};

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fails++; if (fails < 20) { printf("FAIL %s:%d: ", __FILE__, __LINE__); printf(__VA_ARGS__); printf("\n"); } } } while (0)

// reference decode_offset on concrete values; returns 0 / -41 / -90
static int ref_decode(uint64_t o[3], uint64_t ofv, uint64_t ll, uint64_t* out) {
  if (ofv == 0) return -41;
  if (ofv == 3 && ll == 0) { o[2] = o[1]; o[1] = o[0]; if (o[0] == 0) return -90; o[0] -= 1; }
  else if (ofv == 3 || (ofv == 2 && ll == 0)) { uint64_t t = o[2]; o[2] = o[1]; o[1] = o[0]; o[0] = t; }
  else if (ofv == 2 || (ofv == 1 && ll == 0)) { uint64_t t = o[0]; o[0] = o[1]; o[1] = t; }
  else if (ofv == 1) {}
  else { o[2] = o[1]; o[1] = o[0]; o[0] = ofv - 3; }
  *out = o[0];
  return 0;
}

int main() {
  for (uint32_t c = 0; c < 36; c++) {
    uint32_t b, n; ll_code(c, &b, &n);
    CHECK(b == LL_BASE[c] && n == LL_BITS[c], "ll code %u: %u/%u vs %u/%u", c, b, n, LL_BASE[c], LL_BITS[c]);
  }
  for (uint32_t c = 0; c < 53; c++) {
    uint32_t b, n; ml_code(c, &b, &n);
    CHECK(b == ML_BASE[c] && n == ML_BITS[c], "ml code %u: %u/%u vs %u/%u", c, b, n, ML_BASE[c], ML_BITS[c]);
  }
  // FSE entry: nb/baseline from nextState (fse.rs:169-189 closed form)
  for (int al = 0; al <= 9; al++) {
    uint32_t T = 1u << al;
    for (uint32_t ns = 1; ns < 2 * T && ns < 1024; ns++) {
      uint16_t e = fse_entry(5, ns);
      uint32_t nb = fse_nb(e, al), base = fse_base(e, al);
      int hb = 31 - __builtin_clz(ns);
      CHECK(nb == (uint32_t)(al - hb) && base == (ns << (al - hb)) - T && fse_sym(e) == 5, "fse al %d ns %u", al, ns);
    }
  }
  // K3 chain entries: nextState, extra bits of the code, code-max flag
  for (int k = 0; k < 3; k++) {
    for (uint32_t c = 0; c < 64; c++) {
      for (uint32_t ns = 1; ns < 1024; ns += 37) {
        uint32_t e = k3_entry(fse_entry(c, ns), k);
        uint32_t bits = k == 0 ? (c < 36 ? LL_BITS[c] : 0) : (k == 2 ? (c < 53 ? ML_BITS[c] : 0) : c);
        bool bad = k == 0 ? c > 35 : (k == 2 ? c > 52 : c > 31);
        CHECK((e & 1023) == ns, "k3 ns");
        CHECK(((e & K3_BAD) != 0) == bad, "k3 bad k=%d c=%u", k, c);
        if (!bad) CHECK(((e >> 10) & 31) == bits, "k3 bits k=%d c=%u", k, c);
      }
    }
  }
  // K3 fast-chain entries: nextState, extra + state bit count, 63 for a code above the maximum
  for (int k = 0; k < 3; k++) {
    for (int al = 5; al <= 9; al++) {
      for (uint32_t c = 0; c < 64; c++) {
        for (uint32_t ns = 1; ns < (2u << al); ns += 13) {
          uint32_t e = k3f_entry(fse_entry(c, ns), k, al);
          uint32_t bits = k == 0 ? (c < 36 ? LL_BITS[c] : 0) : (k == 2 ? (c < 53 ? ML_BITS[c] : 0) : c);
          bool bad = k == 0 ? c > 35 : (k == 2 ? c > 52 : c > 31);
          int nb = al - (31 - __builtin_clz(ns));
          CHECK((e & 1023) == ns, "k3f ns");
          CHECK(bad ? (e >> 10) == 63 : (e >> 10) == bits + nb, "k3f count k=%d al=%d c=%u ns=%u", k, al, c, ns);
        }
      }
    }
  }
  // direct records round trip (offset values past DIRECT_GIANT saturate)
  std::mt19937_64 g(7);
  for (int i = 0; i < 100000; i++) {
    uint32_t ll = g() % 131072, ml = g() % 131075, ov = (uint32_t)g();
    uint64_t s = seq_pack(ll, ml, ov);
    CHECK(seq_ll(s) == ll && seq_ml(s) == ml && seq_off(s) == (ov > DIRECT_GIANT ? DIRECT_GIANT : ov), "pack");
  }
  // K4's batch walk of decode_offset (zd_kernels.hip zd_k_execute): fresh
  // offsets direct, repeat codes walked in order from the state the fresh
  // lanes before them pushed; the state after lane k - 1 the same way.
  for (int trial = 0; trial < 20000; trial++) {
    uint64_t o[3];
    for (int k = 0; k < 3; k++) o[k] = (g() % 4 == 0) ? g() % 3 : 1 + g() % 100000;
    uint64_t rep[3] = {o[0], o[1], o[2]};
    int n = 1 + g() % 64, kexec = 1 + g() % n;
    uint64_t ofv[64], ll[64], val[64];
    for (int i = 0; i < n; i++) {
      uint64_t pick = g() % 10;
      ll[i] = (g() % 3 == 0) ? 0 : 1 + g() % 50;
      ofv[i] = pick < (trial % 2 ? 2 : 7) ? 1 + g() % 3 : (pick < 9 ? 4 + g() % 5000 : (g() % 50 == 0 ? 0 : 4 + g() % 7));
      val[i] = ofv[i] - 3;
    }
    auto push = [&](int cnt, int end, const uint64_t r[3], uint64_t a[3]) {
      a[0] = r[0]; a[1] = r[1]; a[2] = r[2];
      if (cnt >= 1) { a[0] = val[end - 1]; a[1] = r[0]; a[2] = r[1]; }
      if (cnt >= 2) { a[1] = val[end - 2]; a[2] = r[0]; }
      if (cnt >= 3) a[2] = val[end - 3];
    };
    uint64_t r[3] = {rep[0], rep[1], rep[2]};
    uint64_t off[64];
    int err[64] = {0};
    int prev = -1, stop = -1;
    for (int i = 0; i < kexec; i++) {
      off[i] = val[i];
      if (ofv[i] > 3) continue;
      uint64_t a[3];
      push(i - prev - 1, i, r, a);
      int e = 0; uint64_t v = 0;
      if (ofv[i] == 0) e = -41;
      else {
        uint32_t idx = (uint32_t)ofv[i] - (ll[i] != 0 ? 1 : 0);
        if (idx == 0) v = a[0];
        else if (idx == 1) { v = a[1]; a[1] = a[0]; a[0] = v; }
        else if (idx == 2) { v = a[2]; a[2] = a[1]; a[1] = a[0]; a[0] = v; }
        else if (a[0] == 0) e = -90;
        else { v = a[0] - 1; a[2] = a[1]; a[1] = a[0]; a[0] = v; }
      }
      off[i] = v; err[i] = e;
      r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
      prev = i;
      if (e) { stop = i; break; }
    }
    uint64_t after[3];
    push(kexec - 1 - prev, kexec, r, after);
    // direct restatement
    uint64_t want;
    for (int i = 0; i < kexec; i++) {
      int wst = ref_decode(o, ofv[i], ll[i], &want);
      if (wst) { CHECK(stop == i && err[i] == wst, "trial %d seq %d: status %d vs %d", trial, i, err[i], wst); break; }
      CHECK(off[i] == want, "trial %d seq %d: off %llu vs %llu", trial, i, (unsigned long long)off[i], (unsigned long long)want);
      if (i == kexec - 1)
        CHECK(after[0] == o[0] && after[1] == o[1] && after[2] == o[2], "trial %d: state after the batch", trial);
    }
  }
  if (fails) { printf("%d failures\n", fails); return 1; }
  printf("ok\n");
  return 0;
}
