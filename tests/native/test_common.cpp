// Host unit test of the arithmetic shared by the kernels and the host
// (zstd-decompressor_amd/csrc/zd_common.h): sequence-code baselines, the
// 16-bit FSE entry, and the symbolic repeat-offset codes against a direct
// restatement of DecodingContext::decode_offset (decoding_context.rs:50-75).
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
  // packed record round trip
  std::mt19937_64 g(7);
  for (int i = 0; i < 100000; i++) {
    uint32_t ll = g() % 131072, ml = g() % 131075, oc = g() % (1u << 29);
    uint64_t s = seq_pack(ll, ml, oc);
    CHECK(seq_ll(s) == ll && seq_ml(s) == ml && seq_off(s) == oc, "pack");
  }
  // symbolic repeat offsets == direct decode_offset, per block, from random
  // incoming states, including rep0-1 chains, zeros and underflows
  for (int trial = 0; trial < 20000; trial++) {
    uint64_t in[3];
    for (int k = 0; k < 3; k++) in[k] = (g() % 4 == 0) ? g() % 3 : 1 + g() % 100000;
    uint64_t o[3] = {in[0], in[1], in[2]};
    uint32_t r[3]; rep_init(r);
    int n = 1 + g() % 40;
    for (int i = 0; i < n; i++) {
      uint64_t ofv; uint32_t ll = (g() % 3 == 0) ? 0 : 1 + g() % 50;
      uint64_t pick = g() % 10;
      ofv = pick < 7 ? 1 + g() % 3 : (pick < 9 ? 4 + g() % 5000 : (g() % 50 == 0 ? 0 : (1ull << 28) + 3 + g() % 1000));
      uint64_t want = 0; int wst = ref_decode(o, ofv, ll, &want);
      uint32_t code = rep_step(r, (uint32_t)ofv, ll);
      uint64_t got = 0; int gst = off_resolve(code, in, &got);
      if (wst) { CHECK(gst == wst, "trial %d seq %d: status %d vs %d", trial, i, gst, wst); break; }
      CHECK(gst == 0, "trial %d seq %d: unexpected status %d", trial, i, gst);
      if (want >= (1ull << 28) - (1ull << 24)) CHECK(got >= (1ull << 27), "giant offset %llu -> %llu", (unsigned long long)want, (unsigned long long)got);
      else CHECK(got == want, "trial %d seq %d: off %llu vs %llu", trial, i, (unsigned long long)got, (unsigned long long)want);
    }
  }
  if (fails) { printf("%d failures\n", fails); return 1; }
  printf("ok\n");
  return 0;
}
