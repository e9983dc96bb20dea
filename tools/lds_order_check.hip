// Checks the LDS write-ordering property K4's overshoot copies rely on: when
// the lanes of ONE wave's ds_write_b128 (byte-unaligned addresses) write
// overlapping bytes, each byte ends up holding the value of the HIGHEST lane
// that wrote it.  Random trials: increasing start positions q_i with gaps
// drawn like zstd sequence lengths (1..40 bytes, mostly short), some lanes
// inactive, many waves per CU writing their own LDS at the same time.
// Prints "ok <trials> trials" or the mismatch count; exit status 0 / 1.
// usage: tools/lds_order_check [blocks] [trials per block]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef unsigned long long u64a1 __attribute__((aligned(1)));
constexpr int BUF = 4096;
constexpr int WAVES = 4;   // per workgroup: independent waves, each its own LDS area

__device__ inline unsigned lcg(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  return s >> 8;
}

// kind 0: ds_write_b128; kind 1: ds_write_b64 (8-byte overshoot)
template <int KIND>
__global__ __launch_bounds__(64 * WAVES) void k(unsigned trials, unsigned seed, unsigned long long* bad,
                                                unsigned long long* checked) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[WAVES][BUF];
  __shared__ int qs[WAVES][64];
  __shared__ int act_s[WAVES][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned char* L = lds[w];
  unsigned s = seed ^ (blockIdx.x * 0x9E3779B9u) ^ (w * 0x85EBCA6Bu);
  unsigned long long nb = 0, nc = 0;
  constexpr int SZ = KIND == 0 ? 16 : 8;
  for (unsigned t = 0; t < trials; t++) {
    // every lane draws the same gaps (same seed stream), so q is uniform knowledge
    unsigned ss = s;
    int q = (int)(lcg(ss) & 15), my_q = 0;
    const unsigned mode = lcg(ss) & 3;
    for (int i = 0; i < 64; i++) {
      unsigned r = lcg(ss);
      int len;
      if (mode == 0) len = 1 + (int)(r % 4);            // dense: many writers per byte
      else if (mode == 1) len = 3 + (int)(r % 12);      // zstd-like short sequences
      else if (mode == 2) len = 1 + (int)(r % 40);
      else len = (r & 7) == 0 ? 0 : 1 + (int)(r % 9);   // zero-length writers too
      if (i == lane) my_q = q;
      q += len;
    }
    const bool active = (lcg(ss) >> (lane & 15) & 7) != 0;   // ~1/8 of lanes inactive, varying
    s = ss;
    for (int i = lane; i < BUF; i += 64) L[i] = 0xEE;
    qs[w][lane] = my_q;
    act_s[w][lane] = active;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned tag = (t * 64u + (unsigned)lane) & 0xFFu;
    if (active) {
      if constexpr (KIND == 0) {
        u32x4a1 v;
        v.x = tag * 0x01010101u ^ 0x03020100u;
        v.y = tag * 0x01010101u ^ 0x07060504u;
        v.z = tag * 0x01010101u ^ 0x0B0A0908u;
        v.w = tag * 0x01010101u ^ 0x0F0E0D0Cu;
        *(__attribute__((address_space(3))) u32x4a1*)(__attribute__((address_space(3))) unsigned char*)(L + my_q) = v;
      } else {
        const unsigned long long v = (unsigned long long)(tag * 0x01010101u ^ 0x03020100u) |
                                     ((unsigned long long)(tag * 0x01010101u ^ 0x07060504u) << 32);
        *(__attribute__((address_space(3))) u64a1*)(__attribute__((address_space(3))) unsigned char*)(L + my_q) = v;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0);
    // check: byte b's expected writer is the highest active lane covering it
    const int end = qs[w][63] + SZ;
    for (int b = lane; b < end && b < BUF; b += 64) {
      int owner = -1;
      for (int i = 63; i >= 0; i--)
        if (act_s[w][i] && qs[w][i] <= b && b < qs[w][i] + SZ) { owner = i; break; }
      unsigned char want = 0xEE;
      if (owner >= 0) {
        const unsigned tg = (t * 64u + (unsigned)owner) & 0xFFu;
        want = (unsigned char)(tg ^ (unsigned)(b - qs[w][owner]));
      }
      nc++;
      if (L[b] != want) nb++;
    }
    __builtin_amdgcn_wave_barrier();
  }
  atomicAdd(bad, nb);
  atomicAdd(checked, nc);
}

int main(int argc, char** argv) {
  const unsigned blocks = argc > 1 ? atoi(argv[1]) : 2048, trials = argc > 2 ? atoi(argv[2]) : 256;
  unsigned long long* d;
  if (hipMalloc(&d, 32) != hipSuccess) return 2;
  int rc = 0;
  for (int kind = 0; kind < 2; kind++) {
    hipMemset(d, 0, 32);
    if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64 * WAVES), 0, 0, trials, 0x1234u, d, d + 1);
    else hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64 * WAVES), 0, 0, trials, 0x5678u, d, d + 1);
    unsigned long long h[2];
    if (hipMemcpy(h, d, 16, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    printf("%s: %llu bad of %llu bytes checked, %llu wave trials\n", kind == 0 ? "ds_write_b128" : "ds_write_b64",
           h[0], h[1], (unsigned long long)blocks * WAVES * trials);
    if (h[0]) rc = 1;
  }
  printf(rc ? "FAIL\n" : "ok\n");
  return rc;
}
