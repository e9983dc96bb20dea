// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE on the access patterns
// of the decode kernels (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only
// for 16-B/lane coalesced streams, where it reports half the bytes).  Each
// kernel reads a known number of distinct bytes from a buffer far larger than
// the Infinity Cache (every byte once, or a stated reuse), so
// FETCH_SIZE / bytes per dispatch is the factor to correct that pattern by.
//   stream16   16 B per lane, coalesced (the guide's calibrated case)
//   stream8    8 B per lane, coalesced (K4's record slots, one per lane)
//   pair16     16 B per lane, lane pairs on the same 16 B (K4J / K4F record pairs)
//   win16      16 B per lane at byte positions 4.5 B apart, unaligned (K4's
//              bitstream windows: one per sequence, ~4.5 B of bitstream each)
//   gather16   16 B per lane at random 64-B-aligned lines of a 4 GiB buffer
//              (match sources flushed long ago: one line each)
// usage: fetch_calib  (prints one line per kernel: name, distinct bytes read)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__global__ void k_stream16(const u32x4* __restrict__ p, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void k_stream8(const u32x2* __restrict__ p, uint64_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const u32x2 v = p[i];
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void k_pair16(const u32x4* __restrict__ p, uint64_t n2, uint32_t* sink) {   // n2 = 2 x 16-B units
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n2; i += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 v = p[i >> 1];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void k_win16(const uint8_t* __restrict__ p, uint64_t nwin, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nwin; i += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 v = *(const u32x4a1*)(p + (i * 9) / 2);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void k_gather16(const uint8_t* __restrict__ p, uint64_t lines, uint64_t nloads, uint32_t* sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nloads; i += (uint64_t)gridDim.x * blockDim.x) {
    // a permutation of the lines (odd multiplier mod a power of two): each once
    const uint64_t line = (i * 0x9E3779B97F4A7C15ull) & (lines - 1);
    const u32x4 v = *(const u32x4*)(p + line * 64 + 16 * (i & 3));
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  const uint64_t B = 2ull << 30;                   // 2 GiB: far past the 256 MiB Infinity Cache
  const uint64_t G = 4ull << 30;                   // gather buffer
  uint8_t *a = nullptr, *g = nullptr;
  uint32_t* sink = nullptr;
  CHK(hipMalloc(&a, B + 64));
  CHK(hipMalloc(&g, G + 64));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(a, 1, B + 64));
  CHK(hipMemset(g, 2, G + 64));
  CHK(hipDeviceSynchronize());
  const dim3 grid(4096), blk(256);
  for (int rep = 0; rep < 2; rep++) {                // rep 1 is the one to read (caches cold for it too: 2 GiB between)
    hipLaunchKernelGGL(k_stream16, grid, blk, 0, 0, (const u32x4*)a, B / 16, sink);
    hipLaunchKernelGGL(k_stream8, grid, blk, 0, 0, (const u32x2*)a, B / 8, sink);
    hipLaunchKernelGGL(k_pair16, grid, blk, 0, 0, (const u32x4*)a, 2 * (B / 16), sink);
    hipLaunchKernelGGL(k_win16, grid, blk, 0, 0, (const uint8_t*)a, (B - 64) * 2 / 9, sink);
    hipLaunchKernelGGL(k_gather16, grid, blk, 0, 0, (const uint8_t*)g, G / 64, (G / 64) / 4, sink);
    CHK(hipDeviceSynchronize());
  }
  printf("k_stream16 distinct_bytes %llu\n", (unsigned long long)B);
  printf("k_stream8 distinct_bytes %llu\n", (unsigned long long)B);
  printf("k_pair16 distinct_bytes %llu\n", (unsigned long long)B);
  printf("k_win16 distinct_bytes %llu\n", (unsigned long long)(B - 64));
  printf("k_gather16 distinct_bytes %llu (lines touched %llu x 64 B, 16 B used each)\n",
         (unsigned long long)((G / 64) / 4 * 16), (unsigned long long)((G / 64) / 4));
  return 0;
}
