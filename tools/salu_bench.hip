// Microbenchmark for a scalar-unit FSE chain (the few-frame
// regime): what one wave's dependent step costs when its state lives in
// SGPRs.  One workgroup of one wave (and 1/2/4/8 waves per CU for the shared
// scalar unit), s_memtime around each loop:
//  salu_dep    dependent s_add_u32 chain
//  salu_ind4   four independent s_add_u32 chains interleaved
//  valu_dep    dependent v_add_u32 chain
//  sload_chase s_load_dword pointer chase in a table of S bytes (K$ / L2)
//  lds_chase   ds_read_b32 chase with the address from an SGPR (v_mov) and the
//              value back by v_readfirstlane (the LDS-table form of a scalar chain)
//  movrels     v_movrels_b32 + v_readlane chase over a table in 8 VGPRs
// usage: salu_bench  (prints one line per test: cycles per op)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef __attribute__((address_space(4))) const uint32_t c_u32;

__global__ void k_salu_dep(uint64_t* out, uint32_t seed) {
  uint32_t x = __builtin_amdgcn_readfirstlane(seed), y = __builtin_amdgcn_readfirstlane(seed + 1);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  asm volatile(".rept 512\n\ts_add_u32 %0, %0, %1\n\t.endr" : "+s"(x) : "s"(y));
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = x; }
}
__global__ void k_salu_ind4(uint64_t* out, uint32_t seed) {
  uint32_t a = __builtin_amdgcn_readfirstlane(seed), b = a + 1, c = a + 2, d = a + 3, y = a + 5;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  asm volatile(".rept 128\n\ts_add_u32 %0, %0, %4\n\ts_add_u32 %1, %1, %4\n\ts_add_u32 %2, %2, %4\n\ts_add_u32 %3, %3, %4\n\t.endr"
               : "+s"(a), "+s"(b), "+s"(c), "+s"(d) : "s"(y));
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = a ^ b ^ c ^ d; }
}
__global__ void k_valu_dep(uint64_t* out, uint32_t seed) {
  uint32_t x = seed + threadIdx.x, y = seed;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  asm volatile(".rept 512\n\tv_add_u32 %0, %0, %1\n\t.endr" : "+v"(x) : "v"(y));
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = x; }
}
// s_load chase: idx = T[idx], 256 hops
__global__ void k_sload_chase(uint64_t* out, const uint32_t* T, uint32_t start) {
  c_u32* t = (c_u32*)T;
  uint32_t idx = __builtin_amdgcn_readfirstlane(start);
  for (int i = 0; i < 8; i++) idx = t[idx];     // warm
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 256; i++) idx = t[idx];
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = idx; }
}
// three s_load chases interleaved (the three tables of one step)
__global__ void k_sload_chase3(uint64_t* out, const uint32_t* T, uint32_t start) {
  c_u32* t = (c_u32*)T;
  uint32_t a = __builtin_amdgcn_readfirstlane(start), b = a ^ 1, c = a ^ 2;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 256; i++) {
    const uint32_t na = t[a], nb = t[b], nc = t[c];
    a = na ^ (nb & 0); b = nb; c = nc;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = a + b + c; }
}
// LDS chase from an SGPR address: v_mov, ds_read_b32, wait, v_readfirstlane
__global__ void k_lds_chase(uint64_t* out, const uint32_t* T, uint32_t start) {
  __shared__ uint32_t L[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) L[i] = T[i] & 4095;
  __syncthreads();
  uint32_t idx = __builtin_amdgcn_readfirstlane(start & 4095);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 256; i++) idx = __builtin_amdgcn_readfirstlane(L[idx]);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = idx; }
}
// v_movrels chase over 8 VGPRs (512 entries): idx -> VGPR idx >> 6, lane idx & 63
__global__ void k_movrels_chase(uint64_t* out, const uint32_t* T, uint32_t start) {
  const int l = threadIdx.x;
  uint32_t r0 = T[l] & 511, r1 = T[64 + l] & 511, r2 = T[128 + l] & 511, r3 = T[192 + l] & 511;
  uint32_t r4 = T[256 + l] & 511, r5 = T[320 + l] & 511, r6 = T[384 + l] & 511, r7 = T[448 + l] & 511;
  uint32_t idx = __builtin_amdgcn_readfirstlane(start & 511);
  uint64_t t0 = 0, t1 = 0;
  asm volatile(
      "v_mov_b32 v40, %2\n\tv_mov_b32 v41, %3\n\tv_mov_b32 v42, %4\n\tv_mov_b32 v43, %5\n\t"
      "v_mov_b32 v44, %6\n\tv_mov_b32 v45, %7\n\tv_mov_b32 v46, %8\n\tv_mov_b32 v47, %9\n\t"
      "s_nop 4\n\t"
      "s_memtime %1\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      ".rept 256\n\t"
      "s_lshr_b32 s98, %0, 6\n\t"
      "s_and_b32 s99, %0, 63\n\t"
      "s_set_gpr_idx_on s98, gpr_idx(SRC0)\n\t"
      "v_mov_b32 v48, v40\n\t"
      "s_set_gpr_idx_off\n\t"
      "s_nop 1\n\t"
      "v_readlane_b32 %0, v48, s99\n\t"
      "s_nop 3\n\t"
      ".endr\n\t"
      "s_memtime %10\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "+s"(idx), "=&s"(t0)
      : "v"(r0), "v"(r1), "v"(r2), "v"(r3), "v"(r4), "v"(r5), "v"(r6), "v"(r7), "s"(t1)
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "s98", "s99");
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = idx; }
}

// domain crossings: VALU -> SGPR (v_readfirstlane) -> SALU -> VALU (v_add with the SGPR), dependent
__global__ void k_cross_vsv(uint64_t* out, uint32_t seed) {
  uint32_t v = seed + threadIdx.x * 0, s = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  asm volatile(".rept 256\n\tv_readfirstlane_b32 %1, %0\n\ts_add_u32 %1, %1, 1\n\tv_add_u32 %0, %1, %0\n\t.endr"
               : "+v"(v), "+s"(s));
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = v + s; }
}
// readlane chain: SGPR lane index -> v_readlane -> s_and (next index)
__global__ void k_cross_readlane(uint64_t* out, uint32_t seed) {
  uint32_t w = (threadIdx.x * 7 + 3) & 63, s = seed & 63;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  asm volatile(".rept 256\n\tv_readlane_b32 %1, %0, %1\n\ts_and_b32 %1, %1, 63\n\t.endr" : "+v"(w), "+s"(s));
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = w + s; }
}
// SALU -> VALU: s_add then v_add reading it, then v_readfirstlane back (the round trip of k_cross_vsv without the SALU op)
__global__ void k_cross_vs(uint64_t* out, uint32_t seed) {
  uint32_t v = seed, s = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  asm volatile(".rept 256\n\tv_readfirstlane_b32 %1, %0\n\tv_add_u32 %0, %1, %0\n\t.endr" : "+v"(v), "+s"(s));
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = v + s; }
}
// ds_read_b64 chase, VGPR address straight from the loaded value (no SGPR trip)
__global__ void k_lds_chase_v(uint64_t* out, const uint32_t* T, uint32_t start) {
  __shared__ uint32_t L[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) L[i] = (T[i] & 4095) * 4;
  __syncthreads();
  uint32_t a = (start & 4095) * 4;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int i = 0; i < 256; i++) a = *(volatile __attribute__((address_space(3))) uint32_t*)(uintptr_t)a;
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { out[blockIdx.x * 2] = t1 - t0; out[blockIdx.x * 2 + 1] = a; }
}
template <typename K, typename... A>
static double run(const char* name, int per, int grid, int block, K k, uint64_t* d, A... a) {
  std::vector<uint64_t> h(2 * grid);
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(block), 0, 0, d, a...);
    (void)hipDeviceSynchronize();
  }
  (void)hipMemcpy(h.data(), d, 16 * grid, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < grid; i++) s += (double)h[2 * i];
  s /= grid;
  printf("%-28s grid %5d: %8.1f ticks total, %6.2f ticks/op\n", name, grid, s, s / per);
  return s / per;
}

int main() {
  uint64_t* d;
  CHK(hipMalloc(&d, 16 * 8192));
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("CUs %d (s_memtime ticks; the shader clock on gfx9)\n", cus);
  for (int g : {1, cus, 4 * cus, 8 * cus, 16 * cus}) {
    run("salu_dep", 512, g, 64, k_salu_dep, d, 7u);
    run("salu_ind4", 512, g, 64, k_salu_ind4, d, 7u);
    run("valu_dep", 512, g, 64, k_valu_dep, d, 7u);
  }
  for (int g : {1, cus}) {
    run("cross v->s->v (3 instr)", 256, g, 64, k_cross_vsv, d, 7u);
    run("cross v->s->v (2 instr)", 256, g, 64, k_cross_vs, d, 7u);
    run("readlane s->v->s (2 instr)", 256, g, 64, k_cross_readlane, d, 7u);
  }
  std::mt19937 rng(5);
  for (uint32_t bytes : {1024u, 4096u, 8192u, 16384u, 32768u, 65536u, 1u << 20}) {
    const uint32_t n = bytes / 4;
    std::vector<uint32_t> perm(n), next(n);
    for (uint32_t i = 0; i < n; i++) perm[i] = i;
    std::shuffle(perm.begin(), perm.end(), rng);
    for (uint32_t i = 0; i < n; i++) next[perm[i]] = perm[(i + 1) % n];
    uint32_t* T;
    CHK(hipMalloc(&T, bytes + 4096 * 4));
    CHK(hipMemcpy(T, next.data(), bytes, hipMemcpyHostToDevice));
    char nm[64];
    for (int g : {1, cus, 4 * cus}) {
      snprintf(nm, sizeof nm, "sload_chase %u B", bytes);
      run(nm, 256, g, 64, k_sload_chase, d, (const uint32_t*)T, perm[0]);
      snprintf(nm, sizeof nm, "sload_chase3 %u B", bytes);
      run(nm, 256, g, 64, k_sload_chase3, d, (const uint32_t*)T, perm[0]);
    }
    if (bytes >= 16384) {
      for (int g : {1, cus, 4 * cus}) run("lds_chase", 256, g, 64, k_lds_chase, d, (const uint32_t*)T, perm[0]);
      for (int g : {1, cus, 4 * cus}) run("lds_chase_v (vgpr address)", 256, g, 64, k_lds_chase_v, d, (const uint32_t*)T, perm[0]);
    }
    if (bytes == 2048 || bytes == 4096) {
      for (int g : {1, cus, 4 * cus}) run("movrels_chase", 256, g, 64, k_movrels_chase, d, (const uint32_t*)T, perm[0]);
    }
    CHK(hipFree(T));
  }
  return 0;
}
