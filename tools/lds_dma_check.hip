// Does global_load_lds_dwordx4 (LDS DMA, 16 B per lane) take byte-unaligned
// global addresses on gfx950?  Lane i loads 16 bytes at src + 17*i + (i & 15)
// into LDS at base + 16*i; the host compares with the source bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
__global__ void k(const unsigned char* src, unsigned char* out) {
  __shared__ __attribute__((aligned(16))) unsigned char st[1024];
  const int i = threadIdx.x;
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(src + 17 * i + (i & 15)),
                                   (void __attribute__((address_space(3)))*)st, 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int b = 0; b < 16; b++) out[16 * i + b] = st[16 * i + b];
}
int main() {
  unsigned char h[4096], o[1024];
  for (int i = 0; i < 4096; i++) h[i] = (unsigned char)(i * 7 + (i >> 8));
  unsigned char *ds, *dd;
  if (hipMalloc(&ds, 4096) || hipMalloc(&dd, 1024)) return 2;
  hipMemcpy(ds, h, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, ds, dd);
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 3; }
  hipMemcpy(o, dd, 1024, hipMemcpyDeviceToHost);
  int bad = 0, aligned_bad = 0;
  for (int i = 0; i < 64; i++)
    for (int b = 0; b < 16; b++) {
      const int a = 17 * i + (i & 15);
      if (o[16 * i + b] != h[a + b]) { bad++; if ((a & 3) == 0) aligned_bad++; }
    }
  printf("lds dma unaligned: %d wrong bytes (%d at 4-byte aligned addresses)\n", bad, aligned_bad);
  return 0;
}
