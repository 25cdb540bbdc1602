// Probe: does the instruction offset of global_load_lds_dwordx4 also offset
// the LDS destination?  Writes LDS contents back to global.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(const unsigned *src, unsigned *dst) {
  __shared__ unsigned lds[2048];
  for (int i = threadIdx.x; i < 2048; i += 64) lds[i] = 0xdeadbeef;
  __syncthreads();
  const unsigned base = (unsigned) (uintptr_t) (const __attribute__((address_space(3))) void *) lds;
  const unsigned *g = src + threadIdx.x * 4;
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off offset:1024\n\ts_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
               : "=&s"(keep) : "v"(g), "s"(base) : "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += 64) dst[i] = lds[i];
}
int main() {
  unsigned *s, *d, h[2048];
  hipMalloc(&s, 4 * 4096); hipMalloc(&d, 4 * 2048);
  unsigned init[4096];
  for (int i = 0; i < 4096; i++) init[i] = i;
  hipMemcpy(s, init, sizeof init, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, s, d);
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  int first = -1;
  for (int i = 0; i < 2048; i++) if (h[i] != 0xdeadbeef) { first = i; break; }
  printf("first written LDS dword %d holds %u (global dword index); lds[0]=%x lds[256]=%x\n",
         first, first >= 0 ? h[first] : 0, h[0], h[256]);
  return 0;
}
