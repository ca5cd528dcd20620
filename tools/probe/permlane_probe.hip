// semantics of v_permlane32_swap_b32 on gfx950: prints a / b of lanes 0, 31, 32, 63 after the swap
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  unsigned a = threadIdx.x, b = 100 + threadIdx.x;
  asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  out[threadIdx.x] = a;
  out[64 + threadIdx.x] = b;
}
int main() {
  unsigned* d;
  unsigned h[128];
  (void)hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l : {0, 31, 32, 63}) printf("lane %2d: a %3u b %3u\n", l, h[l], h[64 + l]);
  return 0;
}
