// Microbenchmark: sustained MFMA / VALU rates on gfx950 (operands in registers, no memory).
// Build+run on the GPU box:  hipcc --offload-arch=gfx950 -O3 tools/mfma_peak.hip -o /tmp/mfma_peak && /tmp/mfma_peak
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void mfma_f64(double* out, double s) {
  d4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = s + threadIdx.x, b = s * 0.5;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double r = 0;
  for (int i = 0; i < 8; ++i) r += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (r == 12345.0) out[0] = r;
}

__global__ __launch_bounds__(256) void mfma_f32(float* out, float s) {
  f4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f4{0, 0, 0, 0};
  float a = s + threadIdx.x, b = s * 0.5f;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  float r = 0;
  for (int i = 0; i < 8; ++i) r += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (r == 12345.0f) out[0] = r;
}

typedef int i4 __attribute__((ext_vector_type(4)));

// int8 MFMA 16x16x64 (the Ozaki-scheme candidate for fp64 emulation): random-ish operands
__global__ __launch_bounds__(256) void mfma_i8(int* out, int s) {
  i4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = i4{0, 0, 0, 0};
  const int x = s * 0x01234567 + (int)threadIdx.x * 0x3a5b7c9d;
  i4 a = {x, x ^ 0x5a5a5a5a, x * 3, x + 0x11111111}, b = {x * 7, x ^ 0x0f0f0f0f, x + 12345, ~x};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[i], 0, 0, 0);
  }
  int r = 0;
  for (int i = 0; i < 8; ++i) r += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (r == 12345) out[0] = r;
}

__global__ __launch_bounds__(256) void valu_f64(double* out, double s) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = s + i + threadIdx.x;
  const double m = 0.999999, c = 1e-7;
  for (int it = 0; it < ITERS * 4; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = fma(x[i], m, c);
  }
  double r = 0;
  for (int i = 0; i < 8; ++i) r += x[i];
  if (r == 12345.0) out[0] = r;
}

template <typename K, typename T>
double run(K kern, T* buf, double flops_per_thread_iter, int waves_per_simd) {
  int blocks = 256 * waves_per_simd;  // 256 threads = 1 wave per SIMD per block
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, (T)1.0);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, (T)1.0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double flops = 5.0 * blocks * 256.0 * flops_per_thread_iter;
  return flops / (ms * 1e-3) / 1e12;
}

int main() {
  double* d;
  float* f;
  int* i;
  (void)hipMalloc(&d, 64);
  (void)hipMalloc(&f, 64);
  (void)hipMalloc(&i, 64);
  // per wave MFMA 16x16x4: 2*16*16*4 = 2048 flop -> per thread 32 flop per instruction
  for (int w = 1; w <= 2; ++w) {
    printf("f64 MFMA 16x16x4, %d wave/SIMD: %.1f TFLOP/s\n", w, run(mfma_f64, d, 8.0 * ITERS * 32.0, w));
    printf("f32 MFMA 16x16x4, %d wave/SIMD: %.1f TFLOP/s\n", w, run(mfma_f32, f, 8.0 * ITERS * 32.0, w));
    printf("f64 VALU fma,     %d wave/SIMD: %.1f TFLOP/s\n", w, run(valu_f64, d, 8.0 * ITERS * 4 * 2.0, w));
    // per wave 16x16x64: 2*16*16*64 = 32768 op -> per thread 512 op per instruction
    printf("i8 MFMA 16x16x64, %d wave/SIMD: %.1f TOP/s\n", w, run(mfma_i8, i, 8.0 * ITERS * 512.0, w));
  }
  return 0;
}
