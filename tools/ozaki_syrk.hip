// Prototype: the trailing update C = P P^T (lower 128 x 128 tiles) emulated on the int8 MFMA (Ozaki
// scheme I) -- the measurement behind DESIGN.md §8 item 3, not part of libgpk.
//
// Every row of P is scaled by a power of two so that |r| < 1/2 and split into S signed 7-bit digits
// (P = sc diag sum_s 2^-7(s+1) Q_s, Q_s in [-64, 64]); C = diag(sc) [sum_d 2^-7(d+2) sum_{s+t=d} Q_s Q_t^T] diag(sc)
// keeps the digit pairs s + t < S.  Each Q_s Q_t^T is an exact int8 x int8 -> int32 product
// (v_mfma_i32_16x16x64_i8); the pairs of one d share one int32 accumulator (|sum| <= S K 64^2 < 2^31),
// converted to fp64 once per d.  Operands are read straight from global memory (L2): no LDS staging.
//
// build+run (GPU box): hipcc --offload-arch=gfx950 -O3 tools/ozaki_syrk.hip -o /tmp/oz && /tmp/oz [rows] [S] [staged 0/1]
// Prints the max relative error of sampled tiles against an fp64 host product and the emulated
// rate (2 K x lower elements / kernel time, the f64 update's algorithmic count).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

typedef int i4 __attribute__((ext_vector_type(4)));
typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int KD = 1024;  // panel depth (one group of 8 panels of 128)
constexpr int MAXS = 8;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

// one 256-thread block per row: exponent of the row maximum, then S digits per element
__global__ __launch_bounds__(256) void slice_rows(const double* P, int rows, int S, signed char* Q, double* sc) {
  __shared__ double red[256];
  const int r = blockIdx.x, tid = threadIdx.x;
  const double* p = P + (size_t)r * KD;
  double mx = 0.0;
  for (int k = tid; k < KD; k += 256) mx = fmax(mx, fabs(p[k]));
  red[tid] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] = fmax(red[tid], red[tid + s]);
    __syncthreads();
  }
  int e = 0;
  if (red[0] > 0.0) frexp(red[0], &e);  // max = f 2^e, f in [0.5, 1)
  const double scale = ldexp(1.0, e + 1);  // |p / scale| < 1/2
  if (tid == 0) sc[r] = scale;
  for (int k = tid; k < KD; k += 256) {
    double rem = p[k] / scale;
    for (int s = 0; s < S; ++s) {
      const double qv = rint(ldexp(rem, 7 * (s + 1)));
      Q[((size_t)s * rows + r) * KD + k] = (signed char)qv;
      rem -= ldexp(qv, -7 * (s + 1));
    }
  }
}

// lower 128 x 128 tiles, 512 threads = 2 x 4 waves of 64 x 32 (4 x 2 blocks of 16 x 16)
__global__ __launch_bounds__(512) void syrk_i8(const signed char* Q, const double* sc, int rows, int S, double* C) {
  const int t = blockIdx.x;
  int ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while (ti * (ti + 1) / 2 > t) --ti;
  while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
  const int tj = t - ti * (ti + 1) / 2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 2, wc = w & 3;
  const int lr = lane & 15, q = lane >> 4;
  d4 accd[4][2];
  for (int m = 0; m < 4; ++m)
    for (int n = 0; n < 2; ++n) accd[m][n] = d4{0, 0, 0, 0};
  for (int d = 0; d < S; ++d) {
    i4 acci[4][2];
    for (int m = 0; m < 4; ++m)
      for (int n = 0; n < 2; ++n) acci[m][n] = i4{0, 0, 0, 0};
    for (int s = 0; s <= d; ++s) {
      const int tt = d - s;
      const signed char* Qa = Q + (size_t)s * rows * KD;
      const signed char* Qb = Q + (size_t)tt * rows * KD;
      for (int k0 = 0; k0 < KD; k0 += 64) {
        i4 fa[4], fb[2];
#pragma unroll
        for (int m = 0; m < 4; ++m)
          fa[m] = *reinterpret_cast<const i4*>(Qa + (size_t)(ti * 128 + wr * 64 + m * 16 + lr) * KD + k0 + 16 * q);
#pragma unroll
        for (int n = 0; n < 2; ++n)
          fb[n] = *reinterpret_cast<const i4*>(Qb + (size_t)(tj * 128 + wc * 32 + n * 16 + lr) * KD + k0 + 16 * q);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) acci[m][n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[m], fb[n], acci[m][n], 0, 0, 0);
      }
    }
    const double f = ldexp(1.0, -7 * (d + 2));
    for (int m = 0; m < 4; ++m)
      for (int n = 0; n < 2; ++n)
        for (int r = 0; r < 4; ++r) accd[m][n][r] += f * (double)acci[m][n][r];
  }
  for (int m = 0; m < 4; ++m)
    for (int n = 0; n < 2; ++n)
      for (int r = 0; r < 4; ++r) {
        const int gi = ti * 128 + wr * 64 + m * 16 + 4 * q + r;  // 16x16 int32 C/D: row = 4 (lane >> 4) + reg
        const int gj = tj * 128 + wc * 32 + n * 16 + lr;
        C[(size_t)gi * rows + gj] = sc[gi] * sc[gj] * accd[m][n][r];
      }
}

// LDS-staged variant: per 64-byte K chunk the (d + 1) slices of the tile's A rows and B rows needed by
// the digit pairs of d are staged once (row stride 80 B: a quarter-wave's 16-B reads hit distinct banks)
// and shared by the 8 waves; one workgroup per CU at S = 6 (123 KB of LDS).
constexpr int RS = 80;  // LDS row stride (bytes)

__global__ __launch_bounds__(512) void syrk_i8_lds(const signed char* Q, const double* sc, int rows, int S, double* C) {
  extern __shared__ __attribute__((aligned(16))) signed char lds[];
  signed char* La = lds;                          // [S][128][RS]
  signed char* Lb = lds + (size_t)S * 128 * RS;   // [S][128][RS]
  const int t = blockIdx.x;
  int ti = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while (ti * (ti + 1) / 2 > t) --ti;
  while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
  const int tj = t - ti * (ti + 1) / 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 2, wc = w & 3;
  const int lr = lane & 15, q = lane >> 4;
  const int lrow = tid >> 2, lpc = tid & 3;  // loader: row 0..127, 16-B piece 0..3
  d4 accd[4][2];
  for (int m = 0; m < 4; ++m)
    for (int n = 0; n < 2; ++n) accd[m][n] = d4{0, 0, 0, 0};
  for (int d = 0; d < S; ++d) {
    i4 acci[4][2];
    for (int m = 0; m < 4; ++m)
      for (int n = 0; n < 2; ++n) acci[m][n] = i4{0, 0, 0, 0};
    for (int k0 = 0; k0 < KD; k0 += 64) {
      for (int s = 0; s <= d; ++s) {
        const signed char* qa = Q + ((size_t)s * rows + ti * 128 + lrow) * KD + k0 + 16 * lpc;
        const signed char* qb = Q + ((size_t)s * rows + tj * 128 + lrow) * KD + k0 + 16 * lpc;
        *reinterpret_cast<i4*>(La + ((size_t)s * 128 + lrow) * RS + 16 * lpc) = *reinterpret_cast<const i4*>(qa);
        *reinterpret_cast<i4*>(Lb + ((size_t)s * 128 + lrow) * RS + 16 * lpc) = *reinterpret_cast<const i4*>(qb);
      }
      __syncthreads();
      for (int s = 0; s <= d; ++s) {
        const int tt = d - s;
        i4 fa[4], fb[2];
#pragma unroll
        for (int m = 0; m < 4; ++m)
          fa[m] = *reinterpret_cast<const i4*>(La + ((size_t)s * 128 + wr * 64 + m * 16 + lr) * RS + 16 * q);
#pragma unroll
        for (int n = 0; n < 2; ++n)
          fb[n] = *reinterpret_cast<const i4*>(Lb + ((size_t)tt * 128 + wc * 32 + n * 16 + lr) * RS + 16 * q);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n) acci[m][n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa[m], fb[n], acci[m][n], 0, 0, 0);
      }
      __syncthreads();
    }
    const double f = ldexp(1.0, -7 * (d + 2));
    for (int m = 0; m < 4; ++m)
      for (int n = 0; n < 2; ++n)
        for (int r = 0; r < 4; ++r) accd[m][n][r] += f * (double)acci[m][n][r];
  }
  for (int m = 0; m < 4; ++m)
    for (int n = 0; n < 2; ++n)
      for (int r = 0; r < 4; ++r) {
        const int gi = ti * 128 + wr * 64 + m * 16 + 4 * q + r;
        const int gj = tj * 128 + wc * 32 + n * 16 + lr;
        C[(size_t)gi * rows + gj] = sc[gi] * sc[gj] * accd[m][n][r];
      }
}

int main(int argc, char** argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 4096;
  const int S = argc > 2 ? atoi(argv[2]) : 6;
  if (rows % 128 || S < 1 || S > MAXS) return 2;
  std::vector<double> P((size_t)rows * KD);
  srand(7);
  for (int i = 0; i < rows; ++i) {
    const double rs = pow(10.0, -3.0 * (double)rand() / RAND_MAX);  // rows of very different size
    for (int k = 0; k < KD; ++k) {
      const double u1 = (rand() + 1.0) / (RAND_MAX + 2.0), u2 = (rand() + 1.0) / (RAND_MAX + 2.0);
      P[(size_t)i * KD + k] = rs * sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2) * 0.03;
    }
  }
  double *dP, *dsc, *dC;
  signed char* dQ;
  CHECK(hipMalloc(&dP, P.size() * 8));
  CHECK(hipMalloc(&dsc, rows * 8));
  CHECK(hipMalloc(&dC, (size_t)rows * rows * 8));
  CHECK(hipMalloc(&dQ, (size_t)S * rows * KD));
  CHECK(hipMemcpy(dP, P.data(), P.size() * 8, hipMemcpyHostToDevice));
  const int tiles = (rows / 128) * (rows / 128 + 1) / 2;
  hipEvent_t e0, e1, e2;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventCreate(&e2));
  const bool staged = argc > 3 && atoi(argv[3]) == 1;
  const size_t lds = (size_t)2 * S * 128 * RS;
  if (staged)
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(syrk_i8_lds), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds));
  auto syrk = [&]() {
    if (staged)
      hipLaunchKernelGGL(syrk_i8_lds, dim3(tiles), dim3(512), lds, 0, dQ, dsc, rows, S, dC);
    else
      hipLaunchKernelGGL(syrk_i8, dim3(tiles), dim3(512), 0, 0, dQ, dsc, rows, S, dC);
  };
  hipLaunchKernelGGL(slice_rows, dim3(rows), dim3(256), 0, 0, dP, rows, S, dQ, dsc);
  syrk();  // warm
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(slice_rows, dim3(rows), dim3(256), 0, 0, dP, rows, S, dQ, dsc);
  CHECK(hipEventRecord(e1));
  syrk();
  CHECK(hipEventRecord(e2));
  CHECK(hipEventSynchronize(e2));
  float ms_slice, ms_syrk;
  CHECK(hipEventElapsedTime(&ms_slice, e0, e1));
  CHECK(hipEventElapsedTime(&ms_syrk, e1, e2));
  std::vector<double> C((size_t)rows * rows);
  CHECK(hipMemcpy(C.data(), dC, C.size() * 8, hipMemcpyDeviceToHost));
  // sampled tiles against the fp64 host product: error relative to sum_k |p_ik p_jk|
  double worst = 0.0;
  const int nt = rows / 128;
  const int samples[4][2] = {{0, 0}, {nt - 1, 0}, {nt - 1, nt - 1}, {nt / 2, nt / 3}};
  for (auto& sp : samples) {
    for (int i = sp[0] * 128; i < sp[0] * 128 + 128; i += 7)
      for (int j = sp[1] * 128; j < sp[1] * 128 + 128; j += 5) {
        double ref = 0.0, mag = 0.0;
        for (int k = 0; k < KD; ++k) {
          ref += P[(size_t)i * KD + k] * P[(size_t)j * KD + k];
          mag += fabs(P[(size_t)i * KD + k] * P[(size_t)j * KD + k]);
        }
        const double err = fabs(C[(size_t)i * rows + j] - ref) / mag;
        if (err > worst) worst = err;
      }
  }
  const double lower = (double)tiles * 128.0 * 128.0;
  printf("%s rows %d K %d S %d (int8 GEMMs %d): max err / sum|p p| %.3e; slice %.3f ms, emulated syrk %.3f ms = %.1f TF/s "
         "fp64-equivalent (%.0f int8 TOP/s issued)\n",
         staged ? "lds " : "l2  ", rows, KD, S, S * (S + 1) / 2, worst, ms_slice, ms_syrk, 2.0 * KD * lower / (ms_syrk * 1e-3) / 1e12,
         2.0 * KD * lower * (S * (S + 1) / 2) / (ms_syrk * 1e-3) / 1e12);
  return worst < 1e-10 || S < 5 ? 0 : 3;
}
