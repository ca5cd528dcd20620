// Cycles of the diagonal block's 16 x 16 pivot-tile factorisation (potf2_tile of gpk_diag_dev.h) on one wave,
// the tile in LDS, 64 repetitions (s_memtime).  Build variants with -DGPK_PIPE_NEWTON=1, -DGPK_PIPE_NOINV=1,
// -DGPK_PIPE_NOBAD=1, -DGPK_POTF2_MODE=0 to split the time.
#include <cstdio>
#include "gpk_diag_dev.h"

namespace gpk {
__global__ __launch_bounds__(64) void potf2_probe(const double* M, double* out, unsigned long long* cyc) {
  __shared__ double A[NB * LDA];
  __shared__ double Dk[DTS];
  __shared__ double colbuf[LDS_COL];
  __shared__ int flag;
  const int lane = threadIdx.x;
  unsigned long long t0 = 0, t1 = 0;
  for (int rep = 0; rep < 65; ++rep) {
    for (int e = lane; e < DB * DB; e += 64) A[aidx(e / DB, e % DB)] = M[e];
    if (lane == 0) flag = 0;
    __syncthreads();
    if (rep == 1) t0 = __builtin_amdgcn_s_memtime();
    potf2_tile(A, Dk, colbuf, 0, lane, &flag, 0);
    __syncthreads();
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[0] = t1 - t0;
  for (int e = lane; e < DB * DB; e += 64) out[e] = A[aidx(e / DB, e % DB)] + Dk[(e / DB) * DBS + e % DB];
}
}  // namespace gpk

int main() {
  double h[256];
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) h[i * 16 + j] = (i == j ? 16.0 : 0.0) + 1.0 / (1.0 + i + j);
  double *M, *out;
  unsigned long long* cyc;
  (void)hipMalloc(&M, sizeof(h));
  (void)hipMalloc(&out, sizeof(h));
  (void)hipMalloc(&cyc, 8);
  (void)hipMemcpy(M, h, sizeof(h), hipMemcpyHostToDevice);
  unsigned long long c = 0;
  for (int it = 0; it < 3; ++it) {
    hipLaunchKernelGGL(gpk::potf2_probe, dim3(1), dim3(64), 0, 0, M, out, cyc);
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  }
  double o[256];
  (void)hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
  printf("%-14s %7.0f cycles per 16 x 16 tile (L[15][15] + Dinv[15][15] = %.15f)\n", VARIANT, c / 64.0, o[255]);
  return 0;
}
