// Debug harness: run potf2_tile on one 16 x 16 SPD tile and print L and L^-1 errors.
#include "../../gaussianprocessfundamentals_amd/csrc/gpk_diag.hip"
#include <cstdio>
#include <cmath>
#include <vector>

namespace gpk { namespace {
__global__ void potf2_probe(const double* in, double* Lout, double* Dout) {
  extern __shared__ double sm[];
  double* A = sm;
  double* Dinv = A + LDS_A;
  double* colbuf = Dinv + LDS_DINV;
  int* flag = reinterpret_cast<int*>(colbuf + LDS_COL);
  const int lane = threadIdx.x;
  for (int e = lane; e < 256; e += 64) A[(e / 16) * LDA + e % 16] = in[e];
  if (lane == 0) *flag = 0;
  __syncthreads();
  potf2_tile(A, Dinv, colbuf, 0, lane, flag, 0);
  __syncthreads();
  for (int e = lane; e < 256; e += 64) { Lout[e] = A[(e / 16) * LDA + e % 16]; Dout[e] = Dinv[e]; }
}
} }

int main() {
  std::vector<double> A(256), L(256), D(256);
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) A[i * 16 + j] = (i == j ? 20.0 : 0.0) + 1.0 / (1 + i + j);
  double *dA, *dL, *dD;
  hipMalloc(&dA, 2048); hipMalloc(&dL, 2048); hipMalloc(&dD, 2048);
  hipMemcpy(dA, A.data(), 2048, hipMemcpyHostToDevice);
  const size_t lds = sizeof(double) * (gpk::LDS_A + gpk::LDS_DINV + gpk::LDS_COL) + 16;
  hipFuncSetAttribute((const void*)gpk::potf2_probe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(gpk::potf2_probe, dim3(1), dim3(64), lds, 0, dA, dL, dD);
  hipMemcpy(L.data(), dL, 2048, hipMemcpyDeviceToHost);
  hipMemcpy(D.data(), dD, 2048, hipMemcpyDeviceToHost);
  double eL = 0, eD = 0;
  for (int i = 0; i < 16; ++i) for (int j = 0; j <= i; ++j) {
    double s = 0; for (int k = 0; k <= j; ++k) s += L[i * 16 + k] * L[j * 16 + k];
    eL = fmax(eL, fabs(s - A[i * 16 + j]));
  }
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
    double s = 0; for (int k = 0; k < 16; ++k) s += D[i * 16 + k] * (k >= j ? L[k * 16 + j] : 0.0);
    eD = fmax(eD, fabs(s - (i == j)));
  }
  printf("LL^T err %.3e   Dinv L - I err %.3e\n", eL, eD);
  printf("D row0: "); for (int j = 0; j < 4; ++j) printf("%g ", D[j]); printf("\n");
  printf("D row1: "); for (int j = 0; j < 4; ++j) printf("%g ", D[16 + j]); printf("\n");
  printf("D row2: "); for (int j = 0; j < 4; ++j) printf("%g ", D[32 + j]); printf("\n");
  printf("L diag: "); for (int j = 0; j < 4; ++j) printf("%g ", L[j * 17]); printf("\n");
  return 0;
}
