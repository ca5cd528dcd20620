// Diagonal-block factorisation of the blocked Cholesky: one 512-thread workgroup per batch
// member factors the 128 x 128 block at (j0, j0) of W in LDS and inverts the factor.
//
// The block is handled as 8 x 8 tiles of 16 x 16, every tile operation an f64 MFMA chain
// (v_mfma_f64_16x16x4_f64, 4 MFMAs per 16-deep product):
//   for kb = 0..7:
//     wave 0   : potf2 of tile (kb, kb) in registers (lane r owns row r, columns broadcast
//                through LDS) and its inverse Dinv_kb
//     waves    : panel tiles  X_i = A_{i,kb} Dinv_kb^T                  (i > kb)
//     waves    : trailing     A_{i,j} -= X_i X_j^T                      (kb < j <= i)
//   inverse by block rows (I = 0..7), one wave per tile column J < I:
//     Linv_{I,J} = -Dinv_I (sum_{K=J}^{I-1} L_{I,K} Linv_{K,J}),   Linv_{I,I} = Dinv_I
// The f64 C/D layout (col = lane & 15, row = (lane >> 4) + 4 reg) equals the B-operand layout
// of k-step s = reg, so the inner product T stays in registers between the two MFMA chains.
//
// Writes L_kk to W (lower triangle) and L_kk^-1 (zeros above the diagonal) to Winv; the first
// non-positive pivot (1-based global column) goes to info[b] (LAPACK convention, as the
// InvalidArgumentError of tf.linalg.cholesky at gpbasics/Statistics/CovarianceMatrix.py:250).
//
// The device code (block load, potf2, tile operations, inverse, stores) lives in gpk_diag_dev.h, shared
// with the persistent factorisation of gpk_potrf.hip.
#include "gpk_diag_dev.h"

namespace gpk {
namespace {

template <typename T>
__global__ __launch_bounds__(DT) void diag_kernel(DiagArgs a) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* A = sm;
  double* Dinv = A + LDS_A;
  double* colbuf = Dinv + LDS_DINV;
  int* flag = reinterpret_cast<int*>(colbuf + LDS_COL);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int lr = lane & 15;       // MFMA operand row / C-D column
  const int lk = lane >> 4;       // MFMA operand k within a 4-step / C-D row offset
  const int b = blockIdx.x;
  T* Wb = reinterpret_cast<T*>(a.W) + (int64_t)b * a.w_bs + a.j0 * a.ld + a.j0;
  constexpr int PER = NB * NB / DT;
#ifndef GPK_DIAG_LOAD_BATCH
#define GPK_DIAG_LOAD_BATCH 16
#endif
  {
    // GPK_DIAG_LOAD_BATCH loads in flight per thread before their LDS stores (a plain loop
    // serialises load / store; all 32 at once costs more registers than the kernel has)
    constexpr int LB = GPK_DIAG_LOAD_BATCH;
    const T* src = Wb + (int64_t)(tid >> 7) * a.ld + (tid & (NB - 1));
    const int64_t step = (int64_t)(DT / NB) * a.ld;  // rows advanced per q
    const int c = tid & (NB - 1);
#pragma unroll
    for (int g = 0; g < PER; g += LB) {
      double v[LB];
#pragma unroll
      for (int q = 0; q < LB; ++q) v[q] = (double)src[(g + q) * step];
#pragma unroll
      for (int q = 0; q < LB; ++q) {
        const int r = (tid >> 7) + (g + q) * (DT / NB);
        A[aidx(r, c)] = (c <= r) ? v[q] : 0.0;
      }
    }
  }
  if (tid == 0) *flag = 0;
  __syncthreads();

#pragma unroll 1
  for (int kb = 0; kb < NTL; ++kb) {
    double* Dk = Dinv + kb * DTS;
    if (wave == 0 && !(a.dbg & 2)) potf2_tile(A, Dk, colbuf, kb, lane, flag, a.j0);
    if (a.dbg & 4) continue;
    __syncthreads();
    if (kb == NTL - 1) break;
    // panel: X_i = A_{i,kb} * Dinv_kb^T   (B[k][c] = Dinv[c][k])
    {
      const int i = kb + 1 + wave;
      if (i < NTL) {
        d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const double av = A[aidx(i * DB + lr, kb * DB + 4 * s + lk)];
          const double bv = Dk[lr * DBS + 4 * s + lk];
          acc = mfma64(av, bv, acc);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) A[aidx(i * DB + lk + 4 * q, kb * DB + lr)] = acc[q];
      }
    }
    __syncthreads();
    // trailing tiles (i, j), kb < j <= i: A_ij -= X_i X_j^T
    {
      const int m = NTL - 1 - kb;
      const int ntri = m * (m + 1) / 2;
      for (int t = wave; t < ntri; t += DT / 64) {
        int ti = 0;
        while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
        const int tj = t - ti * (ti + 1) / 2;
        const int i = kb + 1 + ti, j = kb + 1 + tj;
        d4 acc;
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = A[aidx(i * DB + lk + 4 * q, j * DB + lr)];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const double av = -A[aidx(i * DB + lr, kb * DB + 4 * s + lk)];
          const double bv = A[aidx(j * DB + lr, kb * DB + 4 * s + lk)];
          acc = mfma64(av, bv, acc);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) A[aidx(i * DB + lk + 4 * q, j * DB + lr)] = acc[q];
      }
    }
    __syncthreads();
  }

  // L_kk back to W (lower triangle only)
  for (int e = tid; e < NB * NB; e += DT) {
    const int r = e >> 7, c = e & (NB - 1);
    if (c <= r) Wb[(int64_t)r * a.ld + c] = (T)A[aidx(r, c)];
  }
  if (tid == 0 && *flag != 0) atomicCAS(&a.info[b], 0, *flag);

  // inverse by 16-row blocks, in place (block rows < I of A hold Linv, row I still holds L)
  for (int I = 0; I < ((a.dbg & 1) ? 0 : NTL); ++I) {
    const int J = wave;
    const bool active = J < I;
    d4 out = {0.0, 0.0, 0.0, 0.0};
    if (active) {
      d4 tacc = {0.0, 0.0, 0.0, 0.0};
      for (int K = J; K < I; ++K) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const double av = A[aidx(I * DB + lr, K * DB + 4 * s + lk)];
          const double bv = A[aidx(K * DB + 4 * s + lk, J * DB + lr)];
          tacc = mfma64(av, bv, tacc);
        }
      }
      const double* Di = Dinv + I * DTS;
#pragma unroll
      for (int s = 0; s < 4; ++s) out = mfma64(-Di[lr * DBS + 4 * s + lk], tacc[s], out);
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int q = 0; q < 4; ++q) A[aidx(I * DB + lk + 4 * q, J * DB + lr)] = out[q];
    }
    if (wave == NTL - 1) {
      const double* Di = Dinv + I * DTS;
      for (int e = lane; e < DB * DB; e += 64) A[aidx(I * DB + e / DB, I * DB + e % DB)] = Di[(e / DB) * DBS + e % DB];
    }
    __syncthreads();
  }
  T* Ib = reinterpret_cast<T*>(a.Winv) + (int64_t)b * a.inv_bs + a.kblk * NB * NB;
  for (int e = tid; e < NB * NB; e += DT) {
    const int r = e >> 7, c = e & (NB - 1);
    Ib[e] = (T)((c <= r) ? A[aidx(r, c)] : 0.0);
  }
}

template <typename T, bool FUSE, bool SC1 = false>
__global__ __launch_bounds__(DT) void diag2_kernel(DiagArgs a) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  diag2_body<T, FUSE, SC1>(a, (int)blockIdx.x, sm);
}

}  // namespace

hipError_t launch_diag(const DiagArgs& a, int dtype, int32_t batch, hipStream_t s) {
  const bool v2 = a.version != 1;
  const bool fuse = v2 && dtype == GPK_F64 && a.trsm_tiles > 0;
  const void* fn = fuse ? reinterpret_cast<const void*>(diag2_kernel<double, true>)
                 : v2 ? (dtype == GPK_F64 ? reinterpret_cast<const void*>(diag2_kernel<double, false>)
                                          : reinterpret_cast<const void*>(diag2_kernel<float, false>))
                      : (dtype == GPK_F64 ? reinterpret_cast<const void*>(diag_kernel<double>)
                                          : reinterpret_cast<const void*>(diag_kernel<float>));
  {
    hipError_t e = ensure_dyn_lds(fn, DIAG_LDS_BYTES);
    if (e != hipSuccess) return e;
  }
  if (a.version == 3 && dtype == GPK_F64 && !fuse) {  // debugging: the write-through (chain_kernel) variant
    hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(diag2_kernel<double, false, true>), DIAG_LDS_BYTES);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((diag2_kernel<double, false, true>), dim3(batch), dim3(DT), DIAG_LDS_BYTES, s, a);
  } else if (fuse) {
    hipLaunchKernelGGL((diag2_kernel<double, true>), dim3(a.trsm_tiles + 1, batch), dim3(DT), DIAG_LDS_BYTES, s, a);
  } else if (v2) {
    if (dtype == GPK_F64)
      hipLaunchKernelGGL((diag2_kernel<double, false>), dim3(batch), dim3(DT), DIAG_LDS_BYTES, s, a);
    else
      hipLaunchKernelGGL((diag2_kernel<float, false>), dim3(batch), dim3(DT), DIAG_LDS_BYTES, s, a);
  } else if (dtype == GPK_F64) {
    hipLaunchKernelGGL(diag_kernel<double>, dim3(batch), dim3(DT), DIAG_LDS_BYTES, s, a);
  } else {
    hipLaunchKernelGGL(diag_kernel<float>, dim3(batch), dim3(DT), DIAG_LDS_BYTES, s, a);
  }
  return hipGetLastError();
}

}  // namespace gpk
