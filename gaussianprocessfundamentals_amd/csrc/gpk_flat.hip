// Kernels behind the caller-matrix entries of the SURVEY §8(b) sketch (gpk_potrf_lower in fp32,
// gpk_trsv_lower and gpk_posterior on a caller's factor L): moving a caller matrix into / out of the augmented
// layout, inverting the 128 x 128 diagonal blocks of a caller L (the Winv the blocked solves multiply by), and
// the diagonal read-out of the posterior variance.
#include "gpk_internal.h"

namespace gpk {
namespace {

// the augmented matrix [p, p] (ld = p) of a caller matrix A [n, lda] with no extra rows and y = 0: lower
// triangle of A in the training block, identity on the padding rows n .. n_pad - 1, zero elsewhere (the y row
// and the rows below it included)
template <typename T>
__global__ __launch_bounds__(256) void pack_lower_kernel(const T* __restrict__ A, int64_t lda, int64_t n,
                                                         int64_t n_pad, int64_t p, T* __restrict__ W) {
  const int64_t r = blockIdx.y;
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= p) return;
  T v = T(0);
  if (r < n && c < n) v = c <= r ? A[r * lda + c] : T(0);
  else if (r == c && r < n_pad) v = T(1);
  W[r * p + c] = v;
}

// lower triangle of W (ld) back into the caller's A [n, lda]; A's upper triangle untouched
template <typename T>
__global__ __launch_bounds__(256) void unpack_lower_kernel(const T* __restrict__ W, int64_t ld, int64_t n,
                                                           T* __restrict__ A, int64_t lda) {
  const int64_t r = blockIdx.y;
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c > r || r >= n) return;
  A[r * lda + c] = W[r * ld + c];
}

// Winv[kb] = (L_kb,kb)^-1, row-major NB x NB, of a caller lower-triangular L [n, ldl] (the last block padded
// with identity): forward substitution, column j of the inverse by thread j; workgroup = (block kb, half h of
// the columns).  LDS: the block's lower triangle packed by rows (NB (NB + 1) / 2) + the half's columns [NB][64].
__global__ __launch_bounds__(64) void trtri_blocks_kernel(const double* __restrict__ L, int64_t ldl, int64_t n,
                                                          double* __restrict__ Winv) {
  extern __shared__ __attribute__((aligned(16))) double sh[];
  double* Lp = sh;
  double* X = sh + NB * (NB + 1) / 2;
  const int kb = blockIdx.x >> 1, h = blockIdx.x & 1, tid = threadIdx.x;
  const int64_t j0 = (int64_t)kb * NB;
  const int nv = (int)((n - j0) < NB ? (n - j0) : NB);
  for (int i = 0; i < NB; ++i)
    for (int k = tid; k <= i; k += 64)
      Lp[i * (i + 1) / 2 + k] = (i < nv && k < nv) ? L[(j0 + i) * ldl + j0 + k] : (i == k ? 1.0 : 0.0);
  __syncthreads();
  const int j = h * 64 + tid;
  for (int i = 0; i < NB; ++i) {
    double s = (i == j) ? 1.0 : 0.0;
    if (i > j) {
      const double* Li = Lp + i * (i + 1) / 2;
      double s1 = 0.0;
      int k = j;
      for (; k + 1 < i; k += 2) {
        s = fma(-Li[k], X[k * 64 + tid], s);
        s1 = fma(-Li[k + 1], X[(k + 1) * 64 + tid], s1);
      }
      if (k < i) s = fma(-Li[k], X[k * 64 + tid], s);
      s += s1;
    }
    X[i * 64 + tid] = (i >= j) ? s / Lp[i * (i + 1) / 2 + i] : 0.0;
  }
  double* out = Winv + (int64_t)kb * NB * NB;
  for (int i = 0; i < NB; ++i) out[i * NB + j] = X[i * 64 + tid];
}

// var[j] = kdiag[0] - sum_i V[i][j]^2 over the n rows of V [n, m] (ld m): the diagonal of K_ss - V^T V
__global__ __launch_bounds__(256) void posterior_var_kernel(const double* __restrict__ V, int64_t n, int64_t m,
                                                            const double* __restrict__ kdiag, double* __restrict__ var) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= m) return;
  double s0 = 0.0, s1 = 0.0;
  int64_t i = 0;
  for (; i + 1 < n; i += 2) {
    const double a = V[i * m + j], b = V[(i + 1) * m + j];
    s0 = fma(a, a, s0);
    s1 = fma(b, b, s1);
  }
  if (i < n) {
    const double a = V[i * m + j];
    s0 = fma(a, a, s0);
  }
  var[j] = kdiag[0] - (s0 + s1);
}

}  // namespace

hipError_t launch_pack_lower(int dtype, const void* A, int64_t lda, int64_t n, int64_t n_pad, int64_t p, void* W,
                             hipStream_t s) {
  dim3 grid((unsigned)((p + 255) / 256), (unsigned)p);
  if (dtype == GPK_F64)
    hipLaunchKernelGGL(pack_lower_kernel<double>, grid, dim3(256), 0, s, static_cast<const double*>(A), lda, n,
                       n_pad, p, static_cast<double*>(W));
  else
    hipLaunchKernelGGL(pack_lower_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(A), lda, n,
                       n_pad, p, static_cast<float*>(W));
  return hipGetLastError();
}

hipError_t launch_unpack_lower(int dtype, const void* W, int64_t ld, int64_t n, void* A, int64_t lda, hipStream_t s) {
  dim3 grid((unsigned)((n + 255) / 256), (unsigned)n);
  if (dtype == GPK_F64)
    hipLaunchKernelGGL(unpack_lower_kernel<double>, grid, dim3(256), 0, s, static_cast<const double*>(W), ld, n,
                       static_cast<double*>(A), lda);
  else
    hipLaunchKernelGGL(unpack_lower_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(W), ld, n,
                       static_cast<float*>(A), lda);
  return hipGetLastError();
}

size_t trtri_blocks_lds() { return sizeof(double) * ((size_t)NB * (NB + 1) / 2 + (size_t)NB * 64); }

hipError_t launch_trtri_blocks(const double* L, int64_t ldl, int64_t n, double* Winv, hipStream_t s) {
  {
    hipError_t err = ensure_dyn_lds(reinterpret_cast<const void*>(trtri_blocks_kernel), trtri_blocks_lds());
    if (err != hipSuccess) return err;
  }
  const int64_t nblk = (n + NB - 1) / NB;
  hipLaunchKernelGGL(trtri_blocks_kernel, dim3((unsigned)(2 * nblk)), dim3(64), trtri_blocks_lds(), s, L, ldl, n, Winv);
  return hipGetLastError();
}

hipError_t launch_posterior_var(const double* V, int64_t n, int64_t m, const double* kdiag, double* var,
                                hipStream_t s) {
  hipLaunchKernelGGL(posterior_var_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, V, n, m, kdiag, var);
  return hipGetLastError();
}

}  // namespace gpk
