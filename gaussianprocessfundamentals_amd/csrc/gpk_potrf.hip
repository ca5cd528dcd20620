// Blocked right-looking Cholesky of the augmented matrix W (see include/gpk.h), plus the
// read-out and the triangular solves.
//
// Replaces tf.linalg.cholesky / tf.linalg.triangular_solve of
// gpbasics/Statistics/CovarianceMatrix.py:247-265 and the log-determinant / data-fit
// assembly of gpbasics/Metrics/Metrics.py:152-154 and gpbasics/Metrics/LogLikelihood.py:30-65.
//
// Per panel step k (columns j0 = 128k .. j0+127):
//   diag_kernel      one workgroup per batch member factors the 128 x 128 diagonal block in
//                    LDS (inner 16-blocks: register potf2 by one wave + parallel panel solve and
//                    rank-16 update), then inverts it (row-block recursion on the 16-block
//                    inverses).  Writes L_kk to W and L_kk^-1 to Winv.
//   gemm<TRSM>       rows below the block: W[R, j0:j0+128] <- W[R, j0:j0+128] * L_kk^-T
//                    (an MFMA GEMM against the inverted block; every row of the augmented
//                    matrix, so z = L^-1 y and V^T = Ks^T L^-T come out of the same launch)
//   gemm<UPDATE>     lower tiles of the trailing matrix: C -= P P^T on f64 MFMA
//                    (v_mfma_f64_16x16x4_f64) or f32 MFMA (v_mfma_f32_16x16x4_f32)
#include <math.h>

#include "gpk_internal.h"

namespace gpk {
namespace {

constexpr int DB = 16;         // inner block of the diagonal factorisation
constexpr int LDA = NB + 1;    // LDS row stride of the 128 x 128 diagonal block (doubles)

__device__ __forceinline__ double rdlane(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// ================================================================================ diagonal block
// LDS map (doubles): A[128][129] | Dinv[8][16][16] | T[16][112] | flag (int)
constexpr int LDS_A = NB * LDA;
constexpr int LDS_DINV = (NB / DB) * DB * DB;
constexpr int LDS_T = DB * (NB - DB);
constexpr int DT = 512;       // threads of the diagonal-block workgroup
constexpr int DQ = 2048 / DT;  // per-thread items of the 16 x 128 phases
constexpr size_t DIAG_LDS_BYTES = sizeof(double) * (LDS_A + LDS_DINV + LDS_T) + 16;

// One wave factors the 16 x 16 block at (c0, c0) of A in registers (lane r & 15 owns row r)
// and writes L_D back plus its inverse Dinv (lower, zeros above).
__device__ __forceinline__ void potf2_16(double* A, int c0, double* Dv, int* flag, int lane,
                                         int64_t col_base) {
  const int r = lane & 15;
  double v[DB];
#pragma unroll
  for (int c = 0; c < DB; ++c) v[c] = (c <= r) ? A[(c0 + r) * LDA + c0 + c] : 0.0;
#pragma unroll
  for (int j = 0; j < DB; ++j) {
    const double piv = rdlane(v[j], j);
    if (!(piv > 0.0) && lane == 0 && *flag == 0) *flag = (int)(col_base + c0 + j + 1);
    const double dj = sqrt(piv);
    const double rinv = 1.0 / dj;
    v[j] = (r == j) ? dj : v[j] * rinv;
#pragma unroll
    for (int c = j + 1; c < DB; ++c) {
      const double lcj = rdlane(v[j], c);
      v[c] = fma(-v[j], lcj, v[c]);
    }
  }
  // column (lane & 15) of the inverse: forward substitution with rows read lane-uniformly
  double x[DB];
#pragma unroll
  for (int rr = 0; rr < DB; ++rr) {
    double s = (rr == r) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < rr; ++k) s = fma(-rdlane(v[k], rr), x[k], s);
    x[rr] = s / rdlane(v[rr], rr);
  }
  if (lane < DB) {
#pragma unroll
    for (int c = 0; c < DB; ++c)
      if (c <= r) A[(c0 + r) * LDA + c0 + c] = v[c];
#pragma unroll
    for (int rr = 0; rr < DB; ++rr) Dv[rr * DB + r] = x[rr];  // Dinv[rr][r]
  }
}

template <typename T>
__global__ __launch_bounds__(DT) void diag_kernel(DiagArgs a) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* A = sm;
  double* Dinv = A + LDS_A;
  double* Tt = Dinv + LDS_DINV;
  int* flag = reinterpret_cast<int*>(Tt + LDS_T);

  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  T* Wb = reinterpret_cast<T*>(a.W) + (int64_t)b * a.w_bs + a.j0 * a.ld + a.j0;
  for (int e = tid; e < NB * NB; e += DT) {
    const int r = e >> 7, c = e & (NB - 1);
    A[r * LDA + c] = (c <= r) ? (double)Wb[(int64_t)r * a.ld + c] : 0.0;
  }
  if (tid == 0) *flag = 0;
  __syncthreads();

  for (int kb = 0; kb < NB / DB; ++kb) {
    const int c0 = kb * DB;
    double* Dk = Dinv + kb * DB * DB;
    if (tid < 64) potf2_16(A, c0, Dk, flag, tid, a.j0);
    __syncthreads();
    const int nrow = NB - c0 - DB;
    if (nrow == 0) break;
    // panel below the 16-block: X = B * Dinv^T, via registers (in place)
    double xv[DQ];
#pragma unroll
    for (int q = 0; q < DQ; ++q) {
      const int idx = tid + q * DT;
      xv[q] = 0.0;
      if (idx < nrow * DB) {
        const int r = c0 + DB + idx / DB, c = idx % DB;
        double s = 0.0;
        for (int k = 0; k <= c; ++k) s = fma(A[r * LDA + c0 + k], Dk[c * DB + k], s);
        xv[q] = s;
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < DQ; ++q) {
      const int idx = tid + q * DT;
      if (idx < nrow * DB) A[(c0 + DB + idx / DB) * LDA + c0 + idx % DB] = xv[q];
    }
    __syncthreads();
    // trailing rank-16 update of the lower triangle, 4 x 4 micro-tiles
    const int nt = nrow / 4;
    const int ntri = nt * (nt + 1) / 2;
    for (int t = tid; t < ntri; t += DT) {
      int ti = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
      while (ti * (ti + 1) / 2 > t) --ti;
      while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
      const int tj = t - ti * (ti + 1) / 2;
      const int rb = c0 + DB + 4 * ti, cb = c0 + DB + 4 * tj;
      double acc[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
#pragma unroll 2
      for (int k = 0; k < DB; ++k) {
        double ar[4], ac[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) ar[i] = A[(rb + i) * LDA + c0 + k];
#pragma unroll
        for (int j = 0; j < 4; ++j) ac[j] = A[(cb + j) * LDA + c0 + k];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = fma(ar[i], ac[j], acc[i][j]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (cb + j <= rb + i) A[(rb + i) * LDA + cb + j] -= acc[i][j];
    }
    __syncthreads();
  }

  // L_kk back to W (lower triangle only)
  for (int e = tid; e < NB * NB; e += DT) {
    const int r = e >> 7, c = e & (NB - 1);
    if (c <= r) Wb[(int64_t)r * a.ld + c] = (T)A[r * LDA + c];
  }
  if (tid == 0 && *flag != 0) atomicCAS(&a.info[b], 0, *flag);
  __syncthreads();

  // In-place inverse by 16-row blocks:
  //   Linv[I, <I] = -Dinv_I * (L[I, <I] * Linv[<I, <I]),  Linv[I, I] = Dinv_I.
  // Row blocks < I of A already hold Linv; row block I still holds L.
  for (int I = 0; I < NB / DB; ++I) {
    const int r0 = I * DB;
    const int ncol = r0;  // strictly-lower columns of this row block
    double tv[DQ];
#pragma unroll
    for (int q = 0; q < DQ; ++q) {
      const int idx = tid + q * DT;
      tv[q] = 0.0;
      if (idx < DB * ncol) {
        const int r = idx / ncol, c = idx % ncol;
        double s = 0.0;
        for (int k = c; k < r0; ++k) s = fma(A[(r0 + r) * LDA + k], A[k * LDA + c], s);
        tv[q] = s;
      }
    }
#pragma unroll
    for (int q = 0; q < DQ; ++q) {
      const int idx = tid + q * DT;
      if (idx < DB * ncol) Tt[(idx / ncol) * (NB - DB) + idx % ncol] = tv[q];
    }
    __syncthreads();
    const double* Di = Dinv + I * DB * DB;
#pragma unroll
    for (int q = 0; q < DQ; ++q) {
      const int idx = tid + q * DT;
      if (idx < DB * ncol) {
        const int r = idx / ncol, c = idx % ncol;
        double s = 0.0;
        for (int k = 0; k <= r; ++k) s = fma(Di[r * DB + k], Tt[k * (NB - DB) + c], s);
        tv[q] = -s;
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < DQ; ++q) {
      const int idx = tid + q * DT;
      if (idx < DB * ncol) A[(r0 + idx / ncol) * LDA + idx % ncol] = tv[q];
    }
    if (tid < DB * DB) {
      const int r = tid / DB, c = tid % DB;
      A[(r0 + r) * LDA + r0 + c] = Di[r * DB + c];
    }
    __syncthreads();
  }
  T* Ib = reinterpret_cast<T*>(a.Winv) + (int64_t)b * a.inv_bs + a.kblk * NB * NB;
  for (int e = tid; e < NB * NB; e += DT) {
    const int r = e >> 7, c = e & (NB - 1);
    Ib[e] = (T)((c <= r) ? A[r * LDA + c] : 0.0);
  }
}

// ================================================================================ MFMA GEMM
template <typename T>
struct Mfma;
template <>
struct Mfma<double> {
  typedef d4 acc_t;
  static __device__ __forceinline__ acc_t op(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // v_mfma_f64_16x16x4_f64 C/D map: col = lane & 15, row = (lane >> 4) + 4 * reg
  static __device__ __forceinline__ int row(int lane, int reg) { return (lane >> 4) + 4 * reg; }
};
template <>
struct Mfma<float> {
  typedef f4 acc_t;
  static __device__ __forceinline__ acc_t op(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  // f32 16x16 C/D map: col = lane & 15, row = 4 * (lane >> 4) + reg
  static __device__ __forceinline__ int row(int lane, int reg) { return 4 * (lane >> 4) + reg; }
};

constexpr int GBK = 16;   // K depth staged per LDS buffer
constexpr int SLD = 18;   // LDS row stride (elements): rows 0..15 at one k, and k+1, on distinct banks

template <typename T>
struct Stage {
  static constexpr int EPC = 16 / (int)sizeof(T);  // elements per 16-B chunk
  static constexpr int CPR = GBK / EPC;            // chunks per row
  static constexpr int NCH = NB * CPR / 256;       // chunks per thread per operand
};

// One 256-thread workgroup computes one 128 x 128 tile: acc = A_rows(128 x 128) * B_rows(128 x 128)^T
// over the 128-wide panel, 4 waves in a 2 x 2 grid, each 64 x 64 = 4 x 4 MFMA blocks.
// A and B are row-major with the K index contiguous; double-buffered LDS, register-staged.
template <typename T, int MODE>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmArgs a) {
  typedef Stage<T> S;
  typedef typename Mfma<T>::acc_t acc_t;
  __shared__ __attribute__((aligned(16))) T sA[2][NB * SLD];
  __shared__ __attribute__((aligned(16))) T sB[2][NB * SLD];

  const int b = blockIdx.y;
  int64_t ti, tj;
  if (MODE == GEMM_UPDATE) {
    const int64_t t = blockIdx.x;
    const int64_t w = a.c_hi - a.c_lo;
    const int64_t ttri = w * (w + 1) / 2;
    if (t < ttri) {
      int64_t r = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
      while (r * (r + 1) / 2 > t) --r;
      while ((r + 1) * (r + 2) / 2 <= t) ++r;
      ti = a.c_lo + r;
      tj = a.c_lo + (t - r * (r + 1) / 2);
    } else {
      const int64_t u = t - ttri;
      ti = a.c_hi + u / w;
      tj = a.c_lo + u % w;
    }
  } else {
    ti = blockIdx.x;
    tj = 0;
  }
  T* W = reinterpret_cast<T*>(a.W) + (int64_t)b * a.w_bs;
  const int64_t R = a.row0 + ti * NB;
  const T* Ag = W + R * a.ld + a.j0;
  const T* Bg;
  int64_t ldb;
  if (MODE == GEMM_UPDATE) {
    Bg = W + (a.row0 + tj * NB) * a.ld + a.j0;
    ldb = a.ld;
  } else {
    Bg = reinterpret_cast<const T*>(a.Binv) + (int64_t)b * a.inv_bs;
    ldb = NB;
  }

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  uint4 ra[S::NCH], rb[S::NCH];
  const T* pga[S::NCH];
  const T* pgb[S::NCH];
  int loff[S::NCH];
#pragma unroll
  for (int u = 0; u < S::NCH; ++u) {
    const int q = tid + 256 * u;
    const int row = q / S::CPR, ch = q % S::CPR;
    pga[u] = Ag + (int64_t)row * a.ld + ch * S::EPC;
    pgb[u] = Bg + (int64_t)row * ldb + ch * S::EPC;
    loff[u] = row * SLD + ch * S::EPC;
  }
#define GPK_GLOAD(kc)                                                           \
  _Pragma("unroll") for (int u = 0; u < S::NCH; ++u) {                          \
    ra[u] = *reinterpret_cast<const uint4*>(pga[u] + (kc) * GBK);               \
    rb[u] = *reinterpret_cast<const uint4*>(pgb[u] + (kc) * GBK);               \
  }
#define GPK_LSTORE(buf)                                                         \
  _Pragma("unroll") for (int u = 0; u < S::NCH; ++u) {                          \
    T* pa_ = &sA[buf][loff[u]];                                                 \
    T* pb_ = &sB[buf][loff[u]];                                                 \
    if (sizeof(T) == 8) {                                                       \
      *reinterpret_cast<uint4*>(pa_) = ra[u];                                   \
      *reinterpret_cast<uint4*>(pb_) = rb[u];                                   \
    } else {                                                                    \
      reinterpret_cast<uint2*>(pa_)[0] = make_uint2(ra[u].x, ra[u].y);          \
      reinterpret_cast<uint2*>(pa_)[1] = make_uint2(ra[u].z, ra[u].w);          \
      reinterpret_cast<uint2*>(pb_)[0] = make_uint2(rb[u].x, rb[u].y);          \
      reinterpret_cast<uint2*>(pb_)[1] = make_uint2(rb[u].z, rb[u].w);          \
    }                                                                           \
  }

  acc_t acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = acc_t{0, 0, 0, 0};

  constexpr int NK = NB / GBK;
  GPK_GLOAD(0);
  GPK_LSTORE(0);
  __syncthreads();
  const int arow = (wr * 64 + (lane & 15)) * SLD + (lane >> 4);
  const int brow = (wc * 64 + (lane & 15)) * SLD + (lane >> 4);
  for (int kc = 0; kc < NK; ++kc) {
    const int buf = kc & 1;
    if (kc + 1 < NK) { GPK_GLOAD(kc + 1); }
    const T* pa = sA[buf];
    const T* pb = sB[buf];
#pragma unroll
    for (int s = 0; s < GBK / 4; ++s) {
      T af[4], bf[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) af[m] = pa[arow + m * 16 * SLD + s * 4];
#pragma unroll
      for (int n = 0; n < 4; ++n) bf[n] = pb[brow + n * 16 * SLD + s * 4];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = Mfma<T>::op(af[m], bf[n], acc[m][n]);
    }
    if (kc + 1 < NK) { GPK_LSTORE(buf ^ 1); }
    __syncthreads();
  }

  const int col = lane & 15;
  if (MODE == GEMM_UPDATE) {
    T* C = W + R * a.ld + a.row0 + tj * NB;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = wr * 64 + m * 16 + Mfma<T>::row(lane, r);
          const int cc = wc * 64 + n * 16 + col;
          T* p = C + (int64_t)rr * a.ld + cc;
          *p = *p - acc[m][n][r];
        }
  } else {
    T* C = W + R * a.ld + a.j0;
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = wr * 64 + m * 16 + Mfma<T>::row(lane, r);
          const int cc = wc * 64 + n * 16 + col;
          C[(int64_t)rr * a.ld + cc] = acc[m][n][r];
        }
  }
}

// ================================================================================ read-out
template <typename T>
__global__ __launch_bounds__(256) void finalize_kernel(FinArgs a) {
  __shared__ double red[256];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const T* W = reinterpret_cast<const T*>(a.W) + (int64_t)b * a.w_bs;
  double s = 0.0;
  for (int64_t i = tid; i < a.n; i += 256) s += log((double)W[i * a.ld + i]);
  red[tid] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  if (tid == 0) {
    const double logdet = 2.0 * red[0];                          // Metrics.py:153-154
    const double fit = -(double)W[a.y_row * a.ld + a.y_row];     // y^T alpha = z^T z
    const double log2pi = log(2.0 * 3.141592653589793);
    const double ll = (-0.5 * fit + -0.5 * logdet) + (-0.5 * ((double)a.n * log2pi));  // LogLikelihood.py:39-49
    double nl = -ll;
    if (a.info[b] != 0) nl = INFINITY;
    a.out[b * 4 + 0] = nl;
    a.out[b * 4 + 1] = fit;
    a.out[b * 4 + 2] = logdet;
    a.out[b * 4 + 3] = (double)a.n;
  }
  // posterior read-out from the Schur complement corner
  for (int64_t t = tid; t < a.m; t += 256) {
    if (a.mu) a.mu[(int64_t)b * a.m + t] = -(double)W[a.y_row * a.ld + a.n_pad + t];
    if (a.var) a.var[(int64_t)b * a.m + t] = (double)W[(a.n_pad + t) * a.ld + a.n_pad + t];
  }
}

// ================================================================================ triangular solve
// trans = 0 (x <- L^-1 x): block k: x_k <- Linv_kk x_k, then rows below: x_i -= L[i, blk k] x_k
// trans = 1 (x <- L^-T x): block k (descending): x_k <- Linv_kk^T x_k, then x_j -= sum_i L[i, j] x_i
template <typename T>
__global__ __launch_bounds__(NB) void trsv_diag_kernel(TrsvArgs a) {
  __shared__ double xs[NB];
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  double* x = a.x + (int64_t)b * a.x_bs + a.kblk * NB;
  const T* Li = reinterpret_cast<const T*>(a.Winv) + (int64_t)b * a.inv_bs + a.kblk * NB * NB;
  xs[t] = x[t];
  __syncthreads();
  double s = 0.0;
  if (a.trans == 0) {
    for (int k = 0; k <= t; ++k) s = fma((double)Li[t * NB + k], xs[k], s);
  } else {
    for (int k = t; k < NB; ++k) s = fma((double)Li[k * NB + t], xs[k], s);
  }
  x[t] = s;
}

template <typename T>
__global__ __launch_bounds__(256) void trsv_update_kernel(TrsvArgs a) {
  __shared__ double xk[NB];
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  double* x = a.x + (int64_t)b * a.x_bs;
  const T* W = reinterpret_cast<const T*>(a.W) + (int64_t)b * a.w_bs;
  const int64_t j0 = a.kblk * NB;
  if (tid < NB) xk[tid] = x[j0 + tid];
  __syncthreads();
  if (a.trans == 0) {
    const int64_t i = j0 + NB + (int64_t)blockIdx.x * 256 + tid;
    if (i >= a.n_pad) return;
    const T* row = W + i * a.ld + j0;
    double s = 0.0;
    for (int k = 0; k < NB; ++k) s = fma((double)row[k], xk[k], s);
    x[i] -= s;
  } else {
    const int64_t j = (int64_t)blockIdx.x * 256 + tid;
    if (j >= j0) return;
    double s = 0.0;
    for (int k = 0; k < NB; ++k) s = fma((double)W[(j0 + k) * a.ld + j], xk[k], s);
    x[j] -= s;
  }
}

}  // namespace

hipError_t launch_diag(const DiagArgs& a, int dtype, int32_t batch, hipStream_t s) {
  static bool attr_done[2] = {false, false};
  if (dtype == GPK_F64) {
    if (!attr_done[0]) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(diag_kernel<double>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)DIAG_LDS_BYTES);
      attr_done[0] = true;
    }
    hipLaunchKernelGGL(diag_kernel<double>, dim3(batch), dim3(DT), DIAG_LDS_BYTES, s, a);
  } else {
    if (!attr_done[1]) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(diag_kernel<float>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)DIAG_LDS_BYTES);
      attr_done[1] = true;
    }
    hipLaunchKernelGGL(diag_kernel<float>, dim3(batch), dim3(DT), DIAG_LDS_BYTES, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_gemm(const GemmArgs& a, int dtype, int mode, int32_t batch, hipStream_t s) {
  unsigned nblk;
  if (mode == GEMM_UPDATE) {
    const int64_t w = a.c_hi - a.c_lo;
    nblk = (unsigned)(w * (w + 1) / 2 + (int64_t)(a.nt - a.c_hi) * w);
  } else {
    nblk = (unsigned)a.nt;
  }
  if (nblk == 0) return hipSuccess;
  dim3 grid(nblk, batch);
  if (dtype == GPK_F64) {
    if (mode == GEMM_UPDATE)
      hipLaunchKernelGGL((gemm_kernel<double, GEMM_UPDATE>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((gemm_kernel<double, GEMM_TRSM>), grid, dim3(256), 0, s, a);
  } else {
    if (mode == GEMM_UPDATE)
      hipLaunchKernelGGL((gemm_kernel<float, GEMM_UPDATE>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((gemm_kernel<float, GEMM_TRSM>), grid, dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_finalize(const FinArgs& a, int dtype, int32_t batch, hipStream_t s) {
  if (dtype == GPK_F64)
    hipLaunchKernelGGL(finalize_kernel<double>, dim3(batch), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(finalize_kernel<float>, dim3(batch), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_trsv_diag(const TrsvArgs& a, int dtype, int32_t batch, hipStream_t s) {
  if (dtype == GPK_F64)
    hipLaunchKernelGGL(trsv_diag_kernel<double>, dim3(batch), dim3(NB), 0, s, a);
  else
    hipLaunchKernelGGL(trsv_diag_kernel<float>, dim3(batch), dim3(NB), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_trsv_update(const TrsvArgs& a, int dtype, int32_t batch, hipStream_t s) {
  const int64_t j0 = a.kblk * NB;
  const int64_t cnt = (a.trans == 0) ? (a.n_pad - j0 - NB) : j0;
  if (cnt <= 0) return hipSuccess;
  dim3 grid((unsigned)((cnt + 255) / 256), batch);
  if (dtype == GPK_F64)
    hipLaunchKernelGGL(trsv_update_kernel<double>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(trsv_update_kernel<float>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace gpk
