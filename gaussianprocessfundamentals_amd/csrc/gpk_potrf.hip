// MFMA GEMM of the blocked Cholesky (panel solve + trailing update), the read-out, and the
// triangular solves.  The diagonal-block factorisation lives in gpk_diag.hip.
//
// Replaces tf.linalg.cholesky / tf.linalg.triangular_solve of
// gpbasics/Statistics/CovarianceMatrix.py:247-265 and the log-determinant / data-fit
// assembly of gpbasics/Metrics/Metrics.py:152-154 and gpbasics/Metrics/LogLikelihood.py:30-65.
//
// Per panel step k (columns j0 = 128k .. j0+127):
//   gemm<TRSM>    rows below the block: W[R, j0:j0+128] <- W[R, j0:j0+128] * L_kk^-T, an MFMA
//                 GEMM against the inverted diagonal block (upper zero blocks skipped); every
//                 row of the augmented matrix, so z = L^-1 y and V^T = Ks^T L^-T come out of it
//   gemm<UPDATE>  lower tiles of the trailing matrix: C -= P P^T, f64 MFMA
//                 (v_mfma_f64_16x16x4_f64) or f32 MFMA (v_mfma_f32_16x16x4_f32)
// Tiles are TM x TN (128 x 128 while the grid fills the chip, 64 x 64 on small trailing
// matrices); a 256-thread workgroup = 2 x 2 waves, double-buffered LDS staging of 16-deep K
// chunks through registers; block ids are remapped so that each XCD (blockIdx % 8) walks a
// contiguous run of tiles, which share panel rows in its L2.
#include <math.h>

#include "gpk_internal.h"

namespace gpk {
namespace {

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

#ifndef GPK_SCHED_FENCE
#define GPK_SCHED_FENCE 0  // fence the staging loads ahead of the MFMA block (A/B knob)
#endif

constexpr int GBK = 16;   // K depth staged per LDS buffer
constexpr int SLD = 18;   // LDS row stride (elements): 16 rows at one k, and k+1, on distinct banks

// bijective XCD-aware remap: consecutive logical tiles land on one XCD (blockIdx % 8 group)
__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nblk) {
  const int64_t q = nblk / 8, r = nblk % 8;
  const int64_t x = bid % 8, pos = bid / 8;
  const int64_t base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + pos;
}

// One 256-thread workgroup computes a TM x TN tile: acc = A_rows(TM x 128) * B_rows(TN x 128)^T
// over the 128-wide panel.  Waves 2 x 2, each (TM/2) x (TN/2) = MB x NBK blocks of 16 x 16.
template <typename T, int MODE, int TM, int TN>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);   // elements per 16-B chunk
  constexpr int CPR = GBK / EPC;             // chunks per row and K chunk
  constexpr int NCA = TM * CPR / 256;        // A chunks per thread
  constexpr int NCB = TN * CPR / 256;        // B chunks per thread
  constexpr int MB = TM / 32, NBK = TN / 32; // 16 x 16 blocks per wave
  typedef typename Mfma<T>::acc_t acc_t;
  __shared__ __attribute__((aligned(16))) T sA[2][TM * SLD];
  __shared__ __attribute__((aligned(16))) T sB[2][TN * SLD];

  const int b = blockIdx.y;
  const int64_t t = xcd_remap(blockIdx.x, gridDim.x);
  int64_t ti, tj;  // tile coordinates in units of TM (rows) and TN (cols)
  if (MODE == GEMM_UPDATE) {
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
    ti = t;
    tj = 0;
  }
  T* W = reinterpret_cast<T*>(a.W) + (int64_t)b * a.w_bs;
  const int64_t R = a.row0 + ti * TM;
  const T* Ag = W + R * a.ld + a.j0;
  const T* Bg;
  int64_t ldb;
  if (MODE == GEMM_UPDATE) {
    Bg = W + (a.row0 + tj * TN) * a.ld + a.j0;
    ldb = a.ld;
  } else {
    Bg = reinterpret_cast<const T*>(a.Binv) + (int64_t)b * a.inv_bs;
    ldb = NB;
  }

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  uint4 ra[NCA], rb[NCB];
  const T* pga[NCA];
  const T* pgb[NCB];
  int la[NCA], lb[NCB];
#pragma unroll
  for (int u = 0; u < NCA; ++u) {
    const int q = tid + 256 * u;
    pga[u] = Ag + (int64_t)(q / CPR) * a.ld + (q % CPR) * EPC;
    la[u] = (q / CPR) * SLD + (q % CPR) * EPC;
  }
#pragma unroll
  for (int u = 0; u < NCB; ++u) {
    const int q = tid + 256 * u;
    pgb[u] = Bg + (int64_t)(q / CPR) * ldb + (q % CPR) * EPC;
    lb[u] = (q / CPR) * SLD + (q % CPR) * EPC;
  }
#define GPK_GLOAD(kc)                                                                     \
  {                                                                                       \
    _Pragma("unroll") for (int u = 0; u < NCA; ++u) ra[u] =                               \
        *reinterpret_cast<const uint4*>(pga[u] + (kc) * GBK);                             \
    _Pragma("unroll") for (int u = 0; u < NCB; ++u) rb[u] =                               \
        *reinterpret_cast<const uint4*>(pgb[u] + (kc) * GBK);                             \
  }
#define GPK_STORE16(dst, v)                                                               \
  {                                                                                       \
    if (sizeof(T) == 8) {                                                                 \
      *reinterpret_cast<uint4*>(dst) = (v);                                               \
    } else {                                                                              \
      reinterpret_cast<uint2*>(dst)[0] = make_uint2((v).x, (v).y);                        \
      reinterpret_cast<uint2*>(dst)[1] = make_uint2((v).z, (v).w);                        \
    }                                                                                     \
  }
#define GPK_LSTORE(buf)                                                                   \
  {                                                                                       \
    _Pragma("unroll") for (int u = 0; u < NCA; ++u) GPK_STORE16(&sA[buf][la[u]], ra[u]);  \
    _Pragma("unroll") for (int u = 0; u < NCB; ++u) GPK_STORE16(&sB[buf][lb[u]], rb[u]);  \
  }

  acc_t acc[MB][NBK];
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int n = 0; n < NBK; ++n) acc[m][n] = acc_t{0, 0, 0, 0};

  const int NK = (MODE == GEMM_TRSM) ? NB / GBK : a.kdepth / GBK;
  GPK_GLOAD(0);
  GPK_LSTORE(0);
  __syncthreads();
  const int arow = (wr * (TM / 2) + (lane & 15)) * SLD + (lane >> 4);
  const int brow = (wc * (TN / 2) + (lane & 15)) * SLD + (lane >> 4);
  // Fragments are software-pipelined one 4-deep k-step ahead (two register sets), and the next
  // chunk's first fragments are read right after the barrier, under the last step's MFMAs.
  T fa0[MB], fb0[NBK], fa1[MB], fb1[NBK];
#define GPK_FRAG(FA, FB, P, Q, S)                                                          \
  {                                                                                        \
    _Pragma("unroll") for (int m = 0; m < MB; ++m) FA[m] = (P)[arow + m * 16 * SLD + (S) * 4]; \
    _Pragma("unroll") for (int n = 0; n < NBK; ++n) FB[n] = (Q)[brow + n * 16 * SLD + (S) * 4]; \
  }
  // TRSM against the lower-triangular inverse: K chunk KC feeds output columns >= 16 KC only
#define GPK_MMA(FA, FB, KC)                                                                \
  {                                                                                        \
    _Pragma("unroll") for (int n = 0; n < NBK; ++n) {                                      \
      if (MODE == GEMM_TRSM && (KC) > (wc * (TN / 2) + n * 16) / GBK) continue;            \
      _Pragma("unroll") for (int m = 0; m < MB; ++m) acc[m][n] = Mfma<T>::op(FA[m], FB[n], acc[m][n]); \
    }                                                                                      \
  }
  GPK_FRAG(fa0, fb0, sA[0], sB[0], 0);
  for (int kc = 0; kc < NK; ++kc) {
    const int buf = kc & 1;
    // branch-free staging (the last iteration re-stages its own chunk into the idle buffer):
    // a conditional load/store pair makes hipcc spill the staging registers to scratch
    const int knext = (kc + 1 < NK) ? kc + 1 : kc;
    GPK_GLOAD(knext);
    // keep the next chunk's loads in flight under this chunk's MFMAs: without the fence hipcc
    // sinks every load to its ds_write and serialises them (load, vmcnt(0), write, load, ...)
    if (GPK_SCHED_FENCE) __builtin_amdgcn_sched_barrier(0);
    const T* pa = sA[buf];
    const T* pb = sB[buf];
    GPK_FRAG(fa1, fb1, pa, pb, 1);
    GPK_MMA(fa0, fb0, kc);
    GPK_FRAG(fa0, fb0, pa, pb, 2);
    GPK_MMA(fa1, fb1, kc);
    GPK_FRAG(fa1, fb1, pa, pb, 3);
    GPK_MMA(fa0, fb0, kc);
    if (GPK_SCHED_FENCE) __builtin_amdgcn_sched_barrier(0);
    GPK_LSTORE(buf ^ 1);
    __syncthreads();
    GPK_FRAG(fa0, fb0, sA[buf ^ 1], sB[buf ^ 1], 0);
    GPK_MMA(fa1, fb1, kc);
  }
#undef GPK_FRAG
#undef GPK_MMA
#undef GPK_GLOAD
#undef GPK_STORE16
#undef GPK_LSTORE

  const int col = lane & 15;
  T* C = (MODE == GEMM_UPDATE) ? W + R * a.ld + a.row0 + tj * TN : W + R * a.ld + a.j0;
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int n = 0; n < NBK; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = wr * (TM / 2) + m * 16 + Mfma<T>::row(lane, r);
        const int cc = wc * (TN / 2) + n * 16 + col;
        T* p = C + (int64_t)rr * a.ld + cc;
        if (MODE == GEMM_UPDATE)
          *p = *p - acc[m][n][r];
        else
          *p = acc[m][n][r];
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

template <typename T, int MODE, int TM, int TN>
hipError_t launch_gemm_t(const GemmArgs& a, int32_t batch, hipStream_t s) {
  // a.nt / c_lo / c_hi are in units of this launch's tile sizes
  unsigned nblk;
  if (MODE == GEMM_UPDATE) {
    const int64_t w = a.c_hi - a.c_lo;
    nblk = (unsigned)(w * (w + 1) / 2 + (int64_t)(a.nt - a.c_hi) * w);
  } else {
    nblk = (unsigned)a.nt;
  }
  if (nblk == 0) return hipSuccess;
  hipLaunchKernelGGL((gemm_kernel<T, MODE, TM, TN>), dim3(nblk, batch), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_gemm(const GemmArgs& a, int dtype, int mode, int tile, int32_t batch, hipStream_t s) {
  if (dtype == GPK_F64) {
    if (mode == GEMM_UPDATE)
      return tile == 128 ? launch_gemm_t<double, GEMM_UPDATE, 128, 128>(a, batch, s)
                         : launch_gemm_t<double, GEMM_UPDATE, 64, 64>(a, batch, s);
    return tile == 128 ? launch_gemm_t<double, GEMM_TRSM, 128, 128>(a, batch, s)
                       : launch_gemm_t<double, GEMM_TRSM, 64, 128>(a, batch, s);
  }
  if (mode == GEMM_UPDATE)
    return tile == 128 ? launch_gemm_t<float, GEMM_UPDATE, 128, 128>(a, batch, s)
                       : launch_gemm_t<float, GEMM_UPDATE, 64, 64>(a, batch, s);
  return tile == 128 ? launch_gemm_t<float, GEMM_TRSM, 128, 128>(a, batch, s)
                     : launch_gemm_t<float, GEMM_TRSM, 64, 128>(a, batch, s);
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
