// Symmetric eigendecomposition A = V diag(lam) V^T for the pseudo-inverse / slogdet / non-positive-definite
// paths of the metrics (tf.linalg.pinv of K_mm, gpbasics/Statistics/Nystroem_K.py:53; tf.linalg.slogdet / inv /
// pinv of an indefinite K, gpbasics/Metrics/Metrics.py:132-147), tridiagonal route (gpk_syevd):
//
//   1. blocked Householder tridiagonalisation A = Q T Q^T (below; LAPACK dsytrd's reflectors, v_k stored below
//      the subdiagonal of column k, tau_k apart), the rank-2nb trailing updates on the f64 MFMA GEMM
//   2. back-transformation: the reflectors in blocks of 32, compact WY form I - Y S Y^T, applied to T's
//      eigenvectors on the f64 MFMA GEMM (build_y_kernel, larft_kernel, launch_dgemm)
//   3. divide and conquer on T (below): log2 m levels of rank-one merges whose eigenvector updates are MFMA
//      GEMMs; deflation takes the clusters of a kernel matrix's numerically zero tail out of the secular
//      equations (an implicit QL with the rotations applied in parallel measured 87 ms at m = 409: its chain of
//      ~1.5 m^2 dependent rotations is sequential)
// The two-sided Jacobi of gpk_approx.hip (gpk_syevj) stays available; this route replaces its O(m^3)-per-
// sweep rounds (30 sweeps of m - 1 launches at m = 409) with O(m^3) work overall.
#include <float.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#include "gpk_internal.h"

namespace gpk {
namespace {

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();  // red may still be read by the previous reduction
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  const int nw = (blockDim.x + 63) >> 6;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

__device__ __forceinline__ double block_max(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  const int nw = (blockDim.x + 63) >> 6;
  for (int i = 0; i < nw; ++i) s = fmax(s, red[i]);
  return s;
}

__device__ __forceinline__ double wave_sum(double v) {
  // butterfly: every lane ends with the same bits (each stage adds the same two values in either order)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Blocked Householder tridiagonalisation (LAPACK dsytrd / dlatrd, lower): panels of TRD_NB columns; inside a
// panel each column is brought up to date with the panel's earlier reflectors (V, Wp), its reflector built and
// y = A22 v formed against the trailing matrix as of the panel's start, corrected by V (Wp^T v) + Wp (V^T v);
// after the panel one rank-2nb update A22 -= V Wp^T + Wp V^T on the f64 MFMA GEMM.  W [m, m] row-major, full
// symmetric on entry; on exit d[0..m-1], e[0..m-2] hold T, tau[k] the reflector scalars and W[(k + 1 + i) m + k]
// (i >= 1) the reflector vectors v_k (v_k[0] = 1 implicit): H_k = I - tau_k v_k v_k^T acts on rows / columns
// k + 1 .. m - 1, and Q = H_0 H_1 ... H_{m-2}.  Vp / Wp: [m, TRD_NB] row-major panels (zero above row j + 1 in
// column j).  Small m: one workgroup per panel (trd_panel_kernel); large m: three launches per column with the
// product y = A22 v spread over the chip (trd_prep_kernel, trd_matvec_kernel, trd_finish_kernel).
constexpr int TRD_NB = 32;

struct TrdArgs {
  double* W;
  double* PV;  // [3 NB, m] row-major: rows t = V's column t, NB + t = Wp's column t, 2 NB + t = V's column t again
               // (so that [V Wp] and [Wp V] are both contiguous row ranges: one K = 2 NB GEMM for the update)
  double *d, *e, *tau;
  double *vg, *yg;  // v / y in HBM for the split path
  int m;
  unsigned long long* prof;  // timing-only: per-phase cycle sums of trd_panel_kernel (nullptr normally)
};

// update column j (rows >= j) with the panel's q earlier reflectors, build its reflector: v (v[0] = 1, length
// n1 = m - j - 1) into vs, PV's V rows q and 2 NB + q and W's column j; d[j], e[j], tau[j].  Returns tau_j.
__device__ double trd_prep(const TrdArgs& A, int j, int q, double* vs, double* rowj, double* red) {
  const int tid = threadIdx.x, T = blockDim.x, m = A.m, n1 = m - j - 1;
  const double* V = A.PV;
  const double* Wp = A.PV + (int64_t)TRD_NB * m;
  for (int t = tid; t < q; t += T) {
    rowj[t] = V[(int64_t)t * m + j];
    rowj[TRD_NB + t] = Wp[(int64_t)t * m + j];
  }
  __syncthreads();
  for (int r = j + tid; r < m; r += T) {
    // q <= 31 dependent-free products: unrolled so that the loads of 8 columns are in flight together
    double acc = A.W[(int64_t)r * m + j], a1 = 0.0;
#pragma unroll 8
    for (int t = 0; t < q; ++t) {
      acc = fma(-V[(int64_t)t * m + r], rowj[TRD_NB + t], acc);
      a1 = fma(-Wp[(int64_t)t * m + r], rowj[t], a1);
    }
    acc += a1;
    if (r == j) A.d[j] = acc;
    else vs[r - j - 1] = acc;
  }
  __syncthreads();
  const double alpha = vs[0];
  double ss = 0.0;
  for (int i = 1 + tid; i < n1; i += T) ss += vs[i] * vs[i];
  ss = block_sum(ss, red);
  double beta = alpha, tk = 0.0, scale = 0.0;
  if (ss > 0.0) {
    beta = -copysign(sqrt(alpha * alpha + ss), alpha);
    tk = (beta - alpha) / beta;
    scale = 1.0 / (alpha - beta);
  }
  for (int i = tid; i < n1; i += T) vs[i] = (i == 0) ? 1.0 : vs[i] * scale;
  if (tid == 0) {
    A.e[j] = beta;
    A.tau[j] = tk;
  }
  __syncthreads();
  double* Vq = A.PV + (int64_t)q * m;
  double* V2q = A.PV + (int64_t)(2 * TRD_NB + q) * m;
  for (int r = tid; r < m; r += T) {
    const double v = r <= j ? 0.0 : vs[r - j - 1];
    Vq[r] = v;
    V2q[r] = v;
    if (r >= j + 2) A.W[(int64_t)r * m + j] = v;
  }
  return tk;
}

// y[i] = sum_l W[j + 1 + i][j + 1 + l] v[l] for rows i in [i0, i1), one wave per row (two rows per pass)
__device__ void trd_matvec(const TrdArgs& A, int j, const double* vs, double* ys, int i0, int i1, int wave, int nw) {
  const int lane = threadIdx.x & 63, m = A.m, n1 = m - j - 1;
  const double* base = A.W + (int64_t)(j + 1) * m + (j + 1);
  int i = i0 + 2 * wave;
  for (; i + 1 < i1; i += 2 * nw) {
    const double* r0 = base + (int64_t)i * m;
    const double* r1 = r0 + m;
    double a0 = 0.0, a1 = 0.0;
#pragma unroll 4
    for (int l = lane; l < n1; l += 64) {
      const double v = vs[l];
      a0 = fma(r0[l], v, a0);
      a1 = fma(r1[l], v, a1);
    }
    a0 = wave_sum(a0);
    a1 = wave_sum(a1);
    if (lane == 0) {
      ys[i] = a0;
      ys[i + 1] = a1;
    }
  }
  if (i < i1) {
    const double* r0 = base + (int64_t)i * m;
    double a0 = 0.0;
    for (int l = lane; l < n1; l += 64) a0 = fma(r0[l], vs[l], a0);
    a0 = wave_sum(a0);
    if (lane == 0) ys[i] = a0;
  }
}

// In-workgroup form of the product (trd_panel_kernel, m <= 1024): A22 symmetric, so y_i = sum_l A22[l][i] v_l:
// lanes over the outputs i (coalesced row reads, no cross-lane reduction), wave w over rows l = w, w + nw, ...,
// R rows per pass so that R rows' loads are in flight together; per-wave partial sums in LDS, added in wave
// order (deterministic).  C = 64-lane column groups held in registers (n1 <= 64 C).
template <int C, int R>
__device__ void trd_matvec_cols(const TrdArgs& A, int j, const double* vs, double* ys, double* part) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6, T = blockDim.x;
  const int m = A.m, n1 = m - j - 1;
  const double* base = A.W + (int64_t)(j + 1) * m + (j + 1);
  double acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 0.0;
  int l = wave;
  for (; l + (R - 1) * nw < n1; l += R * nw) {
    double x[R][C];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const double* row = base + (int64_t)(l + u * nw) * m;
#pragma unroll
      for (int c = 0; c < C; ++c) x[u][c] = (lane + 64 * c < n1) ? row[lane + 64 * c] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const double vl = vs[l + u * nw];
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = fma(x[u][c], vl, acc[c]);
    }
  }
  for (; l < n1; l += nw) {
    const double* row = base + (int64_t)l * m;
    const double vl = vs[l];
#pragma unroll
    for (int c = 0; c < C; ++c)
      if (lane + 64 * c < n1) acc[c] = fma(row[lane + 64 * c], vl, acc[c]);
  }
#pragma unroll
  for (int c = 0; c < C; ++c)
    if (lane + 64 * c < n1) part[wave * m + lane + 64 * c] = acc[c];
  __syncthreads();
  for (int i = tid; i < n1; i += T) {
    double sum = 0.0;
    for (int w = 0; w < nw; ++w) sum += part[w * m + i];
    ys[i] = sum;
  }
}

// y -= V (Wp^T v) + Wp (V^T v); w = tau y - tau / 2 (tau y^T v) v into PV's Wp row q
__device__ void trd_finish(const TrdArgs& A, int j, int q, double tk, const double* vs, double* ys, double* dots,
                           double* red) {
  const int tid = threadIdx.x, T = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = T >> 6;
  const int m = A.m, n1 = m - j - 1;
  const double* V = A.PV + (j + 1);
  const double* Wp = A.PV + (int64_t)TRD_NB * m + (j + 1);
  for (int t2 = wave; t2 < 2 * q; t2 += nw) {
    const double* P = t2 < q ? Wp + (int64_t)t2 * m : V + (int64_t)(t2 - q) * m;
    double acc = 0.0, acc1 = 0.0;
    int i = lane;
#pragma unroll 4
    for (; i + 64 < n1; i += 128) {
      acc = fma(P[i], vs[i], acc);
      acc1 = fma(P[i + 64], vs[i + 64], acc1);
    }
    if (i < n1) acc = fma(P[i], vs[i], acc);
    acc = wave_sum(acc + acc1);
    if (lane == 0) dots[t2] = acc;
  }
  __syncthreads();
  double wv = 0.0;
  for (int i = tid; i < n1; i += T) {
    double y = ys[i], y1 = 0.0;
#pragma unroll 8
    for (int t = 0; t < q; ++t) {
      y = fma(-V[(int64_t)t * m + i], dots[t], y);
      y1 = fma(-Wp[(int64_t)t * m + i], dots[q + t], y1);
    }
    y = (y + y1) * tk;
    ys[i] = y;
    wv = fma(y, vs[i], wv);
  }
  wv = block_sum(wv, red);
  const double a2 = -0.5 * tk * wv;
  double* Wq = A.PV + (int64_t)(TRD_NB + q) * m;
  for (int r = tid; r < m; r += T) Wq[r] = r <= j ? 0.0 : fma(a2, vs[r - j - 1], ys[r - j - 1]);
  __syncthreads();
}

// one panel (columns k0 .. k0 + nq - 1) in one workgroup (m <= TRD_PANEL_MAX_M);
// LDS: v, y [m], rowj [2 NB], dots [2 NB], red [32], per-wave partial products [16 m]
constexpr int TRD_PANEL_MAX_M = 1024;
__global__ __launch_bounds__(1024) void trd_panel_kernel(TrdArgs A, int k0, int nq) {
  extern __shared__ __attribute__((aligned(16))) double sh[];
  double* vs = sh;
  double* ys = vs + A.m;
  double* rowj = ys + A.m;
  double* dots = rowj + 2 * TRD_NB;
  double* red = dots + 2 * TRD_NB;
  double* part = red + 32;
  unsigned long long t0 = A.prof ? clock64() : 0, c_prep = 0, c_mv = 0, c_fin = 0;
  for (int q = 0; q < nq; ++q) {
    const int j = k0 + q, n1 = A.m - j - 1;
    const double tk = trd_prep(A, j, q, vs, rowj, red);
    __syncthreads();
    if (A.prof) {
      const unsigned long long t = clock64();
      c_prep += t - t0;
      t0 = t;
    }
    if (n1 <= 256) trd_matvec_cols<4, 4>(A, j, vs, ys, part);
    else if (n1 <= 512) trd_matvec_cols<8, 2>(A, j, vs, ys, part);
    else trd_matvec_cols<16, 1>(A, j, vs, ys, part);
    __syncthreads();
    if (A.prof) {
      const unsigned long long t = clock64();
      c_mv += t - t0;
      t0 = t;
    }
    trd_finish(A, j, q, tk, vs, ys, dots, red);
    if (A.prof) {
      const unsigned long long t = clock64();
      c_fin += t - t0;
      t0 = t;
    }
  }
  if (A.prof && threadIdx.x == 0) {
    A.prof[0] += c_prep;
    A.prof[1] += c_mv;
    A.prof[2] += c_fin;
  }
}

__global__ __launch_bounds__(1024) void trd_prep_kernel(TrdArgs A, int j, int q) {
  __shared__ double rowj[2 * TRD_NB];
  __shared__ double red[32];
  trd_prep(A, j, q, A.vg, rowj, red);
}

__global__ __launch_bounds__(256) void trd_matvec_kernel(TrdArgs A, int j) {
  const int n1 = A.m - j - 1;
  const int i0 = blockIdx.x * 8, i1 = min(i0 + 8, n1);  // 8 rows per workgroup of 4 waves
  trd_matvec(A, j, A.vg, A.yg, i0, i1, threadIdx.x >> 6, 4);
}

__global__ __launch_bounds__(1024) void trd_finish_kernel(TrdArgs A, int j, int q) {
  __shared__ double dots[2 * TRD_NB];
  __shared__ double red[32];
  trd_finish(A, j, q, A.tau[j], A.vg, A.yg, dots, red);
}

__global__ void trd_last_kernel(const double* W, int m, double* d) {
  if (threadIdx.x == 0) d[m - 1] = W[(int64_t)(m - 1) * m + (m - 1)];
}

// ---------------------------------------------------------------------------------------------------------
// Divide and conquer on the tridiagonal T (Cuppen; deflation as LAPACK dlaed2, eigenvectors by Gu & Eisenstat's
// recomputed z so that they come out orthogonal without reorthogonalisation), bottom-up over levels: level l
// merges pairs of neighbouring blocks of width w = 2^l (leaves of one row; the last block of a level may be
// narrower or unpaired).  T = diag(T1', T2') + rho u u^T with rho = e[b-1] the coupling of the pair [a, b) | [b, c)
// and u = e_{b-1} + e_b; T1' / T2' carry the -rho on their touching diagonal entries (dc_init_kernel applies it
// for every split at once).  With T_i' = Q_i D_i Q_i^T, T = Q (D + rho z z^T) Q^T, z = (last row of Q1, first
// row of Q2).  Per level: dc_deflate_kernel (sort, deflation), dc_gather_kernel (Q's columns in sorted order,
// deflation rotations, kept columns first), dc_secular_kernel (roots by bisection in a shifted variable),
// dc_zhat_kernel, dc_vec_kernel (the merged problem's eigenvectors U), and one batched MFMA GEMM Q <- Q U^T.
// Q is kept block diagonal in an [m, m] buffer; eigenvalues in lam, in no particular order within a block.
// ---------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dc_init_kernel(const double* d, const double* e, int m, double* lam,
                                                      double* Q) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < m) {
    const int i = (int)t;
    lam[i] = d[i] - (i > 0 ? e[i - 1] : 0.0) - (i < m - 1 ? e[i] : 0.0);
  }
  if (t < (int64_t)m * m) Q[t] = (t / m == t % m) ? 1.0 : 0.0;
}

// One workgroup per pair.  Merged blocks of up to DC_LDS_MAX_K rows sort and deflate in LDS: D[P2] z[k] idx[P2]
// kept[k] defl[k]; larger ones (m > 4096, the non-positive-definite fallbacks of the metrics at large n) use the
// same arrays in the level's HBM scratch L.gscr (pair p at offset 2a / a: the pairs' regions never overlap),
// ordered by the same workgroup barriers (one workgroup, one CU: its stores and loads meet in that CU's L1 / L2).
constexpr int DC_LDS_MAX_K = 4096;
__global__ __launch_bounds__(256) void dc_deflate_kernel(const double* __restrict__ e, const double* __restrict__ Q,
                                                         int m, int w, DcLevel L) {
  extern __shared__ __attribute__((aligned(16))) double sh[];
  __shared__ double red[32];
  const int p = blockIdx.x, tid = threadIdx.x;
  const int a = 2 * w * p, b = a + w, c = min(a + 2 * w, m), k = c - a;
  int P2 = 1;
  while (P2 < k) P2 <<= 1;
  double *D, *z;
  int *idx, *kept, *defl;
  if (k <= DC_LDS_MAX_K) {
    D = sh;
    z = D + P2;
    idx = reinterpret_cast<int*>(z + k);
    kept = idx + P2;
    defl = kept + k;
  } else {
    D = L.gscr + 2 * (int64_t)a;
    z = L.gscr + 2 * (int64_t)m + a;
    int* gi = reinterpret_cast<int*>(L.gscr + 3 * (int64_t)m);
    idx = gi + 2 * (int64_t)a;
    kept = gi + 2 * (int64_t)m + a;
    defl = gi + 3 * (int64_t)m + a;
  }
  const double rho = e[b - 1];
  const bool flip = rho < 0.0;
  auto zorig = [&](int s) -> double { return s < w ? Q[(int64_t)(b - 1) * m + a + s] : Q[(int64_t)b * m + a + s]; };
  double ss = 0.0;
  for (int s = tid; s < k; s += 256) {
    const double v = zorig(s);
    ss += v * v;
  }
  const double zz = block_sum(ss, red);
  for (int s = tid; s < P2; s += 256) {
    D[s] = s < k ? (flip ? -L.lam[a + s] : L.lam[a + s]) : INFINITY;
    idx[s] = s;
  }
  __syncthreads();
  // bitonic sort of (D, idx), ties by index: a deterministic total order
  for (int size = 2; size <= P2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P2; i += 256) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const double di = D[i], dj = D[j];
          const int ii = idx[i], ij = idx[j];
          const bool gt = (di > dj) || (di == dj && ii > ij);
          if (gt == up) {
            D[i] = dj;
            D[j] = di;
            idx[i] = ij;
            idx[j] = ii;
          }
        }
      }
      __syncthreads();
    }
  }
  const double zn = sqrt(zz);
  const double r = fabs(rho) * zz;
  double dmax = 0.0, zmax = 0.0;
  for (int s = tid; s < k; s += 256) {
    z[s] = zorig(idx[s]) / zn;
    dmax = fmax(dmax, fabs(D[s]));
    zmax = fmax(zmax, fabs(z[s]));
  }
  dmax = block_max(dmax, red);
  zmax = block_max(zmax, red);
  const double tol = 8.0 * DBL_EPSILON * fmax(dmax, r * zmax);
  __shared__ int cnt[3];
  if (tid == 0) {
    int K = 0, nd = 0, nr = 0, pj = -1;
    for (int s = 0; s < k; ++s) {
      if (r * fabs(z[s]) <= tol) {
        defl[nd++] = s;
        continue;
      }
      if (pj < 0) {
        pj = s;
        continue;
      }
      const double zs = z[pj], zc = z[s];
      const double tau = hypot(zc, zs);
      const double cs = zc / tau, sn = -zs / tau;
      const double t = D[s] - D[pj];
      if (fabs(t * cs * sn) <= tol) {
        z[s] = tau;
        z[pj] = 0.0;
        L.rp[a + nr] = pj;
        L.rn[a + nr] = s;
        L.rc[a + nr] = cs;
        L.rs[a + nr] = sn;
        ++nr;
        const double t2 = D[pj] * cs * cs + D[s] * sn * sn;
        D[s] = D[pj] * sn * sn + D[s] * cs * cs;
        D[pj] = t2;
        defl[nd++] = pj;
      } else {
        kept[K++] = pj;
      }
      pj = s;
    }
    if (pj >= 0) kept[K++] = pj;
    cnt[0] = K;
    cnt[1] = nd;
    cnt[2] = nr;
    L.kcnt[p] = K;
    L.rcnt[p] = nr;
    L.flip[p] = flip ? 1 : 0;
    L.rho[p] = r;
  }
  __syncthreads();
  const int K = cnt[0], nd = cnt[1];
  const double sg = flip ? -1.0 : 1.0;
  for (int t = tid; t < K; t += 256) {
    L.dK[a + t] = D[kept[t]];
    L.zK[a + t] = z[kept[t]];
    L.ord[a + t] = kept[t];
  }
  for (int t = tid; t < nd; t += 256) {
    L.lam[a + K + t] = sg * D[defl[t]];
    L.ord[a + K + t] = defl[t];
  }
  for (int s = tid; s < k; s += 256) L.idx[a + s] = idx[s];
}

// One wave per row r of a pair's block: the row in sorted column order, the deflation rotations, then written
// kept columns first.  LDS: k doubles for merged blocks of up to DC_GATHER_LDS_MAX_K rows.  Larger ones (m >
// 16384: the top merge of the non-positive-definite fallbacks at large n) stage the row in HBM instead: the sorted
// row goes to Qg's row (the output's own place), is rotated there, written permuted into Q's row (read by no one
// else: Q's row r is this wave's input only, and the level's GEMM overwrites Q afterwards) and copied back.
constexpr int DC_GATHER_LDS_MAX_K = 16384;  // 128 KB of LDS
__global__ __launch_bounds__(64) void dc_gather_kernel(double* __restrict__ Q, int m, int w, DcLevel L,
                                                       double* __restrict__ Qg) {
  extern __shared__ __attribute__((aligned(16))) double xs[];
  const int r = blockIdx.x, lane = threadIdx.x;
  const int p = r / (2 * w);
  const int a = 2 * w * p, c = min(a + 2 * w, m), k = c - a;
  double* row = Q + (int64_t)r * m + a;
  double* out = Qg + (int64_t)r * m + a;
  const bool lds = k <= DC_GATHER_LDS_MAX_K;
  double* x = lds ? xs : out;
  for (int s = lane; s < k; s += 64) x[s] = row[L.idx[a + s]];
  if (!lds) __threadfence_block();
  __syncthreads();
  if (lane == 0) {
    const int nr = L.rcnt[p];
    for (int q = 0; q < nr; ++q) {
      const int i = L.rp[a + q], j = L.rn[a + q];
      const double cs = L.rc[a + q], sn = L.rs[a + q];
      const double xi = x[i], xj = x[j];
      x[i] = cs * xi + sn * xj;
      x[j] = cs * xj - sn * xi;
    }
  }
  if (!lds) __threadfence_block();
  __syncthreads();
  if (lds) {
    for (int t = lane; t < k; t += 64) out[t] = x[L.ord[a + t]];
    return;
  }
  for (int t = lane; t < k; t += 64) row[t] = x[L.ord[a + t]];
  __threadfence_block();
  __syncthreads();
  for (int t = lane; t < k; t += 64) out[t] = row[t];
}

// One wave per root (position s of a pair's kept set): 1 + r sum z_j^2 / (d_j - lambda) = 0 on (d_t, d_{t+1})
// (the last on (d_{K-1}, d_{K-1} + r |z|^2)), lambda = d_o + tau with the origin o the nearer pole, so that the
// differences d_j - lambda = (d_j - d_o) - tau keep their relative accuracy; bisection on tau to the last bit.
__global__ __launch_bounds__(256) void dc_secular_kernel(int m, int w, DcLevel L) {
  const int lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= m) return;
  const int p = s / (2 * w), a = 2 * w * p, t = s - a;
  if ((2 * p + 1) * w >= m) return;  // an unpaired last block
  const int K = L.kcnt[p];
  if (t >= K) return;
  const double r = L.rho[p];
  const double* d = L.dK + a;
  const double* z = L.zK + a;
  int o;
  double lo, hi;
  if (t < K - 1) {
    const double half = 0.5 * (d[t + 1] - d[t]);
    double f = 0.0;
    for (int j = lane; j < K; j += 64) f += z[j] * z[j] / ((d[j] - d[t]) - half);
    f = 1.0 + r * wave_sum(f);
    if (f >= 0.0) {
      o = t;
      lo = 0.0;
      hi = half;
    } else {
      o = t + 1;
      lo = -half;
      hi = 0.0;
    }
  } else {
    double zz = 0.0;
    for (int j = lane; j < K; j += 64) zz += z[j] * z[j];
    o = t;
    lo = 0.0;
    hi = r * wave_sum(zz);
  }
  const double dor = d[o];
  for (int it = 0; it < 400; ++it) {
    const double tau = 0.5 * (lo + hi);
    if (tau == lo || tau == hi) break;
    double f = 0.0;
    for (int j = lane; j < K; j += 64) f += z[j] * z[j] / ((d[j] - dor) - tau);
    f = 1.0 + r * wave_sum(f);
    if (f < 0.0) lo = tau;
    else hi = tau;
  }
  if (lane == 0) {
    L.root_o[s] = o;
    L.root_t[s] = 0.5 * (lo + hi);
  }
}

// zhat_i = sign(z_i) sqrt( prod_j (lambda_j - d_i) / prod_{j != i} (d_j - d_i) / r ), one thread per i
__global__ __launch_bounds__(256) void dc_zhat_kernel(int m, int w, DcLevel L) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= m) return;
  const int p = s / (2 * w), a = 2 * w * p, i = s - a;
  if ((2 * p + 1) * w >= m) return;
  const int K = L.kcnt[p];
  if (i >= K) return;
  const double* d = L.dK + a;
  const double di = d[i];
  double prod = ((d[L.root_o[s]] - di) + L.root_t[s]) / L.rho[p];
  for (int j = 0; j < K; ++j) {
    if (j == i) continue;
    prod *= ((d[L.root_o[a + j]] - di) + L.root_t[a + j]) / (d[j] - di);
  }
  L.zhat[s] = copysign(sqrt(fabs(prod)), L.zK[s]);
}

// One wave per row t of a pair's k x k block of U: t < K the normalised eigenvector zhat_i / (d_i - lambda_t)
// of the merged problem (and lambda_t to lam), t >= K the unit row e_t (deflated columns pass through).
__global__ __launch_bounds__(256) void dc_vec_kernel(int m, int w, DcLevel L, double* __restrict__ U) {
  const int lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= m) return;
  const int p = s / (2 * w), a = 2 * w * p, c = min(a + 2 * w, m), k = c - a, t = s - a;
  if ((2 * p + 1) * w >= m) return;
  const int K = L.kcnt[p];
  double* row = U + (int64_t)s * m + a;
  if (t >= K) {
    for (int i = lane; i < k; i += 64) row[i] = (i == t) ? 1.0 : 0.0;
    return;
  }
  const double* d = L.dK + a;
  const double* zh = L.zhat + a;
  const int o = L.root_o[s];
  const double tau = L.root_t[s], dor = d[o];
  double nn = 0.0;
  for (int i = lane; i < K; i += 64) {
    const double u = zh[i] / ((d[i] - dor) - tau);
    nn += u * u;
  }
  const double inv = 1.0 / sqrt(wave_sum(nn));
  for (int i = lane; i < k; i += 64) row[i] = (i < K) ? inv * zh[i] / ((d[i] - dor) - tau) : 0.0;
  if (lane == 0) L.lam[s] = (L.flip[p] ? -1.0 : 1.0) * (dor + tau);
}

__global__ __launch_bounds__(256) void transpose_kernel(const double* A, int m, double* B) {
  __shared__ double t[32][33];
  const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int r = ty; r < 32; r += 8)
    if (by + r < m && bx + tx < m) t[r][tx] = A[(int64_t)(by + r) * m + bx + tx];
  __syncthreads();
  for (int r = ty; r < 32; r += 8)
    if (bx + r < m && by + tx < m) B[(int64_t)(bx + r) * m + by + tx] = t[tx][r];
}

__global__ __launch_bounds__(256) void identity_kernel(double* Z, int m) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)m * m) return;
  Z[e] = (e / m == e % m) ? 1.0 : 0.0;
}

// Y [m, nb]: columns v_{k0 .. k0 + nb - 1} (zero above row k + 1, 1 at row k + 1, W below)
__global__ __launch_bounds__(256) void build_y_kernel(const double* W, int m, int k0, int nb, double* Y) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)m * nb) return;
  const int i = (int)(e / nb), c = (int)(e % nb);
  const int k = k0 + c;
  double v = 0.0;
  if (i == k + 1) v = 1.0;
  else if (i > k + 1) v = W[(int64_t)i * m + k];
  Y[e] = v;
}

// S [nb, nb] upper triangular with H_{k0} ... H_{k0 + nb - 1} = I - Y S Y^T (dlarft, forward, columnwise):
// S_ii = tau_i, S[0:i, i] = -tau_i S[0:i, 0:i] (Y^T Y)[0:i, i].  G = Y^T Y; one wave, S in LDS (nb <= 64).
__global__ __launch_bounds__(64) void larft_kernel(const double* G, const double* tau, int k0, int nb, double* S) {
  __shared__ double Sl[64 * 65];
  __shared__ double g[64];
  const int r = threadIdx.x;
  for (int i = 0; i < nb; ++i) {
    const double ti = tau[k0 + i];
    g[r] = r < i ? G[r * nb + i] : 0.0;
    __syncthreads();
    if (r < i) {
      double acc = 0.0;
      for (int c = r; c < i; ++c) acc += Sl[r * 65 + c] * g[c];
      Sl[r * 65 + i] = -ti * acc;
    } else if (r < nb) {
      Sl[r * 65 + i] = (r == i) ? ti : 0.0;
    }
    __syncthreads();
  }
  for (int i = 0; i < nb; ++i)
    if (r < nb) S[r * nb + i] = Sl[r * 65 + i];
}

// Back-transformation for m <= BT_MAX_M in two launches (in place of build_y + 4 GEMMs + larft per block):
// bt_larft_kernel computes every block's S (one workgroup per block of BT_NB reflectors: G = Y^T Y from W's
// reflector columns staged through LDS, then dlarft's recurrence), bt_apply_kernel applies all blocks, last to
// first, V <- V - Y (S (Y^T V)), to a slab of BT_CW columns of V held in LDS (one workgroup per slab).
constexpr int BT_NB = 32, BT_CW = 8, BT_RC = 128, BT_MAX_M = 1024;

// Y chunk: rows [i0, i0 + BT_RC) of the block's reflector columns k0 .. k0 + nb - 1 into Yc[BT_RC][BT_NB + 1]
__device__ __forceinline__ void bt_stage_y(const double* W, int m, int k0, int nb, int i0, double* Yc) {
  for (int e = threadIdx.x; e < BT_RC * BT_NB; e += blockDim.x) {
    const int r = e / BT_NB, c = e % BT_NB, i = i0 + r, k = k0 + c;
    double v = 0.0;
    if (c < nb && i < m) v = (i == k + 1) ? 1.0 : (i > k + 1 ? W[(int64_t)i * m + k] : 0.0);
    Yc[r * (BT_NB + 1) + c] = v;
  }
}

__global__ __launch_bounds__(256) void bt_larft_kernel(const double* W, const double* tau, int m, double* Sall) {
  __shared__ double Yc[BT_RC * (BT_NB + 1)];
  __shared__ double G[BT_NB * (BT_NB + 1)];
  __shared__ double Sl[BT_NB * (BT_NB + 1)];
  const int kb = blockIdx.x, k0 = kb * BT_NB, nref = m - 1, nb = min(BT_NB, nref - k0), tid = threadIdx.x;
  const int gr = tid / BT_NB, gc = tid % BT_NB;  // 8 x 32 threads: G rows gr, gr + 8, gr + 16, gr + 24
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int i0 = k0 + 1; i0 < m; i0 += BT_RC) {
    __syncthreads();
    bt_stage_y(W, m, k0, nb, i0, Yc);
    __syncthreads();
    const int rows = min(BT_RC, m - i0);
    for (int r = 0; r < rows; ++r) {
      const double yc = Yc[r * (BT_NB + 1) + gc];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = fma(Yc[r * (BT_NB + 1) + gr + 8 * u], yc, acc[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) G[(gr + 8 * u) * (BT_NB + 1) + gc] = acc[u];
  __syncthreads();
  if (tid < BT_NB) {  // S_ii = tau_i, S[0:i, i] = -tau_i S[0:i, 0:i] G[0:i, i]: lane r reads only its own row
    const int r = tid;
    for (int i = 0; i < nb; ++i) {
      const double ti = tau[k0 + i];
      if (r < i) {
        double s = 0.0;
        for (int c = r; c < i; ++c) s += Sl[r * (BT_NB + 1) + c] * G[c * (BT_NB + 1) + i];
        Sl[r * (BT_NB + 1) + i] = -ti * s;
      } else {
        Sl[r * (BT_NB + 1) + i] = (r == i) ? ti : 0.0;
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < BT_NB * BT_NB; e += 256) {
    const int r = e / BT_NB, c = e % BT_NB;
    Sall[(int64_t)kb * BT_NB * BT_NB + e] = (r < nb && c < nb) ? Sl[r * (BT_NB + 1) + c] : 0.0;
  }
}

__global__ __launch_bounds__(256) void bt_apply_kernel(const double* W, int m, const double* Sall, double* V) {
  extern __shared__ __attribute__((aligned(16))) double sh[];
  double* Vs = sh;                           // [m][BT_CW]
  double* Yc = Vs + (size_t)m * BT_CW;       // [BT_RC][BT_NB + 1]
  double* T1 = Yc + BT_RC * (BT_NB + 1);     // [BT_NB][BT_CW]
  double* T2 = T1 + BT_NB * BT_CW;           // [BT_NB][BT_CW]
  double* S = T2 + BT_NB * BT_CW;            // [BT_NB][BT_NB]
  const int tid = threadIdx.x, c0 = blockIdx.x * BT_CW, ncol = min(BT_CW, m - c0);
  for (int e = tid; e < m * BT_CW; e += 256) {
    const int i = e / BT_CW, c = e % BT_CW;
    Vs[e] = c < ncol ? V[(int64_t)i * m + c0 + c] : 0.0;
  }
  const int nref = m - 1, nblk = (nref + BT_NB - 1) / BT_NB;
  const int tc = tid / BT_CW, tcol = tid % BT_CW;  // 32 x 8 threads: T entry (tc, tcol)
  for (int kb = nblk - 1; kb >= 0; --kb) {
    const int k0 = kb * BT_NB, nb = min(BT_NB, nref - k0);
    __syncthreads();
    for (int e = tid; e < BT_NB * BT_NB; e += 256) S[e] = Sall[(int64_t)kb * BT_NB * BT_NB + e];
    // T1 = Y^T Vs
    double acc = 0.0;
    for (int i0 = k0 + 1; i0 < m; i0 += BT_RC) {
      __syncthreads();
      bt_stage_y(W, m, k0, nb, i0, Yc);
      __syncthreads();
      const int rows = min(BT_RC, m - i0);
      for (int r = 0; r < rows; ++r) acc = fma(Yc[r * (BT_NB + 1) + tc], Vs[(i0 + r) * BT_CW + tcol], acc);
    }
    T1[tc * BT_CW + tcol] = acc;
    __syncthreads();
    // T2 = S T1
    double t2 = 0.0;
    for (int c = 0; c < BT_NB; ++c) t2 = fma(S[tc * BT_NB + c], T1[c * BT_CW + tcol], t2);
    T2[tc * BT_CW + tcol] = t2;
    // Vs -= Y T2 (rows > k0)
    for (int i0 = k0 + 1; i0 < m; i0 += BT_RC) {
      __syncthreads();
      bt_stage_y(W, m, k0, nb, i0, Yc);
      __syncthreads();
      const int rows = min(BT_RC, m - i0);
      for (int e = tid; e < rows * BT_CW; e += 256) {
        const int r = e / BT_CW, col = e % BT_CW;
        double u = 0.0;
#pragma unroll 8
        for (int c = 0; c < BT_NB; ++c) u = fma(Yc[r * (BT_NB + 1) + c], T2[c * BT_CW + col], u);
        Vs[(i0 + r) * BT_CW + col] -= u;
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < m * BT_CW; e += 256) {
    const int i = e / BT_CW, c = e % BT_CW;
    if (c < ncol) V[(int64_t)i * m + c0 + c] = Vs[e];
  }
}

__global__ __launch_bounds__(256) void sym_copy_kernel(const double* A, int64_t lda, int m, double* W) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)m * m) return;
  const int64_t i = e / m, j = e % m;
  // the lower triangle, mirrored (what gpk_syevj reads of a symmetric input as well)
  W[e] = (j <= i) ? A[i * lda + j] : A[j * lda + i];
}

}  // namespace

static size_t trd_panel_lds(int m) { return sizeof(double) * (18 * (size_t)m + 4 * TRD_NB + 32); }

hipError_t launch_eig_tridiag(double* W, int m, double* d, double* e, double* tau, double* PV, double* vg,
                              double* yg, int split_m, hipStream_t s) {
  {
    hipError_t err = ensure_dyn_lds(reinterpret_cast<const void*>(trd_panel_kernel), trd_panel_lds(TRD_PANEL_MAX_M));
    if (err != hipSuccess) return err;
  }
  static unsigned long long* prof = nullptr;
  if (getenv("GPK_TRD_PROF") && !prof) {
    hipError_t err = hipMallocManaged(&prof, 4 * sizeof(unsigned long long));
    if (err != hipSuccess) return err;
    memset(prof, 0, 4 * sizeof(unsigned long long));
    atexit([] {
      hipDeviceSynchronize();
      fprintf(stderr, "trd_panel cycles: prep %llu matvec %llu finish %llu\n", prof[0], prof[1], prof[2]);
    });
  }
  TrdArgs A{W, PV, d, e, tau, vg, yg, m, prof};
  const bool split = m > std::min(split_m, TRD_PANEL_MAX_M);
  for (int k0 = 0; k0 < m - 1; k0 += TRD_NB) {
    const int nq = std::min(TRD_NB, m - 1 - k0);
    if (nq < TRD_NB) {  // a short last panel: the rows it does not write must not carry the previous panel's
      hipError_t err = hipMemsetAsync(PV, 0, sizeof(double) * 3 * TRD_NB * (size_t)m, s);
      if (err != hipSuccess) return err;
    }
    if (!split) {
      hipLaunchKernelGGL(trd_panel_kernel, dim3(1), dim3(1024), trd_panel_lds(m), s, A, k0, nq);
    } else {
      for (int q = 0; q < nq; ++q) {
        const int j = k0 + q, n1 = m - j - 1;
        hipLaunchKernelGGL(trd_prep_kernel, dim3(1), dim3(1024), 0, s, A, j, q);
        hipLaunchKernelGGL(trd_matvec_kernel, dim3((unsigned)((n1 + 7) / 8)), dim3(256), 0, s, A, j);
        hipLaunchKernelGGL(trd_finish_kernel, dim3(1), dim3(1024), 0, s, A, j, q);
      }
    }
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    const int p0 = k0 + nq;
    if (p0 < m) {  // A22 -= [V Wp] [Wp V]^T over the trailing square (both triangles kept), one K = 2 NB GEMM
      const int64_t n2 = m - p0;
      DgemmArgs g{1, 0, n2, n2, 2 * TRD_NB, PV + p0, m, 0, PV + (int64_t)TRD_NB * m + p0, m, 0,
                  W + (int64_t)p0 * m + p0, m, 0, -1.0, 1.0};
      err = launch_dgemm(g, 1, s);
      if (err != hipSuccess) return err;
    }
  }
  hipLaunchKernelGGL(trd_last_kernel, dim3(1), dim3(64), 0, s, W, m, d);
  return hipGetLastError();
}

static size_t dc_deflate_lds(int k) {
  if (k > DC_LDS_MAX_K) return 16;  // (the arrays live in L.gscr)
  int P2 = 1;
  while (P2 < k) P2 <<= 1;
  return sizeof(double) * ((size_t)P2 + k) + sizeof(int) * ((size_t)P2 + 2 * (size_t)k);
}

hipError_t launch_eig_dc(const double* d, const double* e, int m, const DcLevel& L, double* Q, double* Qg, double* U,
                         hipStream_t s) {
  {
    hipError_t err = ensure_dyn_lds(reinterpret_cast<const void*>(dc_deflate_kernel), dc_deflate_lds(DC_LDS_MAX_K));
    if (err == hipSuccess)  // (a pair's row of up to DC_GATHER_LDS_MAX_K doubles; longer rows are staged in HBM)
      err = ensure_dyn_lds(reinterpret_cast<const void*>(dc_gather_kernel), (size_t)DC_GATHER_LDS_MAX_K * 8);
    if (err != hipSuccess) return err;
  }
  const int64_t mm = (int64_t)m * m;
  hipLaunchKernelGGL(dc_init_kernel, dim3((unsigned)((mm + 255) / 256)), dim3(256), 0, s, d, e, m, L.lam, Q);
  for (int w = 1; w < m; w *= 2) {
    int P = 0;
    while ((2 * P + 1) * w < m) ++P;
    const int R = std::min(2 * P * w, m);  // rows / positions covered by the pairs (an unpaired last block stays)
    const int kmax = std::min(2 * w, m);
    hipLaunchKernelGGL(dc_deflate_kernel, dim3(P), dim3(256), dc_deflate_lds(kmax), s, e, Q, m, w, L);
    hipLaunchKernelGGL(dc_gather_kernel, dim3(R), dim3(64), kmax <= DC_GATHER_LDS_MAX_K ? sizeof(double) * kmax : 0,
                       s, Q, m, w, L, Qg);
    hipLaunchKernelGGL(dc_secular_kernel, dim3((R + 3) / 4), dim3(256), 0, s, m, w, L);
    hipLaunchKernelGGL(dc_zhat_kernel, dim3((R + 255) / 256), dim3(256), 0, s, m, w, L);
    hipLaunchKernelGGL(dc_vec_kernel, dim3((R + 3) / 4), dim3(256), 0, s, m, w, L, U);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    // Q block <- Qg block U block^T for every pair (full pairs batched, a narrower last pair on its own)
    const int full = std::min(P, m / (2 * w));
    if (full > 0) {
      const int k = 2 * w;
      const int64_t bs = (int64_t)k * (m + 1);
      DgemmArgs g{0, 1, k, k, k, Qg, m, bs, U, m, bs, Q, m, bs, 1.0, 0.0};
      err = launch_dgemm(g, full, s);
      if (err != hipSuccess) return err;
    }
    if (full < P) {
      const int64_t a = (int64_t)2 * w * full, k = m - a, o = a * (m + 1);
      DgemmArgs g{0, 1, k, k, k, Qg + o, m, 0, U + o, m, 0, Q + o, m, 0, 1.0, 0.0};
      err = launch_dgemm(g, 1, s);
      if (err != hipSuccess) return err;
    }
  }
  return hipSuccess;
}

hipError_t launch_eig_transpose(const double* A, int m, double* B, hipStream_t s) {
  const unsigned t = (unsigned)((m + 31) / 32);
  hipLaunchKernelGGL(transpose_kernel, dim3(t, t), dim3(256), 0, s, A, m, B);
  return hipGetLastError();
}

hipError_t launch_eig_identity(double* Z, int m, hipStream_t s) {
  const int64_t n = (int64_t)m * m;
  hipLaunchKernelGGL(identity_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, Z, m);
  return hipGetLastError();
}

hipError_t launch_eig_build_y(const double* W, int m, int k0, int nb, double* Y, hipStream_t s) {
  const int64_t n = (int64_t)m * nb;
  hipLaunchKernelGGL(build_y_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, W, m, k0, nb, Y);
  return hipGetLastError();
}

hipError_t launch_eig_larft(const double* G, const double* tau, int k0, int nb, double* S, hipStream_t s) {
  hipLaunchKernelGGL(larft_kernel, dim3(1), dim3(64), 0, s, G, tau, k0, nb, S);
  return hipGetLastError();
}

bool eig_bt_fused(int m) { return m <= BT_MAX_M; }

hipError_t launch_eig_backtransform(const double* W, const double* tau, int m, double* Sall, double* V,
                                    hipStream_t s) {
  const size_t lds = sizeof(double) * ((size_t)BT_MAX_M * BT_CW + BT_RC * (BT_NB + 1) + 2 * BT_NB * BT_CW +
                                       BT_NB * BT_NB);
  {
    hipError_t err = ensure_dyn_lds(reinterpret_cast<const void*>(bt_apply_kernel), lds);
    if (err != hipSuccess) return err;
  }
  const int nblk = (m - 1 + BT_NB - 1) / BT_NB;
  if (nblk == 0) return hipSuccess;
  hipLaunchKernelGGL(bt_larft_kernel, dim3(nblk), dim3(256), 0, s, W, tau, m, Sall);
  const size_t need = sizeof(double) * ((size_t)m * BT_CW + BT_RC * (BT_NB + 1) + 2 * BT_NB * BT_CW + BT_NB * BT_NB);
  hipLaunchKernelGGL(bt_apply_kernel, dim3((unsigned)((m + BT_CW - 1) / BT_CW)), dim3(256), need, s, W, m, Sall, V);
  return hipGetLastError();
}

hipError_t launch_sym_copy(const double* A, int64_t lda, int m, double* W, hipStream_t s) {
  const int64_t n = (int64_t)m * m;
  hipLaunchKernelGGL(sym_copy_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, lda, m, W);
  return hipGetLastError();
}

}  // namespace gpk
