// Symmetric eigendecomposition A = V diag(lam) V^T for the pseudo-inverse / slogdet / non-positive-definite
// paths of the metrics (tf.linalg.pinv of K_mm, gpbasics/Statistics/Nystroem_K.py:53; tf.linalg.slogdet / inv /
// pinv of an indefinite K, gpbasics/Metrics/Metrics.py:132-147), tridiagonal route (gpk_syevd):
//
//   1. Householder tridiagonalisation A = Q T Q^T (tridiag_kernel, one 1024-thread workgroup: the trailing
//      matrix is L2-resident for the Nystroem sizes; LAPACK dsytd2's reflectors, v_k stored below the
//      subdiagonal of column k, tau_k apart)
//   2. back-transformation: the reflectors in blocks of 32, compact WY form I - Y S Y^T, applied to T's
//      eigenvectors on the f64 MFMA GEMM (build_y_kernel, larft_kernel, launch_dgemm)
//   3. divide and conquer on T (below): log2 m levels of rank-one merges whose eigenvector updates are MFMA
//      GEMMs; deflation takes the clusters of a kernel matrix's numerically zero tail out of the secular
//      equations (an implicit QL with the rotations applied in parallel measured 87 ms at m = 409: its chain of
//      ~1.5 m^2 dependent rotations is sequential)
// The two-sided Jacobi of gpk_approx.hip (gpk_syevj) stays available; this route replaces its O(m^3)-per-
// sweep rounds (30 sweeps of m - 1 launches at m = 409) with O(m^3) work overall.
#include <float.h>
#include <math.h>

#include "gpk_internal.h"

namespace gpk {
namespace {

constexpr int TT = 1024;  // tridiag_kernel threads

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

// W [m, m] row-major, full symmetric on entry (working copy).  On exit d[0..m-1], e[0..m-2] hold T, tau[k]
// the reflector scalars and W[(k + 1 + i) * m + k] (i >= 1) the reflector vectors v_k (v_k[0] = 1 implicit):
// H_k = I - tau_k v_k v_k^T acts on rows / columns k + 1 .. m - 1, and Q = H_0 H_1 ... H_{m-2}.
__global__ __launch_bounds__(TT) void tridiag_kernel(double* W, int m, double* d, double* e, double* tau) {
  extern __shared__ __attribute__((aligned(16))) double sh[];
  double* v = sh;
  double* p = sh + m;
  double* red = p + m;
  const int tid = threadIdx.x;
  for (int k = 0; k < m - 1; ++k) {
    const int n1 = m - k - 1;
    const int64_t base = (int64_t)(k + 1) * m + (k + 1);  // A22 = W[k + 1 .., k + 1 ..]
    double s = 0.0;
    for (int i = 1 + tid; i < n1; i += TT) {
      const double t = W[(int64_t)(k + 1 + i) * m + k];
      s += t * t;
    }
    s = block_sum(s, red);
    const double alpha = W[(int64_t)(k + 1) * m + k];
    double beta = alpha, tk = 0.0, scale = 0.0;
    if (s > 0.0) {
      beta = -copysign(sqrt(alpha * alpha + s), alpha);
      tk = (beta - alpha) / beta;
      scale = 1.0 / (alpha - beta);
    }
    for (int i = tid; i < n1; i += TT) v[i] = (i == 0) ? 1.0 : W[(int64_t)(k + 1 + i) * m + k] * scale;
    if (tid == 0) {
      d[k] = W[(int64_t)k * m + k];
      e[k] = beta;
      tau[k] = tk;
    }
    __syncthreads();
    for (int i = 1 + tid; i < n1; i += TT) W[(int64_t)(k + 1 + i) * m + k] = v[i];
    if (tk == 0.0) continue;  // H_k = I (wave-uniform)
    // p = tau A22 v (A22 symmetric: column i read as row i, coalesced across threads)
    for (int i = tid; i < n1; i += TT) {
      double acc0 = 0.0, acc1 = 0.0;
      int j = 0;
      for (; j + 1 < n1; j += 2) {
        acc0 = fma(W[base + (int64_t)j * m + i], v[j], acc0);
        acc1 = fma(W[base + (int64_t)(j + 1) * m + i], v[j + 1], acc1);
      }
      if (j < n1) acc0 = fma(W[base + (int64_t)j * m + i], v[j], acc0);
      p[i] = tk * (acc0 + acc1);
    }
    __syncthreads();
    double pv = 0.0;
    for (int i = tid; i < n1; i += TT) pv += p[i] * v[i];
    pv = block_sum(pv, red);
    const double a2 = -0.5 * tk * pv;
    for (int i = tid; i < n1; i += TT) p[i] = fma(a2, v[i], p[i]);  // w
    __syncthreads();
    // A22 -= v w^T + w v^T
    for (int i = tid; i < n1; i += TT) {
      const double vi = v[i], wi = p[i];
      for (int j = 0; j < n1; ++j) {
        const int64_t o = base + (int64_t)j * m + i;
        W[o] = W[o] - (v[j] * wi + p[j] * vi);
      }
    }
    __syncthreads();
  }
  if (tid == 0) d[m - 1] = W[(int64_t)(m - 1) * m + (m - 1)];
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

// One workgroup per pair.  LDS: D[P2] z[k] idx[P2] kept[k] defl[k] red[32]
__global__ __launch_bounds__(256) void dc_deflate_kernel(const double* __restrict__ e, const double* __restrict__ Q,
                                                         int m, int w, DcLevel L) {
  extern __shared__ __attribute__((aligned(16))) double sh[];
  const int p = blockIdx.x, tid = threadIdx.x;
  const int a = 2 * w * p, b = a + w, c = min(a + 2 * w, m), k = c - a;
  int P2 = 1;
  while (P2 < k) P2 <<= 1;
  double* D = sh;
  double* z = D + P2;
  double* red = z + k;
  int* idx = reinterpret_cast<int*>(red + 32);
  int* kept = idx + P2;
  int* defl = kept + k;
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
// kept columns first.  LDS: k doubles.
__global__ __launch_bounds__(64) void dc_gather_kernel(const double* __restrict__ Q, int m, int w, DcLevel L,
                                                       double* __restrict__ Qg) {
  extern __shared__ __attribute__((aligned(16))) double x[];
  const int r = blockIdx.x, lane = threadIdx.x;
  const int p = r / (2 * w);
  const int a = 2 * w * p, c = min(a + 2 * w, m), k = c - a;
  const double* row = Q + (int64_t)r * m + a;
  for (int s = lane; s < k; s += 64) x[s] = row[L.idx[a + s]];
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
  __syncthreads();
  double* out = Qg + (int64_t)r * m + a;
  for (int t = lane; t < k; t += 64) out[t] = x[L.ord[a + t]];
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

__global__ __launch_bounds__(256) void sym_copy_kernel(const double* A, int64_t lda, int m, double* W) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)m * m) return;
  const int64_t i = e / m, j = e % m;
  // the lower triangle, mirrored (what gpk_syevj reads of a symmetric input as well)
  W[e] = (j <= i) ? A[i * lda + j] : A[j * lda + i];
}

}  // namespace

size_t eig_tridiag_lds(int m) { return sizeof(double) * (2 * (size_t)m + 32); }

hipError_t launch_eig_tridiag(double* W, int m, double* d, double* e, double* tau, hipStream_t s) {
  const size_t lds = eig_tridiag_lds(m);
  static bool attr = false;
  if (!attr) {
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(tridiag_kernel),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (err != hipSuccess) return err;
    attr = true;
  }
  hipLaunchKernelGGL(tridiag_kernel, dim3(1), dim3(TT), lds, s, W, m, d, e, tau);
  return hipGetLastError();
}

static size_t dc_deflate_lds(int k) {
  int P2 = 1;
  while (P2 < k) P2 <<= 1;
  return sizeof(double) * ((size_t)P2 + k + 32) + sizeof(int) * ((size_t)P2 + 2 * (size_t)k);
}

hipError_t launch_eig_dc(const double* d, const double* e, int m, const DcLevel& L, double* Q, double* Qg, double* U,
                         hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(dc_deflate_kernel),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)dc_deflate_lds(4096));
    if (err == hipSuccess)
      err = hipFuncSetAttribute(reinterpret_cast<const void*>(dc_gather_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 4096 * 8);
    if (err != hipSuccess) return err;
    attr = true;
  }
  const int64_t mm = (int64_t)m * m;
  hipLaunchKernelGGL(dc_init_kernel, dim3((unsigned)((mm + 255) / 256)), dim3(256), 0, s, d, e, m, L.lam, Q);
  for (int w = 1; w < m; w *= 2) {
    int P = 0;
    while ((2 * P + 1) * w < m) ++P;
    const int R = std::min(2 * P * w, m);  // rows / positions covered by the pairs (an unpaired last block stays)
    const int kmax = std::min(2 * w, m);
    hipLaunchKernelGGL(dc_deflate_kernel, dim3(P), dim3(256), dc_deflate_lds(kmax), s, e, Q, m, w, L);
    hipLaunchKernelGGL(dc_gather_kernel, dim3(R), dim3(64), sizeof(double) * kmax, s, Q, m, w, L, Qg);
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

hipError_t launch_sym_copy(const double* A, int64_t lda, int m, double* W, hipStream_t s) {
  const int64_t n = (int64_t)m * m;
  hipLaunchKernelGGL(sym_copy_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, lda, m, W);
  return hipGetLastError();
}

}  // namespace gpk
