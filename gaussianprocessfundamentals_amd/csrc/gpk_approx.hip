// Dense building blocks of the approximation paths: a batched f64 MFMA GEMM, a
// batched two-sided Jacobi eigensolver (the symmetric pseudo-inverse), the SKI interpolation
// weights and a diagonal add.  None of these is on the exact −LML hot path; they turn the
// reference's Nyström / SKC / SKI matrices (gpbasics/Statistics/Nystroem_K.py,
// gpbasics/Metrics/StructuredKernelInterpolation.py) into dense device matrices that the augmented
// factorisation (gpk_assemble_dense + gpk_potrf_aug) then handles like K.
#include <math.h>

#include "gpk_internal.h"

namespace gpk {
namespace {

typedef double d2 __attribute__((ext_vector_type(2)));

// ============================================================================================ GEMM
// C = alpha op(A) op(B) + beta C (row-major; op(A) M x K, op(B) K x N).  64 x 64 tiles, 256 threads
// = 2 x 2 waves of 32 x 32 (2 x 2 f64 MFMA 16x16x4 blocks).  K is staged 16 at a time in LDS as
// [row][k] (row stride 18 doubles: the 16 rows a quarter-wave reads sit on distinct banks), and the
// MFMA k-step s of lane group q = lane >> 4 takes k = 4 q + s -- the same permutation for both
// operands -- so two ds_read_b128 per 16-row block feed all four k-steps.  Two LDS stages; the next
// chunk's global loads are issued before the current chunk's MFMAs (one barrier per chunk).
constexpr int GT = 64, GKC = 16, GLD = GKC + 2;

struct GemmStage {
  double a[4], b[4];
};

__device__ __forceinline__ void dgemm_fetch(const DgemmArgs& g, const double* A, const double* B, int64_t i0,
                                            int64_t j0, int64_t k0, int tid, GemmStage& st) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid * 4 + u;  // 1024 elements of each operand chunk
    int ii, kk;
    if (g.ta) { kk = e / GT; ii = e % GT; } else { ii = e / GKC; kk = e % GKC; }
    const int64_t gi = i0 + ii, gk = k0 + kk;
    st.a[u] = (gi < g.M && gk < g.K) ? (g.ta ? A[gk * g.lda + gi] : A[gi * g.lda + gk]) : 0.0;
    int jj, kb;
    if (g.tb) { jj = e / GKC; kb = e % GKC; } else { kb = e / GT; jj = e % GT; }
    const int64_t gj = j0 + jj, gkb = k0 + kb;
    st.b[u] = (gj < g.N && gkb < g.K) ? (g.tb ? B[gj * g.ldb + gkb] : B[gkb * g.ldb + gj]) : 0.0;
  }
}

__device__ __forceinline__ void dgemm_store(const DgemmArgs& g, int tid, const GemmStage& st, double* As, double* Bs) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = tid * 4 + u;
    int ii, kk;
    if (g.ta) { kk = e / GT; ii = e % GT; } else { ii = e / GKC; kk = e % GKC; }
    As[ii * GLD + kk] = st.a[u];
    int jj, kb;
    if (g.tb) { jj = e / GKC; kb = e % GKC; } else { kb = e / GT; jj = e % GT; }
    Bs[jj * GLD + kb] = st.b[u];
  }
}

__global__ __launch_bounds__(256) void dgemm_kernel(DgemmArgs g) {
  __shared__ __attribute__((aligned(16))) double As[2][GT * GLD];
  __shared__ __attribute__((aligned(16))) double Bs[2][GT * GLD];
  const int b = blockIdx.z;
  const int64_t i0 = (int64_t)blockIdx.y * GT, j0 = (int64_t)blockIdx.x * GT;
  const double* A = g.A + (int64_t)b * g.a_bs;
  const double* B = g.B + (int64_t)b * g.b_bs;
  double* C = g.C + (int64_t)b * g.c_bs;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int lr = lane & 15, q = lane >> 4;
  d4 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) acc[mi][ni] = d4{0.0, 0.0, 0.0, 0.0};

  GemmStage st;
  dgemm_fetch(g, A, B, i0, j0, 0, tid, st);
  dgemm_store(g, tid, st, As[0], Bs[0]);
  __syncthreads();
  const int nk = (int)((g.K + GKC - 1) / GKC);
  for (int c = 0; c < nk; ++c) {
    const int cur = c & 1;
    if (c + 1 < nk) dgemm_fetch(g, A, B, i0, j0, (int64_t)(c + 1) * GKC, tid, st);
    d2 fa[2][2], fb[2][2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const d2* src = reinterpret_cast<const d2*>(&As[cur][(wr * 32 + mi * 16 + lr) * GLD + 4 * q]);
      fa[mi][0] = src[0];
      fa[mi][1] = src[1];
    }
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const d2* src = reinterpret_cast<const d2*>(&Bs[cur][(wc * 32 + ni * 16 + lr) * GLD + 4 * q]);
      fb[ni][0] = src[0];
      fb[ni][1] = src[1];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mi][s >> 1][s & 1], fb[ni][s >> 1][s & 1],
                                                             acc[mi][ni], 0, 0, 0);
    if (c + 1 < nk) dgemm_store(g, tid, st, As[cur ^ 1], Bs[cur ^ 1]);
    __syncthreads();
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gi = i0 + wr * 32 + mi * 16 + q + 4 * r;  // f64 C/D row = (lane >> 4) + 4 reg
        const int64_t gj = j0 + wc * 32 + ni * 16 + lr;
        if (gi < g.M && gj < g.N) {
          double v = g.alpha * acc[mi][ni][r];
          if (g.beta != 0.0) v += g.beta * C[gi * g.ldc + gj];
          C[gi * g.ldc + gj] = v;
        }
      }
}

// ================================================================================ Jacobi (syevj)
// Two-sided cyclic Jacobi with the round-robin (circle) ordering: sweep = mm - 1 rounds (mm = m
// rounded up to even), every round rotates mm / 2 disjoint index pairs at once, A <- J^T A J,
// V <- V J, out of place (ping-pong buffers).  Each workgroup recomputes the rotations of its 32
// rows and 32 columns from the input matrix; a pair is skipped once |a_pq| <= eps sqrt(|a_pp a_qq|)
// (the relative off-diagonal criterion), and the sweep loop stops after a sweep without rotations.

// partner of index i in round r of the circle method (position 0 fixed, 1 .. mm-1 rotating)
__device__ __forceinline__ int jac_partner(int i, int r, int mm) {
  const int M1 = mm - 1;
  const int k = (i == 0) ? 0 : (((i - 1 - r) % M1) + M1) % M1 + 1;
  const int kp = mm - 1 - k;
  return kp == 0 ? 0 : 1 + (kp - 1 + r) % M1;
}

// rotation seen from index i: new_i = cs x_i + cp x_partner (rows of J^T A, columns of A J)
__device__ __forceinline__ void jac_rotation(const double* A, int m, int i, int j, double tol_abs, int* part,
                                             double* cs, double* cp, int* flag) {
  *part = i;
  *cs = 1.0;
  *cp = 0.0;
  if (i >= m || j >= m || i == j) return;
  const int p = i < j ? i : j, qq = i < j ? j : i;
  const double apq = A[(int64_t)p * m + qq];
  const double app = A[(int64_t)p * m + p], aqq = A[(int64_t)qq * m + qq];
  if (fabs(apq) <= tol_abs || fabs(apq) <= 2.220446049250313e-16 * sqrt(fabs(app) * fabs(aqq))) return;
  const double th = (aqq - app) / (2.0 * apq);
  double t;
  if (fabs(th) > 1e150) t = 0.5 / th;
  else t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(1.0 + th * th));
  const double c = 1.0 / sqrt(1.0 + t * t), s = t * c;
  *part = j;
  *cs = c;
  *cp = (i == p) ? -s : s;
  *flag = 1;
}

constexpr int JT = 32;

__global__ __launch_bounds__(256) void jacobi_round_kernel(JacobiArgs a, int r) {
  __shared__ int rpart[JT], cpart[JT];
  __shared__ double rcs[JT], rcp[JT], ccs[JT], ccp[JT];
  const int b = blockIdx.z;
  const int64_t bs = (int64_t)a.m * a.m;
  const double* A = a.Ain + b * bs;
  const double* V = a.Vin + b * bs;
  double* Ao = a.Aout + b * bs;
  double* Vo = a.Vout + b * bs;
  const int i0 = blockIdx.y * JT, j0 = blockIdx.x * JT;
  const int tid = threadIdx.x;
  if (tid < 2 * JT) {
    const int idx = (tid < JT ? i0 : j0) + (tid % JT);
    int part, fl = 0;
    double cs, cp;
    jac_rotation(A, a.m, idx, idx < a.mm ? jac_partner(idx, r, a.mm) : idx, a.tol_abs, &part, &cs, &cp, &fl);
    if (fl) *a.flag = 1;
    if (tid < JT) { rpart[tid] = part; rcs[tid] = cs; rcp[tid] = cp; }
    else { cpart[tid - JT] = part; ccs[tid - JT] = cs; ccp[tid - JT] = cp; }
  }
  __syncthreads();
  const int jj = tid % JT;
  const int j = j0 + jj;
  if (j >= a.m) return;
  const int jp = cpart[jj];
  const double csj = ccs[jj], cpj = ccp[jj];
  for (int ii = tid / JT; ii < JT; ii += 256 / JT) {
    const int i = i0 + ii;
    if (i >= a.m) break;
    const int ip = rpart[ii];
    const double csi = rcs[ii], cpi = rcp[ii];
    const double x = A[(int64_t)i * a.m + j], xb = A[(int64_t)i * a.m + jp];
    const double xc = A[(int64_t)ip * a.m + j], xd = A[(int64_t)ip * a.m + jp];
    double v = csj * (csi * x + cpi * xc) + cpj * (csi * xb + cpi * xd);
    if (ip == j && jp == i && ip != i) v = 0.0;  // the rotated pair's off-diagonal element
    Ao[(int64_t)i * a.m + j] = v;
    Vo[(int64_t)i * a.m + j] = csj * V[(int64_t)i * a.m + j] + cpj * V[(int64_t)i * a.m + jp];
  }
}

__global__ __launch_bounds__(256) void jacobi_init_kernel(const double* A, int64_t lda, int64_t a_bs, int m,
                                                          double* A0, double* V0) {
  const int b = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t mm = (int64_t)m * m;
  if (e >= mm) return;
  const int64_t i = e / m, j = e % m;
  A0[b * mm + e] = A[b * a_bs + i * lda + j];
  V0[b * mm + e] = (i == j) ? 1.0 : 0.0;
}

// max |A_ii| over every member (the absolute scale of the rotation threshold)
__global__ __launch_bounds__(256) void diag_absmax_kernel(const double* A0, int m, int32_t batch, double* out) {
  __shared__ double red[256];
  const int64_t mm = (int64_t)m * m;
  double mx = 0.0;
  for (int64_t e = threadIdx.x; e < (int64_t)m * batch; e += 256) mx = fmax(mx, fabs(A0[(e / m) * mm + (e % m) * (m + 1)]));
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}

__global__ __launch_bounds__(256) void jacobi_out_kernel(const double* Af, const double* Vf, int m, double* V,
                                                         double* lam) {
  const int b = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t mm = (int64_t)m * m;
  if (e >= mm) return;
  V[b * mm + e] = Vf[b * mm + e];
  const int64_t i = e / m, j = e % m;
  if (i == j) lam[(int64_t)b * m + i] = Af[b * mm + e];
}

// per member: mu_i = 1 / lam_i (mode 0), 1 / sqrt(lam_i) (mode 1) or 1 / sqrt(|lam_i|) (mode 2: the symmetric
// factor of an indefinite pinv, whose signs the caller keeps) for |lam_i| > rcond max|lam|, else 0
// (tf.linalg.pinv's cutoff); rank[b] = kept count, -1 if mode 1 keeps a negative value
__global__ __launch_bounds__(256) void pinv_mu_kernel(const double* lam, int m, double rcond, int mode, double* mu,
                                                      int32_t* rank) {
  __shared__ double red[256];
  __shared__ int cnt[256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const double* l = lam + (int64_t)b * m;
  double mx = 0.0;
  for (int i = tid; i < m; i += 256) mx = fmax(mx, fabs(l[i]));
  red[tid] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] = fmax(red[tid], red[tid + s]);
    __syncthreads();
  }
  const double cut = rcond * red[0];
  int kept = 0, neg = 0;
  for (int i = tid; i < m; i += 256) {
    const double v = l[i];
    double u = 0.0;
    if (fabs(v) > cut) {
      kept += 1;
      if (mode == 0) u = 1.0 / v;
      else if (mode == 2) u = 1.0 / sqrt(fabs(v));
      else if (v > 0.0) u = 1.0 / sqrt(v);
      else neg = 1;
    }
    mu[(int64_t)b * m + i] = u;
  }
  cnt[tid] = kept + (neg << 20);
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) cnt[tid] += cnt[tid + s];
    __syncthreads();
  }
  if (tid == 0) rank[b] = (cnt[0] >> 20) ? -1 : (cnt[0] & ((1 << 20) - 1));
}

// Reverse mode of tf.linalg.pinv on a symmetric matrix A = V diag(lam) V^T (Statistics/Nystroem_K.py:53,
// the gradient TensorFlow's SVD backward gives for the kept singular values): with T = V^T Pbar V,
// Abar = V (F o sym(T)) V^T, F_ij = (f_i - f_j) / (lam_i - lam_j), f = 1/lam on the kept values, 0 on the
// dropped ones (mu of pinv_mu_kernel, mode 0): kept / kept -mu_i mu_j (the same quotient without its
// cancellation), kept i / dropped j mu_i / (lam_i - lam_j), dropped / dropped 0.  In place, one thread per
// pair i <= j.
__global__ __launch_bounds__(256) void pinv_bwd_scale_kernel(const double* lam, const double* mu, int m, double* T) {
  const int b = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t mm = (int64_t)m * m;
  if (e >= mm) return;
  const int i = (int)(e / m), j = (int)(e % m);
  if (j < i) return;
  const double* l = lam + (int64_t)b * m;
  const double* u = mu + (int64_t)b * m;
  double* Tb = T + b * mm;
  const double t = 0.5 * (Tb[(int64_t)i * m + j] + Tb[(int64_t)j * m + i]);
  const double ui = u[i], uj = u[j];
  double f;
  if (ui != 0.0 && uj != 0.0) f = -ui * uj;
  else if (ui != 0.0) f = ui / (l[i] - l[j]);
  else if (uj != 0.0) f = uj / (l[j] - l[i]);
  else f = 0.0;
  Tb[(int64_t)i * m + j] = f * t;
  Tb[(int64_t)j * m + i] = f * t;
}

__global__ __launch_bounds__(256) void scale_cols_kernel(const double* V, const double* mu, int m, double* U) {
  const int b = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t mm = (int64_t)m * m;
  if (e >= mm) return;
  U[b * mm + e] = V[b * mm + e] * mu[(int64_t)b * m + e % m];
}

// ================================================================================ SKI weights
// get_weight_matrix (gpbasics/Metrics/StructuredKernelInterpolation.py:31-49): euclidean distances
// (the expanded norm of Auxiliary/Distances.py:4-7, unclamped) of every training point to every
// inducing point; the nearest (all ties) gets 1 - d1 / (d1 + d2), the second nearest (after adding
// the global maximum distance to the nearest ones) the rest.
__device__ __forceinline__ double ski_dist(const double* x, const double* z, int d) {
  double xx = 0.0, zz = 0.0, xz = 0.0;
  for (int k = 0; k < d; ++k) {
    xx += x[k] * x[k];
    zz += z[k] * z[k];
    xz += x[k] * z[k];
  }
  return sqrt((xx - 2.0 * xz) + zz);
}

// one wave per training point: row minimum and row maximum
__global__ __launch_bounds__(256) void ski_rowstats_kernel(const double* X, int64_t n, const double* Z, int64_t m,
                                                           int d, double* rmin, double* rmax) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  double mn = INFINITY, mx = -INFINITY;
  for (int64_t j = lane; j < m; j += 64) {
    const double v = ski_dist(X + i * d, Z + j * d, d);
    mn = fmin(mn, v);
    mx = fmax(mx, v);
  }
  for (int o = 32; o > 0; o >>= 1) {
    mn = fmin(mn, __shfl_xor(mn, o));
    mx = fmax(mx, __shfl_xor(mx, o));
  }
  if (lane == 0) {
    rmin[i] = mn;
    rmax[i] = mx;
  }
}

__global__ __launch_bounds__(256) void max_reduce_kernel(const double* v, int64_t n, double* out) {
  __shared__ double red[256];
  double mx = -INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += 256) mx = fmax(mx, v[i]);
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}

__global__ __launch_bounds__(256) void ski_weights_kernel(const double* X, int64_t n, const double* Z, int64_t m,
                                                          int d, const double* rmin, const double* gmax,
                                                          double* Wm) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const double d1 = rmin[i], g = *gmax;
  double d2 = INFINITY;
  for (int64_t j = lane; j < m; j += 64) {
    const double v = ski_dist(X + i * d, Z + j * d, d);
    d2 = fmin(d2, v + g * (v == d1 ? 1.0 : 0.0));
  }
  for (int o = 32; o > 0; o >>= 1) d2 = fmin(d2, __shfl_xor(d2, o));
  const double wi = 1.0 - d1 / (d1 + d2);
  for (int64_t j = lane; j < m; j += 64) {
    const double v = ski_dist(X + i * d, Z + j * d, d);
    const double c1 = (v == d1) ? 1.0 : 0.0;
    const double c2 = (v + g * c1 == d2) ? 1.0 : 0.0;
    Wm[i * m + j] = (0.0 + wi * c1) + (1.0 - wi) * c2;
  }
}

__global__ __launch_bounds__(256) void add_diag_kernel(double* A, int64_t n, int64_t lda, int64_t a_bs,
                                                       double value) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) A[(int64_t)blockIdx.y * a_bs + i * lda + i] += value;
}

__global__ __launch_bounds__(256) void copy_lower_kernel(const double* src, int64_t lds, double* dst, int64_t ldd,
                                                         int64_t n) {
  const int64_t i = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j <= i && j < n) dst[i * ldd + j] = src[i * lds + j];
}

// Pairwise distances of Auxiliary/Distances.py, one thread per output element (threads along the
// row of the output: coalesced stores; the row's A point and the B points come through L1 / L2).
// mode 0: euclidian_distance (:4-7), sqrt((|a|^2 - 2 a.b) + |b|^2) unclamped -- NaN where rounding
// makes the argument negative, as the reference; 1: manhattan_distance (:10-12); 2: sqrt(sum (a-b)^2).
__global__ __launch_bounds__(256) void distance_kernel(int mode, const double* __restrict__ A, int64_t a_bs,
                                                       const double* __restrict__ B, int64_t m, int64_t b_bs, int d,
                                                       double* __restrict__ out, int64_t ldo, int64_t o_bs) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= m) return;
  const int64_t i = blockIdx.y;
  const double* a = A + (int64_t)blockIdx.z * a_bs + i * d;
  const double* b = B + (int64_t)blockIdx.z * b_bs + j * d;
  double r;
  if (mode == 0) {
#pragma clang fp contract(off)
    // the reference's arithmetic shape: the norms as reduce_sum of rounded squares (no FMA), the cross
    // term as a matmul (fused multiply-add chain), so that they round differently and a == b can give
    // a slightly negative argument (NaN), as in TensorFlow -- with one shared FMA form it never would
    double na = 0.0, nb = 0.0, ab = 0.0;
    for (int k = 0; k < d; ++k) {
      na += a[k] * a[k];  // contraction off in this block: rounded square, then the add
      nb += b[k] * b[k];
      ab = fma(a[k], b[k], ab);
    }
    r = sqrt((na - 2.0 * ab) + nb);
  } else if (mode == 1) {
    r = 0.0;
    for (int k = 0; k < d; ++k) r += fabs(a[k] - b[k]);
  } else {
    r = 0.0;
    for (int k = 0; k < d; ++k) {
      const double t = a[k] - b[k];
      r += t * t;
    }
    r = sqrt(r);
  }
  out[(int64_t)blockIdx.z * o_bs + i * ldo + j] = r;
}

}  // namespace

hipError_t launch_distance(int mode, const double* A, int64_t n, int64_t a_bs, const double* B, int64_t m,
                           int64_t b_bs, int d, int32_t batch, double* out, int64_t ldo, int64_t o_bs, hipStream_t s) {
  if (n <= 0 || m <= 0 || batch <= 0) return hipSuccess;
  // rows go to gridDim.y and members to gridDim.z (each at most 65535): larger inputs are split into
  // launches over row / member ranges with offset pointers
  constexpr int64_t kMaxGrid = 65535;
  for (int64_t b0 = 0; b0 < batch; b0 += kMaxGrid) {
    const int64_t nb = batch - b0 < kMaxGrid ? batch - b0 : kMaxGrid;
    for (int64_t i0 = 0; i0 < n; i0 += kMaxGrid) {
      const int64_t ni = n - i0 < kMaxGrid ? n - i0 : kMaxGrid;
      hipLaunchKernelGGL(distance_kernel, dim3((unsigned)((m + 255) / 256), (unsigned)ni, (unsigned)nb), dim3(256),
                         0, s, mode, A + b0 * a_bs + i0 * d, a_bs, B + b0 * b_bs, m, b_bs, d,
                         out + b0 * o_bs + i0 * ldo, ldo, o_bs);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

hipError_t launch_copy_lower(const double* src, int64_t lds, double* dst, int64_t ldd, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(copy_lower_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)n), dim3(256), 0, s, src, lds, dst,
                     ldd, n);
  return hipGetLastError();
}

hipError_t launch_dgemm(const DgemmArgs& g, int32_t batch, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || batch <= 0) return hipSuccess;
  dim3 grid((unsigned)((g.N + GT - 1) / GT), (unsigned)((g.M + GT - 1) / GT), (unsigned)batch);
  hipLaunchKernelGGL(dgemm_kernel, grid, dim3(256), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_jacobi_init(const double* A, int64_t lda, int64_t a_bs, int m, double* A0, double* V0,
                              int32_t batch, hipStream_t s) {
  const int64_t mm = (int64_t)m * m;
  hipLaunchKernelGGL(jacobi_init_kernel, dim3((unsigned)((mm + 255) / 256), batch), dim3(256), 0, s, A, lda, a_bs,
                     m, A0, V0);
  return hipGetLastError();
}

hipError_t launch_diag_absmax(const double* A0, int m, int32_t batch, double* out, hipStream_t s) {
  hipLaunchKernelGGL(diag_absmax_kernel, dim3(1), dim3(256), 0, s, A0, m, batch, out);
  return hipGetLastError();
}

hipError_t launch_jacobi_round(const JacobiArgs& a, int r, int32_t batch, hipStream_t s) {
  const unsigned t = (unsigned)((a.m + JT - 1) / JT);
  hipLaunchKernelGGL(jacobi_round_kernel, dim3(t, t, batch), dim3(256), 0, s, a, r);
  return hipGetLastError();
}

hipError_t launch_jacobi_out(const double* Af, const double* Vf, int m, double* V, double* lam, int32_t batch,
                             hipStream_t s) {
  const int64_t mm = (int64_t)m * m;
  hipLaunchKernelGGL(jacobi_out_kernel, dim3((unsigned)((mm + 255) / 256), batch), dim3(256), 0, s, Af, Vf, m, V,
                     lam);
  return hipGetLastError();
}

hipError_t launch_pinv_factor(const double* V, const double* lam, int m, double rcond, int mode, double* mu,
                              double* U, int32_t* rank, int32_t batch, hipStream_t s) {
  hipLaunchKernelGGL(pinv_mu_kernel, dim3(batch), dim3(256), 0, s, lam, m, rcond, mode, mu, rank);
  const int64_t mm = (int64_t)m * m;
  hipLaunchKernelGGL(scale_cols_kernel, dim3((unsigned)((mm + 255) / 256), batch), dim3(256), 0, s, V, mu, m, U);
  return hipGetLastError();
}

hipError_t launch_pinv_bwd_scale(const double* lam, const double* mu, int m, double* T, int32_t batch, hipStream_t s) {
  const int64_t mm = (int64_t)m * m;
  hipLaunchKernelGGL(pinv_bwd_scale_kernel, dim3((unsigned)((mm + 255) / 256), batch), dim3(256), 0, s, lam, mu, m, T);
  return hipGetLastError();
}

hipError_t launch_ski_weights(const double* X, int64_t n, const double* Z, int64_t m, int d, double* Wm,
                              double* work, hipStream_t s) {
  double* rmin = work;
  double* rmax = work + n;
  double* gmax = work + 2 * n;
  const unsigned rows = (unsigned)((n + 3) / 4);
  hipLaunchKernelGGL(ski_rowstats_kernel, dim3(rows), dim3(256), 0, s, X, n, Z, m, d, rmin, rmax);
  hipLaunchKernelGGL(max_reduce_kernel, dim3(1), dim3(256), 0, s, rmax, n, gmax);
  hipLaunchKernelGGL(ski_weights_kernel, dim3(rows), dim3(256), 0, s, X, n, Z, m, d, rmin, gmax, Wm);
  return hipGetLastError();
}

hipError_t launch_add_diag(double* A, int64_t n, int64_t lda, int64_t a_bs, double value, int32_t batch,
                           hipStream_t s) {
  if (n <= 0 || batch <= 0) return hipSuccess;
  hipLaunchKernelGGL(add_diag_kernel, dim3((unsigned)((n + 255) / 256), batch), dim3(256), 0, s, A, n, lda, a_bs,
                     value);
  return hipGetLastError();
}

}  // namespace gpk
