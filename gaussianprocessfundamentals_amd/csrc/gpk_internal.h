// Internal declarations shared by the libgpk translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <utility>

#include "gpk.h"

namespace gpk {

constexpr int NB = 128;     // panel width == update tile edge == diagonal block edge
constexpr int ATILE = 64;   // assemble tile edge

// Dynamic LDS above 64 KB needs hipFuncAttributeMaxDynamicSharedMemorySize, which is a per-device
// attribute of the kernel: raised (never lowered -- one kernel may be launched with several sizes) to the
// largest size requested so far on the device, before the launch that needs it.
inline hipError_t ensure_dyn_lds(const void* fn, size_t bytes) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, size_t> done;
  if (bytes <= 65536) return hipSuccess;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(mu);
  size_t& have = done[{dev, fn}];
  if (have >= bytes) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) have = bytes;
  return e;
}

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

// ----------------------------------------------------------------------------------- launch args
struct AsmArgs {
  const double* hyp;
  int64_t hyp_stride;
  const double* noise;
  int64_t noise_stride;
  const double* X;
  int64_t x_bs;
  const double* Xs;
  int64_t xs_bs;
  const double* E;   // explicit extra rows (NULL: kernel rows of Xs)
  int64_t e_bs;
  const double* y;
  int64_t y_bs;
  void* W;
  int64_t ld;
  int64_t w_bs;
  int64_t n, m, n_pad, y_row, p;
  int32_t d;
  int32_t dp;        // LDS row stride of a point (odd when d is even: no bank conflicts)
  int32_t plain;     // 0 = augmented layout, 1 = plain rectangular kernel matrix
  int32_t uplo;      // plain mode: 1 = write j <= i only
  int64_t ntile;     // augmented: 64-tiles per dimension
  double diag_add;   // plain mode
  int32_t eye;       // augmented: the m extra rows are the identity (E = I, m == n), zero corner
  int64_t tcol_hi;   // augmented: > 0 builds only the tiles of 64-tile columns [0, tcol_hi) (all rows below)
  int32_t generic;   // 1: interior tiles too through the generic per-element loop (bitwise A/B of the fast one)
  // ragged batches (NULL: every member uses n / m): member b uses its first nb[b] training points
  // (rows nb[b] .. n_pad-1 become identity rows) and its first mb[b] test points (zero rows after)
  const int64_t* nb;
  const int64_t* mb;
  // dense mode (gpk_assemble_dense): the training block is read from A (lower triangle, mirrored)
  // instead of evaluated from the kernel program
  const double* A;
  int64_t a_ld;
  int64_t a_bs;
  // set by launch_assemble only (callers leave them): the two-leaf SE + periodic MFMA path's per-point features
  // (pair_feat_kernel: rows of feat_fs doubles [u_1..u_D | C_1..C_D | S_1..S_D | |u|^2 | 0], member stride feat_bs)
  // and per 64-point block (max |u|^2, sin / cos form allowed) in faux; NULL: features staged per tile
  const double* feat;
  const double* faux;
  int64_t feat_bs;
  int32_t feat_fs;
  // set by launch_assemble only: tiles the MFMA fast kernel left (count, then (member, ti, tj) triples); the
  // general instantiation then loops over this list instead of the grid
  const int32_t* tlist;
};

struct GemmArgs {
  void* W;
  int64_t ld;
  int64_t w_bs;
  const void* Binv;  // trsm: inverted diagonal block of this step
  int64_t inv_bs;
  int64_t j0;        // first column of the panel
  int64_t row0;      // first row (and column) of the trailing region
  int32_t nt;        // 128-tiles of the trailing region
  int32_t c_lo, c_hi;  // tile-column range handled by this launch (update)
  int32_t kdepth;      // panel width summed over (multiple of 16): 128, or 256 for the deferred update
  // rows [zlo, zhi) are structurally zero in the panel columns [j0, j0 + kdepth) (identity extra
  // rows: row n_pad + t of E L^-T is zero left of column t); tiles inside the range are skipped
  int64_t zlo, zhi;
  // tiles [bz0, bz0 + bzn) (launch-tile units from row0) lie inside [zlo, zhi): the grid enumerates the
  // remaining tiles only -- tile index t >= bz0 stands for t + bzn (rows and, for the update, columns)
  int32_t bz0, bzn;
  // ragged batches (NULL: uniform): member b's training rows nb[b] .. n_pad-1 are identity rows and
  // its test rows n_pad + mb[b] .. y_row-1 zero rows; tiles of rows that are zero in the panel are skipped
  const int64_t* nb;
  const int64_t* mb;
  int64_t n_pad, y_row, p;
  // fused K build (first trailing update of an m = 0, single-base-node factorisation): the tile's C is
  // evaluated -- k(x_i, x_j) + noise [i == j], identity padding, y row -- instead of loaded; the K
  // build then wrote only the panel columns of the first group
  int32_t band;    // update tile order: 0 row-major lower triangle, B > 0 bands of B tile rows
  int64_t row_end; // rows >= row_end are zero in every panel (0: unknown); MFMAs on them are skipped
  int32_t kbuild;
  int32_t d;
  int64_t n;
  gpk_node node;
  const double* hyp;
  int64_t hyp_stride;
  const double* noise;
  int64_t noise_stride;
  const double* X;
  int64_t x_bs;
  const double* y;
  int64_t y_bs;
};

struct DiagArgs {
  void* W;
  int64_t ld;
  int64_t w_bs;
  void* Winv;
  int64_t inv_bs;
  int64_t j0;
  int64_t kblk;
  int32_t* info;
  int32_t dbg;  // timing-only ablations (GPK_DIAG_DEBUG): 1 no inverse, 2 no potf2, 4 no tile ops,
                // 8 no stores, 16 no step loop, 32 no final block row (diag2)
  int32_t version;  // 2: look-ahead schedule (default), 1: the phase-serial kernel (A/B measurements)
  // Fused panel solve (f64, diag2 only; 0: the diagonal block alone): trsm_tiles + 1 workgroups per
  // member each factor the block like the plain kernel.  After loading the block every workgroup draws
  // a ticket from ctr[b] (zero on entry): the last one to load writes L, L^-1 and info and resets the
  // counter -- so no workgroup can still be reading the block when L overwrites it (workgroups of one
  // launch may start far apart when other streams hold the CUs) -- and ticket t < trsm_tiles solves
  // the 64 rows row0 + 64 t .. +63 of member b against its L^-1 in LDS; the gemm<TRSM> launch of that
  // panel is then skipped.  Rows that are zero in the panel are skipped as in gemm<TRSM> (zlo / zhi,
  // nb / mb).  ctr: per-stream device counters (launches on one stream never overlap).
  int32_t trsm_tiles;
  int64_t row0, p, n_pad, y_row, zlo, zhi;
  const int64_t* nb;
  const int64_t* mb;
  int32_t* ctr;
  uint64_t* prof;  // (GPK_DIAG_PROF builds) per step and wave: s_memtime stamps of the phases, else NULL
  int32_t* half_flag;     // (persistent factorisation) set once block rows 0 .. half_step - 1 of L_kk^-1 are stored
  int32_t half_step;      //   (P phase after which they are; half_flag NULL: no early flag)
  int32_t defer_l_store;  // 1: L_kk stays in LDS only (the persistent factorisation stores it after publishing:
                          // no task of the launch reads it)
  int32_t no_inv_zeros;  // 1: leave the tiles of Winv above the diagonal tiles unwritten (the persistent
                         // factorisation's panel solves never read them; the launch path's TRSM does)
};

// rows of L_kk^-1 behind the diagonal task's early flag (multiples of 16; D publishes after its step rows / 16), for
// chains of more than / at most 32 diagonal blocks
#ifndef GPK_CHAIN_SHALF_ROWS
#define GPK_CHAIN_SHALF_ROWS 96
#endif
#ifndef GPK_CHAIN_SHALF_ROWS_SMALL
#define GPK_CHAIN_SHALF_ROWS_SMALL 112
#endif

// persistent factorisation (gpk_potrf.hip chain_kernel<T>): one member (or a small batch), tasks in host-computed order
struct ChainArgs {
  void* W;               // f64 or f32 (chain_kernel<double> / <float>), like Winv
  int64_t ld;
  void* Winv;
  int32_t* info;
  const int32_t* tasks;  // [ntasks + ntasks_b][4]: type (0 D, 1 S, 2 U32, 3 BLK), panel, slice / block row, block column
  int32_t ntasks;        // tasks of list A (all of them unless xcd_b >= 0)
  int32_t ntasks_b;      // chain_xcd: list B (the diagonal chain's D / S / UQ tasks), claimed first by the workgroups
  int32_t xcd_b;         //   running on XCD xcd_b (up to b_seats of them; -1: one list), then by everyone
  int32_t b_seats;
  int32_t* ctl;          // [0] claim counter (list A), [1] timeout flag, [2] list B's claim counter, [3] B seats
  int32_t* dflag;        // [nblk]: D(k) done
  int32_t* sdone;        // [nblk][nsl]: S(k, r) done
  int32_t* ucnt;         // [nsl][nbc]: panels applied to slice r of block column j
  int32_t* qdone;        // [nblk][nsl]: quarter updates (UQ) of panel k done on slice r of diagonal block k + 1
  int32_t* hflag;        // [nblk]: rows 0 .. 16 half_step - 1 of L_kk^-1 stored (D(k) before its end: the diagonal
                         // chain's S(k, .) start their first column blocks)
  int32_t half_step;     //   (D's step after which it sets hflag)
  int32_t uq;            // D(k) waits for the UQ tasks of panel k - 1 (else for ucnt)
  int32_t nsl, nbc;      // live 32-row slices (the last one holds the y row), live block columns
  int32_t nmem;          // members (task word bits 8..): W + m w_bs, Winv + m inv_bs, info + m, counters + m ctl_stride
  int64_t w_bs, inv_bs, ctl_stride;
  int64_t row_end;       // y_row + 1: rows below are zero
  int64_t timeout;       // per wait, in s_memrealtime ticks (100 MHz)
  int32_t* trace;        // debugging (GPK_CHAIN_TRACE=1, else NULL): host-visible [grid][32] progress words
  int32_t dbg;           // debugging (GPK_CHAIN_DBG): 4 = one diagonal task alone (chain_d_only_kernel)
  int32_t force_abort;   // testing (gpk_tune "chain_force_timeout"): the first wait reports a timeout
  uint64_t* dprof;       // (GPK_DIAG_PROF builds) the D tasks' phase stamps, else NULL
  uint64_t* times;       // profiling (GPK_CHAIN_TIMES=1, else NULL): per task [claimed, inputs ready, wave 0's body done, published, S / U32: loads returned, MFMAs retired] (100 MHz)
};

struct FinArgs {
  const void* W;
  int64_t ld;
  int64_t w_bs;
  int64_t n, m, n_pad, y_row;
  const int32_t* info;
  double* out;
  double* mu;
  double* var;
  const int64_t* nb;  // ragged batches: training points of member b (NULL: n)
};

struct GradArgs {
  const void* W;       // factored augmented matrix with identity extra rows (m == n)
  int64_t ld;
  int64_t w_bs;
  int64_t n, n_pad, y_row;
  const double* hyp;
  int64_t hyp_stride;
  const double* X;
  int64_t x_bs;
  int32_t d;
  int32_t dp;
  int64_t ntile;       // 64-tiles per edge of the n x n training block
  double* part;        // [batch][ntile (ntile + 1) / 2][n_hyp + 1] per-tile partial sums
  double* grad;        // [batch][n_hyp + 1]
  const int32_t* info;
  uint32_t adj_mask[GPK_MAX_NODES];  // per node: nodes whose values multiply its adjoint
};

// gpk_kernel_vjp (gpk_assemble.hip): adjoints of K(X, Z) = kernel(X, Z) for a weight matrix G [n, ldg]
struct VjpArgs {
  const double* hyp;   // [n_hyp] device
  const double* G;     // dense weights, or (G == NULL) the rank-1 weights gu[i] gv[j]
  int64_t ldg;
  const double* gu;
  const double* gv;
  double* part_h;      // [row tiles * column tiles][n_hyp] per-tile partial sums
  double* part_z;      // [row tiles][m][d] (set by launch_vjp)
  int32_t want_z;
  uint32_t adj_mask[GPK_MAX_NODES];
};

struct TrsvArgs {
  const void* W;
  int64_t ld;
  int64_t w_bs;
  const void* Winv;
  int64_t inv_bs;
  double* x;
  int64_t x_bs;
  int64_t kblk;
  int64_t n_pad;
  int32_t trans;
  int64_t n_valid;  // rows / columns of W that exist (n_pad for an augmented matrix; n for a caller's L)
};

// ----------------------------------------------------------------------------------- launchers
bool tune_asm_feat();  // gpk_tune("asm_feat") in effect on this thread
bool tune_asm_f32_fast();  // gpk_tune("asm_f32_fast") in effect on this thread
int tune_asm_f32_chunk();  // gpk_tune("asm_f32_chunk"), clamped to 1 .. 64
hipError_t launch_assemble(const gpk_kdesc& kd, const AsmArgs& a, int dtype, int32_t batch,
                           hipStream_t s);
hipError_t launch_diag(const DiagArgs& a, int dtype, int32_t batch, hipStream_t s);
hipError_t launch_gemm(const GemmArgs& a, int dtype, int mode, int tile, int32_t batch, hipStream_t s);
hipError_t launch_finalize(const FinArgs& a, int dtype, int32_t batch, hipStream_t s);
hipError_t launch_chain(const ChainArgs& a, int dtype, int grid, hipStream_t s);
hipError_t chain_timeouts_read(int64_t* out);  // timed-out persistent launches on this device (synchronous)
hipError_t launch_grad(const gpk_kdesc& kd, const GradArgs& g, int dtype, int32_t batch, hipStream_t s);
size_t vjp_workspace_elems(const gpk_kdesc& kd, int64_t n, int64_t m, int32_t d, bool want_z);
hipError_t launch_vjp(const gpk_kdesc& kd, const VjpArgs& g, const double* X, int64_t n, const double* Z, int64_t m,
                      int32_t d, double* grad_hyp, double* grad_z, hipStream_t s);
hipError_t launch_trsv_diag(const TrsvArgs& a, int dtype, int32_t batch, hipStream_t s);
hipError_t launch_trsv_update(const TrsvArgs& a, int dtype, int32_t batch, hipStream_t s);
hipError_t launch_gemv(const double* A, int64_t n, int64_t m, int64_t lda, const double* x, double* y,
                       double alpha, double beta, hipStream_t s);

// approximation paths (gpk_approx.hip)
struct DgemmArgs {
  int32_t ta, tb;
  int64_t M, N, K;
  const double* A;
  int64_t lda, a_bs;
  const double* B;
  int64_t ldb, b_bs;
  double* C;
  int64_t ldc, c_bs;
  double alpha, beta;
};

struct JacobiArgs {
  const double* Ain;
  double* Aout;
  const double* Vin;
  double* Vout;
  int32_t m, mm;
  int32_t* flag;
  double tol_abs;  // pairs with |a_pq| <= tol_abs are not rotated (besides the relative criterion)
};

hipError_t launch_dgemm(const DgemmArgs& g, int32_t batch, hipStream_t s);
hipError_t launch_jacobi_init(const double* A, int64_t lda, int64_t a_bs, int m, double* A0, double* V0,
                              int32_t batch, hipStream_t s);
hipError_t launch_jacobi_round(const JacobiArgs& a, int r, int32_t batch, hipStream_t s);
hipError_t launch_diag_absmax(const double* A0, int m, int32_t batch, double* out, hipStream_t s);
hipError_t launch_jacobi_out(const double* Af, const double* Vf, int m, double* V, double* lam, int32_t batch,
                             hipStream_t s);
hipError_t launch_pinv_factor(const double* V, const double* lam, int m, double rcond, int mode, double* mu,
                              double* U, int32_t* rank, int32_t batch, hipStream_t s);
// tridiagonal eigensolver (gpk_eig.hip)
hipError_t launch_eig_tridiag(double* W, int m, double* d, double* e, double* tau, double* PV, double* vg,
                              double* yg, int split_m, hipStream_t s);
struct DcLevel {  // divide-and-conquer scratch, every array [m] (pair arrays [m / 2 + 1])
  double *lam, *dK, *zK, *rc, *rs, *root_t, *zhat, *rho;
  double* gscr;  // [5 m]: the deflation's sort arrays of merged blocks too large for LDS
  int32_t *idx, *ord, *rp, *rn, *root_o, *kcnt, *rcnt, *flip;
};
hipError_t launch_eig_dc(const double* d, const double* e, int m, const DcLevel& L, double* Q, double* Qg, double* U,
                         hipStream_t s);
hipError_t launch_eig_transpose(const double* A, int m, double* B, hipStream_t s);
hipError_t launch_eig_identity(double* Z, int m, hipStream_t s);
hipError_t launch_eig_build_y(const double* W, int m, int k0, int nb, double* Y, hipStream_t s);
hipError_t launch_eig_larft(const double* G, const double* tau, int k0, int nb, double* S, hipStream_t s);
bool eig_bt_fused(int m);
hipError_t launch_eig_backtransform(const double* W, const double* tau, int m, double* Sall, double* V,
                                    hipStream_t s);
hipError_t launch_sym_copy(const double* A, int64_t lda, int m, double* W, hipStream_t s);
hipError_t launch_pinv_bwd_scale(const double* lam, const double* mu, int m, double* T, int32_t batch, hipStream_t s);
hipError_t launch_ski_weights(const double* X, int64_t n, const double* Z, int64_t m, int d, double* Wm,
                              double* work, hipStream_t s);
hipError_t launch_copy_lower(const double* src, int64_t lds, double* dst, int64_t ldd, int64_t n, hipStream_t s);
// caller-matrix entries of the §8(b) sketch (gpk_flat.hip)
hipError_t launch_pack_lower(int dtype, const void* A, int64_t lda, int64_t n, int64_t n_pad, int64_t p, void* W,
                             hipStream_t s);
hipError_t launch_unpack_lower(int dtype, const void* W, int64_t ld, int64_t n, void* A, int64_t lda, hipStream_t s);
hipError_t launch_trtri_blocks(const double* L, int64_t ldl, int64_t n, double* Winv, hipStream_t s);
hipError_t launch_posterior_var(const double* V, int64_t n, int64_t m, const double* kdiag, double* var,
                                hipStream_t s);
hipError_t launch_distance(int mode, const double* A, int64_t n, int64_t a_bs, const double* B, int64_t m,
                           int64_t b_bs, int d, int32_t batch, double* out, int64_t ldo, int64_t o_bs, hipStream_t s);
hipError_t launch_add_diag(double* A, int64_t n, int64_t lda, int64_t a_bs, double value, int32_t batch,
                           hipStream_t s);

enum { GEMM_UPDATE = 0, GEMM_TRSM = 1 };

}  // namespace gpk
