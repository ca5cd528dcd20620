/*
 * gpk.h -- C ABI of libgpk.so, the MI355X (gfx950) exact-GP likelihood engine.
 *
 * This is the drop-in boundary underneath the Python mirror of gpbasics' plugin API.
 * The reference has no native layer: every entry point below replaces a TensorFlow call
 * site on the reference's hot path (citations are relative to
 * Bernsai/GaussianProcessFundamentals main/gpbasics/):
 *
 *   gpk_kernel_matrix  <- Kernel.get_tf_tensor                 KernelBasics/Kernel.py:51-52
 *                         (SE :277-294, PER :440-457, MAT32 :702-720, MAT52 :859-880 of
 *                          KernelBasics/BaseKernels.py; ADD/MUL KernelBasics/Operators.py:207-225,
 *                          :306-326; distances Auxiliary/Distances.py:4-12)
 *   gpk_assemble       <- HolisticCovarianceMatrix.get_K / get_K_noised / get_K_s / get_K_ss
 *                                                               Statistics/CovarianceMatrix.py:187-225, :277-286
 *   gpk_potrf_aug      <- tf.linalg.cholesky + both tf.linalg.triangular_solve of get_L_K /
 *                         get_L_alpha                           Statistics/CovarianceMatrix.py:247-265
 *   gpk_finalize       <- LogLikelihood.get_metric (-LML)       Metrics/LogLikelihood.py:30-65,
 *                         Metrics/Metrics.py:138-139, :152-154;
 *                         posterior mu / var                    Statistics/Auxiliary.py:57-93
 *   gpk_trsv           <- the backward triangular_solve of get_L_alpha
 *                                                               Statistics/CovarianceMatrix.py:260-262
 *   gpk_nlml           <- LogLikelihood.get_metric, composed of the three calls above
 *
 * Conventions
 *  - Every device buffer is allocated and owned by the caller (PyTorch-ROCm); the library
 *    never allocates or frees caller memory and never synchronises the stream.
 *  - Points are row-major fp64: X[batch][n][d] with a caller-given batch stride (0 =
 *    shared by every batch member), y[batch][n], hyperparameters hyp[batch][n_hyp] fp64.
 *  - Return value: 0 on success, -i for an invalid i-th argument, > 0 for a HIP error
 *    code.  A matrix that is not positive definite is NOT an error of the call: it is
 *    reported through info_dev[b] (LAPACK convention: 1-based index of the first
 *    non-positive pivot, 0 when the factorisation succeeded).  info_dev[b] = -1 is an
 *    infrastructure failure of the persistent factorisation (a bounded wait timed out, gpk_tune
 *    "chain"), never "not positive definite": that member's results are undefined and the call must
 *    be repeated with gpk_tune("chain", 0) (or gpk_tune_thread).  Every entry that factors a single
 *    f64 member, or a batch of at most "chain_max_batch" members, can report it -- gpk_nlml,
 *    gpk_potrf_aug(_ex), gpk_nlml_batched, gpk_potrf_lower included.
 *  - gpk_last_error() returns a thread-local description of the last failure.
 *  - `stream` is a hipStream_t passed as void* (0 = the null stream).
 *
 * Augmented layout: the engine factors one matrix per batch member
 *
 *      W = [ K + noise*I    .      .  ]   rows 0 .. n_pad-1   (padding rows: identity)
 *          [ Ks^T          Kss     .  ]   rows n_pad .. n_pad+m-1
 *          [ y^T            0      0  ]   row  y_row = n_pad+m
 *
 * over its first n_pad columns only.  Afterwards the first n_pad columns hold L, the test
 * rows hold V^T = Ks^T L^-T, the y row holds z^T = (L^-1 y)^T and the trailing corner holds
 * the Schur complement  [[Kss - V^T V, .], [-mu^T, -z^T z]]: posterior covariance,
 * posterior mean and the data-fit term of the LML fall out of one factorisation.
 */
#ifndef GPK_H
#define GPK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPK_ABI_VERSION 6

/* arithmetic types of the factorisation */
enum { GPK_F64 = 0, GPK_F32 = 1 };

/* kernel-tree op codes: values follow KernelManifestation (KernelBasics/Kernel.py:23-37) */
enum {
  GPK_OP_PER = 104,
  GPK_OP_SE = 105,
  GPK_OP_MAT32 = 107,
  GPK_OP_MAT52 = 108,
  GPK_OP_ADD = 201, /* binary: pops two, pushes sum (left fold of an n-ary ADD) */
  GPK_OP_MUL = 202  /* binary: pops two, pushes product                         */
};

/* per-node flags of a base-kernel node */
enum {
  GPK_NODE_SCALED = 1,     /* p_scaled_base_kernel: signal variance sg multiplies the kernel */
  GPK_NODE_ARD = 2,        /* build extension: one length scale per input dimension          */
  GPK_NODE_SE_EXPANDED = 4, /* SE distance by the reference's expanded norm (Distances.py:5-7) */
  GPK_NODE_STANDARD = 8     /* MAT: Euclidean distance; PER: sum_d sin^2 per dimension (build
                               option; equal to the reference's L1 forms when d == 1)          */
};

#define GPK_MAX_NODES 16
#define GPK_MAX_DIM 16
#define GPK_MAX_ARD 2
#define GPK_MAX_HYP 64

/* one postfix-program node */
typedef struct {
  int32_t op;         /* GPK_OP_*                                               */
  int32_t hyp_offset; /* first hyperparameter of a base node inside hyp[b][:]   */
  int32_t ard_slot;   /* 0..GPK_MAX_ARD-1 for GPK_NODE_ARD nodes, else -1       */
  int32_t flags;      /* GPK_NODE_*                                             */
} gpk_node;

/* kernel tree flattened to postfix (children left to right, binary ADD/MUL after each
 * child beyond the first), hyperparameters in the reference's DFS order */
typedef struct {
  int32_t n_nodes;
  int32_t n_hyp;
  int32_t dim;
  int32_t n_ard;
  gpk_node nodes[GPK_MAX_NODES];
} gpk_kdesc;

/* sizes of the augmented factorisation of one problem shape */
typedef struct {
  int32_t dtype;          /* GPK_F64 / GPK_F32                                   */
  int32_t batch;          /* independent problems factored by every launch       */
  int64_t n;              /* training points                                     */
  int64_t m;              /* test points carried through the factorisation       */
  int64_t d;              /* input dimensions                                    */
  int64_t nb;             /* panel width (columns per factorisation step)        */
  int64_t n_pad;          /* factored columns: n rounded up to nb                */
  int64_t y_row;          /* row holding y (= n_pad + m)                         */
  int64_t p;              /* rows and columns of W (multiple of nb)              */
  int64_t ld;             /* leading dimension of W in elements                  */
  int64_t w_batch_stride; /* elements between consecutive batch members of W     */
  int64_t inv_batch_stride; /* elements between batch members of Winv            */
  size_t w_bytes;         /* bytes of W for the whole batch                      */
  size_t inv_bytes;       /* bytes of Winv (inverted diagonal blocks), whole batch */
} gpk_layout;

int gpk_abi_version(void);
const char* gpk_last_error(void);

/* fill *out for the given shape (no device work) */
int gpk_plan(int dtype, int32_t batch, int64_t n, int64_t m, int64_t d, gpk_layout* out);

/* Build W (see layout above) for every batch member.  hyp_dev[b*hyp_stride ...],
 * noise_dev[b*noise_stride]; X/Xs/E/y batch strides in elements (0 = shared).
 * The m extra rows are either kernel rows k(Xs_t, X_j) with the Kss corner (E == NULL), or the
 * explicit dense rows E[b][t][j] (t < m, j < n) with a zero corner (Xs ignored): E = I gives
 * L^-T in the extra rows and -K^-1 in the corner.  Xs and E may both be NULL when m == 0. */
int gpk_assemble(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev,
                 int64_t hyp_stride, const double* noise_dev, int64_t noise_stride,
                 const double* X, int64_t x_bstride, const double* Xs, int64_t xs_bstride,
                 const double* E, int64_t e_bstride, const double* y, int64_t y_bstride,
                 void* W, void* stream);

/* Blocked right-looking Cholesky of the first n_pad columns of every W, all rows.
 * Winv receives the inverted nb x nb diagonal blocks (needed by gpk_trsv).
 * info_dev[batch] must be zeroed by the caller before the call. */
int gpk_potrf_aug(const gpk_layout* lay, void* W, void* Winv, int32_t* info_dev, void* stream);

/* gpk_potrf_aug with flags: GPK_AUG_EXTRA_IDENTITY declares that the m (= n) extra rows were
 * assembled as the identity (gpk_assemble_inverse); row n_pad + t of E L^-T is then zero left of
 * column t, so every panel-solve and trailing-update tile made of such zero rows is skipped and the
 * factorisation costs n^3 flops instead of 7 n^3 / 3 (potrf + trtri + lauum, the work of
 * tf.linalg.inv(L) and L^-T L^-1 in get_L_inv_K / get_K_inv, Statistics/CovarianceMatrix.py:267-275). */
#define GPK_AUG_EXTRA_IDENTITY 1
int gpk_potrf_aug_ex(const gpk_layout* lay, void* W, void* Winv, int32_t* info_dev, int32_t flags,
                     void* stream);
/* gpk_assemble with E = I (layout planned with m = n) without materialising E: after
 * gpk_potrf_aug_ex(.., GPK_AUG_EXTRA_IDENTITY, ..) the extra rows hold L^-T (upper triangle),
 * the corner -K^-1 (lower triangle) and the corner's y row -alpha^T. */
int gpk_assemble_inverse(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev,
                         int64_t hyp_stride, const double* noise_dev, int64_t noise_stride,
                         const double* X, int64_t x_bstride, const double* y, int64_t y_bstride,
                         void* W, void* stream);
/* Read the results out of a factored W.  out_dev[b*4 + {0,1,2,3}] =
 * {nlml, fit = y^T alpha, logdet = 2 sum log L_ii, n}; nlml = +inf where info != 0.
 * mu_dev[b*m + t] = posterior mean (may be NULL), var_dev[b*m + t] = posterior variance
 * diagonal (may be NULL). */
int gpk_finalize(const gpk_layout* lay, const void* W, const int32_t* info_dev,
                 double* out_dev, double* mu_dev, double* var_dev, void* stream);

/* assemble + potrf_aug + finalize with m = 0 */
int gpk_nlml(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev,
             int64_t hyp_stride, const double* noise_dev, int64_t noise_stride,
             const double* X, int64_t x_bstride, const double* y, int64_t y_bstride,
             void* W, void* Winv, int32_t* info_dev, double* out_dev, void* stream);

/* -LML and its gradient for every batch member (layout planned with m = n):
 *   gpk_assemble_inverse + gpk_potrf_aug_ex(GPK_AUG_EXTRA_IDENTITY) + gpk_finalize, then
 *   grad_dev[b*(n_hyp+1) + p] = d(-LML)/d hyp[p] (p < n_hyp, DFS order of the kernel tree) and
 *   grad_dev[b*(n_hyp+1) + n_hyp] = d(-LML)/d noise, from
 *   1/2 sum_ij ((K^-1)_ij - alpha_i alpha_j) dK_ij/d theta  -- the derivative the reference takes by
 *   tf.GradientTape through LogLikelihood.get_metric (Optimizer/Fitter.py:104-158).
 * grad_dev may be NULL (then only -LML and the inverse, e.g. for get_K_inv); NaN where info != 0.
 * work: device scratch of gpk_grad_workspace_bytes(kd, lay) bytes. */
size_t gpk_grad_workspace_bytes(const gpk_kdesc* kd, const gpk_layout* lay);
int gpk_nlml_grad(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev, int64_t hyp_stride,
                  const double* noise_dev, int64_t noise_stride, const double* X, int64_t x_bstride,
                  const double* y, int64_t y_bstride, void* W, void* Winv, int32_t* info_dev,
                  double* out_dev, double* grad_dev, void* work, size_t work_bytes, void* stream);
/* Ragged batches: independent problems of different sizes factored by the same launches.
 * Replaces the per-segment loops of SegmentedCovarianceMatrix.get_K_noised_blocks / get_L_K_blocks /
 * get_L_alpha_blocks (Statistics/CovarianceMatrix.py:346-357, :445-456, :469-484) and the per-block
 * LogLikelihood of BlockwiseLogLikelihood.get_metric (Metrics/LogLikelihood.py:68-104), which the
 * reference runs one TensorFlow Cholesky after another.
 * The layout is planned for the largest member (n = max n_b, m = max m_b); member b uses the first
 * n_dev[b] points of X[b] / y[b] and the first m_dev[b] points of Xs[b] (device int64 arrays,
 * 1 <= n_dev[b] <= n, 0 <= m_dev[b] <= m).  Its rows n_dev[b] .. n_pad-1 are assembled as identity
 * rows (contributing log 1 = 0 to the log-determinant and 0 to the data fit) and its test rows past
 * m_dev[b] as zero rows; the factorisation skips every tile made of such rows.  m_dev may be NULL
 * when the layout has m = 0.  Results are those of each member factored on its own:
 * out_dev[b*4 + 3] = n_dev[b] and the -LML uses n_dev[b] in its normalising constant.
 * The flop counts of gpk_timing_read for ragged launches are those of the padded problem. */
int gpk_assemble_ragged(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev,
                        int64_t hyp_stride, const double* noise_dev, int64_t noise_stride,
                        const double* X, int64_t x_bstride, const double* Xs, int64_t xs_bstride,
                        const double* y, int64_t y_bstride, const int64_t* n_dev, const int64_t* m_dev,
                        void* W, void* stream);
int gpk_potrf_aug_ragged(const gpk_layout* lay, void* W, void* Winv, int32_t* info_dev,
                         const int64_t* n_dev, const int64_t* m_dev, void* stream);
int gpk_finalize_ragged(const gpk_layout* lay, const void* W, const int32_t* info_dev, const int64_t* n_dev,
                        double* out_dev, double* mu_dev, double* var_dev, void* stream);
/* gpk_assemble_ragged + gpk_potrf_aug_ragged + gpk_finalize_ragged with m = 0 */
int gpk_nlml_ragged(const gpk_kdesc* kd, const gpk_layout* lay, const double* hyp_dev, int64_t hyp_stride,
                    const double* noise_dev, int64_t noise_stride, const double* X, int64_t x_bstride,
                    const double* y, int64_t y_bstride, const int64_t* n_dev, void* W, void* Winv,
                    int32_t* info_dev, double* out_dev, void* stream);

/* Plain kernel matrix K[i*ldk + j] = k(X_i, Y_j) (+ diag_add where i == j) for i < n, j < m.
 * uplo: 0 = full, 1 = lower triangle only.  dtype selects the stored element type. */
int gpk_kernel_matrix(const gpk_kdesc* kd, const double* hyp_dev, int dtype, int uplo,
                      const double* X, int64_t n, const double* Y, int64_t m, int32_t d,
                      double diag_add, void* K, int64_t ldk, void* stream);

/* Triangular solve with the factor held in W (first n_pad columns):
 *   trans = 0: x <- L^-1 x      trans = 1: x <- L^-T x
 * x is fp64 of length n_pad per batch member (batch stride n_pad; entries >= n must be 0). */
int gpk_trsv(const gpk_layout* lay, int trans, const void* W, const void* Winv, double* x,
             void* stream);

/* y <- alpha A x + beta y for a row-major fp64 matrix A [n, m] (leading dimension lda >= m).
 * The matrix-vector products of the non-Cholesky numerical handlings of the metrics:
 * A p_k of linear_cg (Auxiliary/LinearConjugateGradients.py:44-45) and inv(K) y of
 * get_alpha_strict_inverse (Metrics/Metrics.py:132-133).  Timed under class 5. */
int gpk_gemv(const double* A, int64_t n, int64_t m, int64_t lda, const double* x, double* y, double alpha,
             double beta, void* stream);

/* ------------------------------------------------------ workspace-style entries
 * The flat signatures of the survey's boundary sketch: one caller scratch buffer of
 * gpk_workspace_bytes(op, dtype, n, m, batch) bytes replaces the layout and W / Winv (the sketch's
 * gpk_trsv_lower / gpk_posterior take that buffer as two extra arguments).  The single-problem gpk_nlml of
 * the sketch is gpk_nlml_batched with batch = 1.  GPK_WS_POTRF: fp64 or fp32; GPK_WS_TRSV, GPK_WS_POSTERIOR
 * (m = test points): fp64.  0 for an unsupported combination. */
enum { GPK_WS_NLML = 0, GPK_WS_POTRF = 1, GPK_WS_TRSV = 2, GPK_WS_POSTERIOR = 3 };
size_t gpk_workspace_bytes(int op, int dtype, int64_t n, int64_t m, int32_t batch);

/* x <- L^-1 x (trans 0) or L^-T x (trans 1) for a caller's lower-triangular fp64 L [n, ldl] (row-major, the
 * upper triangle not read) and a device vector x [n]: the triangular_solve of get_L_alpha
 * (Statistics/CovarianceMatrix.py:256-265) on an arbitrary factor.  The 128 x 128 diagonal blocks of L are
 * inverted once into the workspace (forward substitution), then the blocked solve of gpk_trsv runs on L itself. */
int gpk_trsv_lower(int dtype, int trans, const double* L, int64_t n, int64_t ldl, double* x, void* work,
                   size_t work_bytes, void* stream);

/* Posterior of a GP from a caller's factor L [n, ldl] of K + noise I and alpha = (K + noise I)^-1 y
 * (Statistics/Auxiliary.py:57-103, GaussianProcess.predict): mu [m] = K_s^T alpha (may be NULL) and, if var is not
 * NULL, var_mode 0: var [m] = diag(K_ss - V^T V), var_mode 1: var [m, ldv] = K_ss - V^T V, with K_s = k(X, Xs),
 * V = L^-1 K_s (blocked, MFMA GEMMs against the inverted diagonal blocks).  var_mode 0 takes k(x*, x*) from the
 * first test point (every kernel of a descriptor is stationary).  fp64.  (The augmented factorisation's test rows
 * -- gpk_assemble with Xs + gpk_potrf_aug + gpk_finalize -- give the same without a separate pass over L.) */
int gpk_posterior(const gpk_kdesc* kd, const double* hyp_dev, int dtype, const double* L, int64_t ldl,
                  const double* alpha, const double* X, int64_t n, const double* Xs, int64_t m, int32_t d,
                  int32_t var_mode, double* mu, double* var, int64_t ldv, void* work, size_t work_bytes,
                  void* stream);

/* -LML of `batch` hyperparameter / noise candidates on shared X [n, d], y [n] (device):
 * hyp_dev [batch][kd->n_hyp], noise_dev [batch], nlml_dev [batch] (+inf where info_dev[b] != 0; info_dev[b] = -1:
 * the persistent launch timed out, see Conventions -- repeat the call with gpk_tune("chain", 0)).
 * LogLikelihood.get_metric for each candidate (Metrics/LogLikelihood.py:30-65). */
int gpk_nlml_batched(const gpk_kdesc* kd, int32_t batch, const double* hyp_dev, const double* noise_dev, int dtype,
                     const double* X, const double* y, int64_t n, int32_t d, void* work, size_t work_bytes,
                     double* nlml_dev, int32_t* info_dev, void* stream);

/* In-place lower Cholesky of a row-major fp64 (double*) or fp32 (float*, dtype GPK_F32: factored on the f32
 * MFMA path) A [n, lda] (upper triangle untouched, LAPACK potrf semantics) through the blocked MFMA
 * factorisation: tf.linalg.cholesky of get_L_K
 * (Statistics/CovarianceMatrix.py:247-254).  *info_dev: 0 or the first non-positive pivot
 * (1-based), or -1 when the persistent launch timed out (A undefined; see Conventions); *logdet_dev (may be
 * NULL) = 2 sum log diag L (Metrics/Metrics.py:152-154). */
int gpk_potrf_lower(int dtype, void* A, int64_t n, int64_t lda, void* work, size_t work_bytes, int32_t* info_dev,
                    double* logdet_dev, void* stream);

/* ---------------------------------------------------------------- approximation paths (§8f.4)
 * Building blocks of the Nyström / SKC / SKI matrices of the reference
 * (Statistics/Nystroem_K.py, Metrics/SkcLogLikelihood.py, Metrics/StructuredKernelInterpolation.py);
 * the resulting dense matrices are factored through gpk_assemble_dense + gpk_potrf_aug. */

/* Training block of the augmented matrix from a caller matrix A [n, lda] (fp64; the lower
 * triangle is read and mirrored) + noise[b] on its diagonal, instead of a kernel evaluation
 * (the metrics' get_covariance_matrix for an approximate K, Metrics/Metrics.py:113-126).  Extra
 * rows: E [m, n] (corner 0: it becomes -E A^-1 E^T) or, with eye != 0 and a layout planned with
 * m = n, the identity (corner -A^-1 after gpk_potrf_aug_ex(GPK_AUG_EXTRA_IDENTITY)). */
int gpk_assemble_dense(const gpk_layout* lay, const double* A, int64_t lda, int64_t a_bstride,
                       const double* noise_dev, int64_t noise_stride, const double* E, int64_t e_bstride,
                       int32_t eye, const double* y, int64_t y_bstride, void* W, void* stream);

/* C <- alpha op(A) op(B) + beta C, row-major fp64, op(A) [M, K], op(B) [K, N], batched by
 * strides (f64 MFMA 16x16x4, 64 x 64 tiles): the tf.matmul / tf.tensordot products of
 * Nystroem_K.py:62, :81-88, :98-104 and StructuredKernelInterpolation.py:25. */
int gpk_dgemm(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t K, double alpha,
              const double* A, int64_t lda, int64_t a_bstride, const double* B, int64_t ldb, int64_t b_bstride,
              double beta, double* C, int64_t ldc, int64_t c_bstride, int32_t batch, void* stream);

/* Symmetric eigendecomposition A = V diag(lam) V^T (V [m, m] row-major, eigenvectors in its
 * columns) by two-sided cyclic Jacobi (round-robin pairs, one launch per round), batched.  The
 * spectral half of tf.linalg.pinv (Nystroem_K.py:53).  Synchronises the stream once per sweep;
 * *sweeps_out = sweeps run (the last one without rotations).  work: gpk_syevj_workspace_bytes. */
size_t gpk_syevj_workspace_bytes(int64_t m, int32_t batch);
int gpk_syevj(int64_t m, int32_t batch, const double* A, int64_t lda, int64_t a_bstride, double* V, double* lam,
              void* work, size_t work_bytes, int32_t max_sweeps, int32_t* sweeps_out, void* stream);

/* Symmetric eigendecomposition, tridiagonal route (the default of the metrics): Householder
 * tridiagonalisation, divide and conquer on the tridiagonal matrix (deflation, Gu-Eisenstat eigenvectors,
 * MFMA GEMM merges), compact-WY back-transformation on the f64 MFMA GEMM.  Same outputs as gpk_syevj
 * (V [m, m] row-major, eigenvectors in its columns; lam in no particular order); A's lower triangle is read.
 * m <= 46340 (merged blocks above 4096 rows sort in the workspace instead of LDS, and above 16384 rows their
 * gather stages each row in the workspace too).  Asynchronous on the stream.
 * work: gpk_syevd_workspace_bytes(m) (reused across the batch). */
size_t gpk_syevd_workspace_bytes(int64_t m);
int gpk_syevd(int64_t m, int32_t batch, const double* A, int64_t lda, int64_t a_bstride, double* V, double* lam,
              void* work, size_t work_bytes, void* stream);

/* U = V diag(mu) with mu_i = 1 / lam_i (mode 0; pinv = U V^T), 1 / sqrt(lam_i) (mode 1;
 * pinv = U U^T) or 1 / sqrt(|lam_i|) (mode 2; pinv = U diag(sign lam) U^T, for an indefinite matrix) for
 * |lam_i| > rcond max|lam| and 0 otherwise -- tf.linalg.pinv's cutoff (rcond < 0: its default 10 m eps).
 * rank_dev[b] = kept eigenvalues, -1 if mode 1 keeps a negative one. */
int gpk_pinv_factor(int64_t m, int32_t batch, const double* V, const double* lam, double rcond, int32_t mode,
                    double* mu, double* U, int32_t* rank_dev, void* stream);

/* Reverse mode of pinv for symmetric matrices (tf.linalg.pinv, Nystroem_K.py:53, as TensorFlow's tape
 * differentiates it): with lam, V the eigendecomposition (gpk_syevd or gpk_syevj) and mu the mode-0 factors of
 * gpk_pinv_factor, and T = V^T Pbar V for the adjoint Pbar of pinv(A), replaces T (in place, [batch, m, m])
 * by F o (T + T^T)/2 with F_ij = (mu_i - mu_j) / (lam_i - lam_j) (-mu_i mu_j for two kept values, 0 for two
 * dropped ones); the adjoint of A is then V T V^T. */
int gpk_pinv_backward_scale(int64_t m, int32_t batch, const double* lam, const double* mu, double* T, void* stream);

/* SKI interpolation weights W [n, m] (row-major) of training points X [n, d] on inducing points
 * Z [m, d]: get_weight_matrix (StructuredKernelInterpolation.py:31-49), expanded-norm euclidean
 * distances, nearest (all ties) 1 - d1 / (d1 + d2), second nearest d1 / (d1 + d2).
 * work: 2 n + 1 doubles. */
int gpk_ski_weights(const double* X, int64_t n, const double* Z, int64_t m, int32_t d, double* Wm, double* work,
                    void* stream);

/* Pairwise distance matrices out[b] [n, m] (row stride ldo) of A[b] [n, d] and B[b] [m, d] (row-major),
 * replacing gpbasics/Auxiliary/Distances.py: mode 0 euclidian_distance (:4-7, the expanded norm
 * sqrt(|a|^2 - 2 a.b + |b|^2), unclamped: NaN where rounding makes it negative), 1 manhattan_distance
 * (:10-12), 2 the direct euclidean sqrt(sum (a - b)^2).  Batch strides 0 broadcast one operand. */
int gpk_distance_matrix(int mode, const double* A, int64_t n, int64_t a_bstride, const double* B, int64_t m,
                        int64_t b_bstride, int32_t d, int32_t batch, double* out, int64_t ldo, int64_t o_bstride,
                        void* stream);

/* Reverse mode of the kernel matrix K = kernel(X, Z) (X [n, d], Z [m, d], hyp_dev [kd->n_hyp], all
 * device fp64) for a weight matrix G [n, ldg] -- or, with G = NULL, the rank-1 weights G_ij = gu[i] gv[j]
 * (gu [n], gv [m]) -- (the adjoint of K, e.g. what tf.GradientTape hands back
 * to get_tf_tensor, Optimizer/Fitter.py:124-132 / :155-156, through the Nystroem metrics'
 * K_nm and K_mm, Statistics/Nystroem_K.py:36-47):
 *   grad_hyp[p]     = sum_ij G_ij dK_ij / d hyp_p        (device [n_hyp]; may be NULL if n_hyp == 0)
 *   grad_z[j*d + k] = sum_i  G_ij dK_ij / d Z_jk         (device [m, d]; NULL: not computed)
 * For a symmetric K(Z, Z) pass X = Z and G + G^T: grad_z is then the full derivative and grad_hyp
 * twice the hyperparameter adjoint.  Derivatives of the distance terms at coincident points are 0
 * (tf.abs' sign(0); TensorFlow would give NaN through the SE kernel's sqrt-then-square there).
 * work: gpk_kernel_vjp_workspace_bytes(kd, n, m, d, grad_z != NULL).  Deterministic (fixed-order
 * reductions). */
size_t gpk_kernel_vjp_workspace_bytes(const gpk_kdesc* kd, int64_t n, int64_t m, int32_t d, int32_t want_z);
int gpk_kernel_vjp(const gpk_kdesc* kd, const double* hyp_dev, const double* X, int64_t n, const double* Z, int64_t m,
                   int32_t d, const double* G, int64_t ldg, const double* gu, const double* gv, double* grad_hyp,
                   double* grad_z, void* work, size_t work_bytes, void* stream);

/* A[b] += value * I (the "+ tf.eye(n) * noise" of Nystroem_K.py:68-69 and
 * StructuredKernelInterpolation.py:27). */
int gpk_add_diagonal(double* A, int64_t n, int64_t lda, int64_t a_bstride, int32_t batch, double value,
                     void* stream);

/* Per-kernel-class timing with HIP events recorded on the launch stream.
 * class: 0 assemble, 1 diag, 2 trsm, 3 update, 4 finalize, 5 trsv, 6 grad */
#define GPK_NUM_CLASSES 7
int gpk_timing_enable(int on);
/* synchronises the recorded events; returns totals since the last reset */
int gpk_timing_read(double* ms_by_class, int64_t* launches_by_class, double* flops_by_class,
                    double* bytes_by_class);
int gpk_timing_reset(void);

/* Scheduling knobs of the factorisation (no reference counterpart: tf.linalg.cholesky exposes
 * none).  Keys: "lookahead" (1: panel chain on a high-priority stream overlapping the bulk
 * trailing update, 0: one stream, 2: auto -- on from "la_min_blocks" (64) 128-blocks of the augmented
 * matrix, the default), "panel_stream" (the look-ahead's chain: 0 high-priority side stream, 1 the
 * caller's, 2 a normal-priority side stream), "fuse_trsm" (f64 panel solve inside the diagonal-block
 * launch while batch x (64-row tiles + 1) <= "fuse_trsm_max": 1 with the look-ahead off, 2 always,
 * 0 never; bitwise identical results; callers that overlap factorisations on several streams set
 * 0), "reserve_cus" (CUs masked off the bulk-update stream; read
 * when that stream is first created), "group" (panels per trailing update, K = 128 group), "group_first"
 * (panels of the first group), "fuse_kbuild" (K build inside the first trailing update),
 * "upd_band" (trailing-update tile order), "skip_zero_rows" (skip the MFMAs of the zero rows below
 * the y row), "upd_t128_min", "trsm_t128_min" (128-tile thresholds), "diag_version" (2: look-ahead
 * diagonal-block kernel, 1: the phase-serial one; bitwise identical results), "ingroup" (in-group
 * updates: 0 auto, 1 left-looking, 2 right-looking, 3 two-level left-looking) with "rl_max_tiles"
 * (auto picks right-looking while batch x block rows stays below it, two-level otherwise),
 * "band_skip" (1: with identity extra rows, the grid leaves out the tiles of the structurally zero
 * band instead of launching them to exit at once), "group_eye" (panels per trailing update of the
 * identity-augmented factorisations, gpk_potrf_aug_ex / gpk_nlml_grad; "group" for the others),
 * "asm_generic" (1: the K build's interior tiles through the generic per-element loop as well; the
 * same bits, slower -- for A/B checks), "trd_split_m" (gpk_syevd: above this m, at most 1024, the
 * tridiagonalisation's A22 v runs over the chip, three launches per column, instead of one workgroup per
 * panel; default 1024), "chain" (every f64, batch-1, non-ragged factorisation with at most
 * "chain_max_p" (12416) rows -- identity-augmented ones (gpk_potrf_aug_ex, gpk_nlml_grad) while "chain_eye" (1) and
 * at most "chain_max_p_eye" (16640) rows -- that is not being captured runs as ONE persistent launch -- "chain_grid"
 * workgroups (0: one per CU), every wait bounded by "chain_timeout_ms": 1, the default, auto: unless a
 * factorisation this library enqueued on another stream of the device is still in flight (each
 * persistent launch claims every CU); 2 always; 0 never), with "chain_group" panels per deferred tile update
 * (0, the default: 4 below 80 diagonal blocks, 8 from there), "chain_uq" (1: the next diagonal block's update by each panel as 32-column quarter tasks; 0: one task
 * per 32-row slice; 2: slice r's panel solve and the next diagonal block's quarter updates as one task) and, for
 * batches, "chain_max_batch" members (8) while batch x p <= "chain_batch_max_rows" (17500).  Several persistent
 * launches may run side by side on different streams, each with "chain_grid" workgroups (a CU share): no launch
 * waits for another's workgroups (bench.py's C2 schedule: 8 in flight, 64 workgroups each on 256 CUs).
 * With "chain" 1 (auto) factorisations of fewer than "chain_min_p" (768) rows -- identity-augmented ones:
 * "chain_min_p_eye" (3072) -- keep the launch path (a handful of panels: its few launches are faster).
 * Identity-augmented plans take "chain_group_eye" (8) panels per deferred tile update (0: chain_group's
 * rule) and defer the corner's tile updates (-K^-1, read by no later task) in groups of
 * "chain_group_corner" (16) panels, except the last "chain_corner_tail" (8) panels, which keep "chain_group"; a
 * deferred (grouped) update covers only block columns at least "chain_group_la" (2) columns past the group's last
 * panel.  Every knob the planner reads is part of its plan cache key.
 * "asm_f32_fast" (1: the f32 K build of a single SE / MAT32 / MAT52 node writes its interior tiles with f64
 * distances and the f32 hardware sqrt / exp -- a few f32 ulps from the f64 build; 0: every tile through the
 * general f64 evaluation, A/B; "asm_f32_chunk" (4) consecutive lower tiles per workgroup).
 * "chain_xcd" (0; 1: the persistent launch's diagonal-chain tasks -- D, the next diagonal block's panel solves and
 * quarter updates -- as a second task list claimed first by up to "chain_xcd_seats" (16) workgroups of XCD 0, the
 * rest by everyone else, each workgroup falling back to the other list once its own is exhausted; measured no
 * faster).
 * "chain_f32" (1: f32 factorisations without identity rows take the persistent launch under the same rules --
 * chain_kernel<float>: f32 MFMA panel solves and tile updates, the diagonal blocks as the launch path's; bitwise
 * the f32 launch path's results; one slice-update task per slice whatever "chain_uq"; 0: the launch path).
 * Planner knobs of the persistent launch (all part of the plan cache key, all bitwise the launch path's results):
 * "chain_group_near" (2: the tile updates of the columns too near the diagonal for the deferred group go in
 * sub-groups of this many panels, for columns at least "chain_near_la" (1) past the sub-group's last panel; 1: one
 * panel at a time), "chain_u128" (2 auto, 1, 0: below the next diagonal block the next panel's column is updated by
 * one 128 x 128 tile task per block row instead of four 32-row slice tasks; auto: except below 48 diagonal blocks on
 * a grid of more than 2 workgroups per block), "chain_s128" (2 auto, 1, 0: the panel solves below the next diagonal
 * block as one task per block row; auto: on grids of at most 2 workgroups per diagonal block -- the CU-share launches
 * side by side -- and identity-augmented plans of at least 64 diagonal blocks).
 * "asm_feat" (1: the K build of a two-leaf SE + periodic tree at D = 4 or 8 computes the per-point features in a
 * pre-pass and runs its interior tiles on the f64 MFMA fast-tile kernel; 0: every tile stages its points itself
 * -- the same bits, slower; A/B).
 * A persistent launch whose wait timed out
 * sets info = -1 -- an infrastructure failure, not a non-positive pivot: the factorisation is
 * incomplete and W undefined; re-assemble and re-run it with "chain" 0 (the Python layer does,
 * engine.AugmentedFactorization).  "chain_force_timeout" (testing) makes the next `value` persistent
 * launches report a timeout at their first wait.
 * Stores the value and returns the previous one through *old (may be NULL); 0 or -1 (unknown
 * key).  Defaults come from the environment (GPK_LOOKAHEAD, GPK_RESERVE_CUS, ...). */
int gpk_tune(const char* key, int64_t value, int64_t* old);

/* Per-host-thread override of a gpk_tune knob (no reference counterpart): set = 1 pins `value` for
 * the calls of the calling thread only, set = 0 removes the thread's override (the global knob applies
 * again).  *old_value / *old_set (may be NULL) return the override in effect before the call (old_set
 * 0: none, *old_value is then the global value).  0 or -1 (unknown key). */
int gpk_tune_thread(const char* key, int64_t value, int32_t set, int64_t* old_value, int32_t* old_set);

/* Counters of the persistent factorisation: out[0] persistent launches enqueued (all threads),
 * out[1] factorisations that took the launch path because another stream was busy (chain = 1),
 * out[2] 1 if the calling thread's last factorisation was a persistent launch (its info must then be
 * checked for -1, see gpk_tune "chain"), out[3] forced timeouts still pending, out[4] (n >= 5 only: a
 * synchronous device read) persistent launches on the current device whose waits timed out so far (each
 * such launch aborted and set info = -1 on its unfinished members; forced timeouts included).
 * Writes min(n, 5). */
int gpk_chain_stats(int64_t* out, int32_t n);

/* The task list of the persistent single-member factorisation (gpk_tune "chain"; no reference
 * counterpart): the order in which the workgroups of its one launch claim the tasks, for an augmented
 * matrix with n_pad training rows, the y row at y_row and `grid` workgroups.  Four int32 per task:
 * type (0: factor diagonal block k; 1: solve 32-row slice r below block k; 2: slice r of block column
 * j = k + 1 -= panel k; 3: 128 x 128 tile (r, j) -= panel k), k, r, j.  Host only (no device call):
 * tasks_out may be NULL to query *ntasks; cap = its capacity in tasks. */
int gpk_chain_plan(int64_t n_pad, int64_t y_row, int32_t grid, int32_t* tasks_out, int64_t cap, int64_t* ntasks);
/* gpk_chain_plan with flags: GPK_AUG_EXTRA_IDENTITY plans the identity-augmented factorisation (gpk_potrf_aug_ex,
 * gpk_nlml_grad; y_row = n_pad + n): tasks that would only move the structurally zero parts of E L^-T are left
 * out, and a task word with bit 6 set updates cells no earlier task updated (its counter wait is for 0).  The
 * type word: type (bits 0..1) | (g - 1) << 2 (bits 2..5; type 3: an update over the g panels k .. k + g - 1;
 * type 2 with g > 1: the 32 x 32 quarter g - 2 of slice r in diagonal block j) | bit 6 | bit 7 (an SQ task of
 * "chain_uq" 2: the slice's panel solve, then the next diagonal block's quarter updates) | member << 8.
 * GPK_CHAIN_PLAN_F32: the plan of an f32 factorisation (chain_kernel<float>: one slice-update task per slice, the
 * f32 deferred-update depth). */
#define GPK_CHAIN_PLAN_F32 256
int gpk_chain_plan_ex(int64_t n_pad, int64_t y_row, int32_t grid, int32_t flags, int32_t* tasks_out, int64_t cap,
                      int64_t* ntasks);

#ifdef __cplusplus
}
#endif
#endif /* GPK_H */
