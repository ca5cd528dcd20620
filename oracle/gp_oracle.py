"""CPU oracle: a numpy/SciPy fp64 restatement of the reference's exact-GP likelihood path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the checker or
as the timed CPU baseline.  The product package (``gaussianprocessfundamentals_amd``)
never imports it and has no CPU fallback.

Parity status: **parity unpinned by the reference itself.**  The reference
(Bernsai/GaussianProcessFundamentals, ``gpbasics`` 2.0.0) ships no tests, fixtures or
golden vectors, and it cannot be imported here (TensorFlow is absent: an ordinary
``ModuleNotFoundError``, not a permission denial).  This restatement is therefore pinned
by closed-form known answers (``known_answers()`` below, exercised in
``tests/test_oracle.py``) and it generates the committed golden vectors under
``tests/golden/`` (script: ``tests/golden/make_golden.py``).

Every function follows the reference op-for-op; citations are
``path:line`` relative to ``/root/reference/main/gpbasics``.  TensorFlow's own rounding
(Eigen LLT blocking, reduction order) cannot be reproduced and is covered by tolerance.

Kernel trees are given as nested tuples, independent of the product package:
  ("SE",    {"ard": False})      SquaredExponentialKernel   hyp [l, (sg)]
  ("PER",   {})                  PeriodicKernel              hyp [l, p, (sg)]
  ("MAT32", {"ard": False})      MaternKernel3_2             hyp [l, (sg)]
  ("MAT52", {"ard": False})      MaternKernel5_2             hyp [l, (sg)]
  ("ADD", [child, child, ...])   AdditionOperator
  ("MUL", [child, child, ...])   MultiplicationOperator
``standard=True`` (MAT/PER) selects the build's well-posed multi-dimensional form: Euclidean
distance for the Matern kernels, a per-dimension sum of sin^2 for PER.  Both equal the
reference form when D == 1; for D > 1 the reference's L1 forms are not positive definite
(e.g. min eigenvalue -0.94 for the C3 inputs, -29 for C5's PER), so its Cholesky fails there.
``ard=True`` is the build's ARD extension (the reference has only scalar length scales,
SURVEY Q4): the length-scale hyperparameter is a vector of D values and the kernel equals
the reference kernel with l = 1 evaluated on inputs divided elementwise by that vector.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np
import scipy.linalg as sla

LOG_2PI = math.log(2.0 * math.pi)


# ---------------------------------------------------------------- distances (A/Distances.py)
def euclidian_distance(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Expanded-norm L2 distance, unclamped: A/Distances.py:4-7.

    sqrt(rowsum(a*a) - 2 a b^T + rowsum(b*b)^T); a negative argument gives NaN exactly as in
    the reference."""
    na = np.sum(a * a, axis=-1, keepdims=True)
    nb = np.sum(b * b, axis=-1, keepdims=True)
    with np.errstate(invalid="ignore"):
        return np.sqrt((na - 2.0 * (a @ np.swapaxes(b, -1, -2))) + np.swapaxes(nb, -1, -2))


def manhattan_distance(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """L1 distance via broadcast: A/Distances.py:10-12."""
    return np.sum(np.abs(a[..., :, None, :] - b[..., None, :, :]), axis=-1)


def squared_l2_direct(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Build's default SE distance: sum_d (a_d - b_d)^2 (identical to the reference where the
    reference is finite, up to rounding; never NaN).  Not in the reference."""
    diff = a[..., :, None, :] - b[..., None, :, :]
    return np.sum(diff * diff, axis=-1)


# ---------------------------------------------------------------- base kernels (K/BaseKernels.py)
def n_hyp(tree, scaled: bool, dim: int) -> int:
    """Hyperparameter count in DFS order: K/Operators.py:28-32 and the per-kernel
    get_number_of_hyper_parameter (K/BaseKernels.py:308-314, :475-481, :734-740, :894-900)."""
    op, arg = tree
    if op in ("ADD", "MUL"):
        return sum(n_hyp(c, scaled, dim) for c in arg)
    base = 2 if op == "PER" else 1
    return base + (1 if scaled else 0)


def _scale_inputs(x, ls):
    return x / np.asarray(ls, dtype=np.float64)


def eval_base(op: str, opts: dict, hyp: Sequence, x: np.ndarray, x_: np.ndarray,
              scaled: bool, se_expanded: bool) -> np.ndarray:
    ard = bool(opts.get("ard", False))
    if op == "SE":
        # K/BaseKernels.py:277-294
        if ard:
            x, x_ = _scale_inputs(x, hyp[0]), _scale_inputs(x_, hyp[0])
            l = 1.0
        else:
            l = float(hyp[0])
        if se_expanded:
            dist = euclidian_distance(x, x_)
            sq = dist * dist                                   # tf.square(dist)
        else:
            sq = squared_l2_direct(x, x_)
        r = np.exp(-0.5 * (sq / (l * l)))
        if scaled:
            r = float(hyp[1]) * r                              # :289-290
        return r
    if op in ("MAT52", "MAT32"):
        # K/BaseKernels.py:859-880 (MAT52), :702-720 (MAT32); L1 distance
        if ard:
            x, x_ = _scale_inputs(x, hyp[0]), _scale_inputs(x_, hyp[0])
            l = 1.0
        else:
            l = abs(float(hyp[0]))
        if opts.get("standard", False):
            # build option: Euclidean distance (the textbook Matern; PD in any D).  Equal to the
            # reference's L1 form when D == 1.
            dist = np.sqrt(squared_l2_direct(x, x_))
        else:
            dist = manhattan_distance(x, x_)
        if op == "MAT52":
            frac = (math.sqrt(5.0) * dist) / l
            third = (5.0 * (dist * dist)) / (3.0 * (l * l))
            r = ((1.0 + frac) + third) * np.exp(-frac)
        else:
            frac = (math.sqrt(3.0) * dist) / l
            r = (1.0 + frac) * np.exp(-frac)
        if scaled:
            r = float(hyp[1]) * r
        return r
    if op == "PER":
        # K/BaseKernels.py:440-457; L1 distance, hyp [l, p, (sg)]
        if ard:
            raise ValueError("PER has no ARD form")
        l, p = float(hyp[0]), float(hyp[1])
        if opts.get("standard", False):
            # build option: per-dimension form exp(-2 sum_d sin^2(pi |x_d - y_d| / p) / l^2),
            # a product of 1-D periodic kernels (PD in any D); equal to the reference when D == 1.
            dd = np.abs(x[..., :, None, :] - x_[..., None, :, :])
            sd = np.sin(math.pi * (dd / p))
            sine = np.sum(sd * sd, axis=-1)
        else:
            dist = manhattan_distance(x, x_)
            sine = np.sin(math.pi * (dist / p))
            sine = sine * sine
        r = np.exp((-2.0 * sine) / (l * l))
        if scaled:
            r = float(hyp[2]) * r
        return r
    raise ValueError("unsupported kernel op %r" % op)


def kernel_matrix(tree, hyp: List, x: np.ndarray, x_: np.ndarray, scaled: bool = False,
                  se_expanded: bool = False, row_chunk: int = 1024) -> np.ndarray:
    """Kernel.get_tf_tensor (K/Kernel.py:51-52) for a tree; ADD/MUL fold left over children
    with DFS hyperparameter slicing exactly as K/Operators.py:207-225 / :306-326.
    Rows are evaluated in chunks (elementwise identical; bounds the [rows, m, D] temporaries)."""
    if x.ndim == 2 and x.shape[0] > row_chunk:
        return np.concatenate([_kernel_matrix(tree, hyp, x[i:i + row_chunk], x_, scaled, se_expanded)
                               for i in range(0, x.shape[0], row_chunk)], axis=0)
    return _kernel_matrix(tree, hyp, x, x_, scaled, se_expanded)


def _kernel_matrix(tree, hyp, x, x_, scaled, se_expanded):
    op, arg = tree
    if op in ("ADD", "MUL"):
        idx = 0
        result = None
        dim = x.shape[-1]
        for child in arg:
            k = n_hyp(child, scaled, dim)
            m = _kernel_matrix(child, hyp[idx:idx + k], x, x_, scaled, se_expanded)
            idx += k
            if result is None:
                result = m
            else:
                result = result + m if op == "ADD" else result * m
        return result
    return eval_base(op, arg, hyp, x, x_, scaled, se_expanded)


# ---------------------------------------------------------------- covariance + likelihood
def k_noised(tree, hyp, noise, x, scaled=False, se_expanded=False):
    """HolisticCovarianceMatrix.get_K_noised: S/CovarianceMatrix.py:197-206."""
    K = kernel_matrix(tree, hyp, x, x, scaled, se_expanded)
    n = x.shape[-2]
    return K + noise * np.eye(n)


def cholesky_lower(A):
    """tf.linalg.cholesky (S/CovarianceMatrix.py:250): lower factor; raises
    np.linalg.LinAlgError when not positive definite (TF raises InvalidArgumentError)."""
    return sla.cholesky(A, lower=True, check_finite=False)


def l_alpha(L, y):
    """get_L_alpha: alpha = L^T \\ (L \\ y)  (S/CovarianceMatrix.py:256-265)."""
    z = sla.solve_triangular(L, y, lower=True, check_finite=False)
    return sla.solve_triangular(L.T, z, lower=False, check_finite=False)


def nlml_components(tree, hyp, noise, x, y, scaled=False, se_expanded=False):
    """One LogLikelihood.get_metric evaluation, CHOLESKY_BASED strategy
    (M/LogLikelihood.py:30-65, M/Metrics.py:138-139 and :152-154).

    Returns dict(nlml, fit, logdet, n) with nlml = -LML (minimise convention,
    M/Metrics.py:27), fit = y^T alpha, logdet = 2 sum log diag L."""
    y = np.asarray(y, dtype=np.float64).reshape(-1, 1)
    A = k_noised(tree, hyp, noise, x, scaled, se_expanded)
    L = cholesky_lower(A)
    alpha = l_alpha(L, y)
    fit = float((y.T @ alpha)[0, 0])                               # :39
    logdet = float(2.0 * np.sum(np.log(np.diag(L))))               # M/Metrics.py:153-154
    n = x.shape[-2]
    ll = (-0.5 * fit + -0.5 * logdet) + (-0.5 * (n * LOG_2PI))     # :41-49
    return {"nlml": -ll, "fit": fit, "logdet": logdet, "n": n, "L": L, "alpha": alpha}


def nlml(tree, hyp, noise, x, y, scaled=False, se_expanded=False) -> float:
    return nlml_components(tree, hyp, noise, x, y, scaled, se_expanded)["nlml"]


def batch_nlml(tree, hyp, noise, xb, yb, scaled=False, se_expanded=False) -> float:
    """BatchDataInput mode: the data-fit term is averaged over the
    batch by p_batch_metric_aggregator=reduce_mean (M/LogLikelihood.py:62-63) while the
    Cholesky log-determinant is a reduce_sum with no axis (M/Metrics.py:153-154), i.e.
    summed over the whole batch before being broadcast into every member."""
    fits, logdets = [], []
    for b in range(xb.shape[0]):
        c = nlml_components(tree, hyp, noise, xb[b], yb[b], scaled, se_expanded)
        fits.append(c["fit"])
        logdets.append(c["logdet"])
    n = xb.shape[-2]
    logdet_total = float(np.sum(logdets))
    lls = [(-0.5 * f + -0.5 * logdet_total) + (-0.5 * (n * LOG_2PI)) for f in fits]
    return -float(np.mean(lls))


def posterior(tree, hyp, noise, x, y, xs, scaled=False, se_expanded=False):
    """get_posterior_mu / get_posterior_var (S/Auxiliary.py:57-93) with the explicit
    inverse of L used by get_L_inv_K (S/CovarianceMatrix.py:267-275); K_ss carries no noise
    (S/CovarianceMatrix.py:218-225).  Returns (mu [M], full covariance [M, M])."""
    y = np.asarray(y, dtype=np.float64).reshape(-1, 1)
    A = k_noised(tree, hyp, noise, x, scaled, se_expanded)
    L = cholesky_lower(A)
    alpha = l_alpha(L, y)
    Ks = kernel_matrix(tree, hyp, x, xs, scaled, se_expanded)             # [N, M]
    mu = (Ks.T @ alpha).reshape(-1)                                         # :75-77
    Linv = np.linalg.inv(L)                                                 # :270
    v = Linv @ Ks                                                           # :60-62
    Kss = kernel_matrix(tree, hyp, xs, xs, scaled, se_expanded)
    var = Kss - v.T @ v                                                     # :86-88
    return mu, var


def n_prior_functions(tree, hyp, noise, xs, y_train, z, scaled=False, se_expanded=False):
    """get_n_prior_functions (S/GaussianProcess.py:87-95) for a given standard-normal draw z
    [M, n]: L_K_ss (z std(y) + mean(y)), L_K_ss = chol(K_ss + noise I) (S/CovarianceMatrix.py:238-245),
    mean / population std of the training targets (np.mean / np.std, :90-92)."""
    y = np.asarray(y_train, dtype=np.float64).reshape(-1)
    L = cholesky_lower(k_noised(tree, hyp, noise, xs, scaled, se_expanded))
    return L @ (np.asarray(z, dtype=np.float64) * np.std(y) + np.mean(y))


def n_posterior_functions(tree, hyp, noise, x, y, xs, z, jitter, scaled=False, se_expanded=False):
    """get_n_posterior_functions (S/GaussianProcess.py:97-110) for a given standard-normal draw
    z [M, n]: mu + chol(Sigma + jitter I) z, (mu, Sigma) from :func:`posterior`."""
    mu, var = posterior(tree, hyp, noise, x, y, xs, scaled, se_expanded)
    L = cholesky_lower(var + jitter * np.eye(var.shape[0]))
    return mu.reshape(-1, 1) + L @ np.asarray(z, dtype=np.float64)


# ---------------------------------------------------------------- segmented models
def cp_indicator(x, cp, mode: str = "INDICATOR"):
    """Change-point masks of ChangePointOperator (K/Operators.py:379-408) on 1-D inputs:
    INDICATOR = [x < cp]; SIGMOID = 0.5 (1 + tanh((cp - x) / 0.0025)); APPROX_INDICATOR =
    1 / (1 + exp(-100 (x - cp)))."""
    x = np.asarray(x, dtype=np.float64).reshape(-1)
    if mode == "SIGMOID":
        return 0.5 * (1 + np.tanh((cp - x) / 0.0025))
    if mode == "APPROX_INDICATOR":
        return 1.0 / (1.0 + np.exp(-100.0 * (x - cp)))
    return (x < cp).astype(np.float64)


def change_point_matrix(trees, hyps, cps, x, x_, mode: str = "INDICATOR", scaled=False):
    """ChangePointOperator.get_tf_tensor (K/Operators.py:410-476): child i's matrix times
    previous_sigmoid (the complement mask of cp_{i-1}) times the outer indicator of cp_i, summed."""
    prev = np.ones((x.shape[0], x_.shape[0]))
    total = np.zeros((x.shape[0], x_.shape[0]))
    for i, (t, h) in enumerate(zip(trees, hyps)):
        K = kernel_matrix(t, h, x, x_, scaled) * prev                                  # :414-417
        if i < len(cps):
            xi, xsi = cp_indicator(x, cps[i], mode), cp_indicator(x_, cps[i], mode)
            K = K * np.outer(xi, xsi)                                                   # :431-436
            prev = np.outer(1.0 - xi, 1.0 - xsi)                                        # :433-434
        total = total + K                                                               # :476
    return total


def blockwise_nlml(segments, noise, scaled=False) -> float:
    """BlockwiseLogLikelihood.get_metric (M/LogLikelihood.py:76-104): the sum of the segments'
    -LML; segments = [(tree, hyp, x_i, y_i)], an empty segment contributes 0."""
    return float(sum(nlml(t, h, noise, x, y, scaled) if x.shape[0] > 0 else 0.0 for t, h, x, y in segments))


def bic(nl: float, n_hyp: int, n_train: int) -> float:
    """BIC.get_metric (M/BayesianInformationCriterion.py:27-38): -2 LL + |M| log n with LL = -nl."""
    return -2.0 * (-nl) + n_hyp * math.log(n_train)


def mse(tree, hyp, noise, x, y, xs, ys, scaled=False) -> float:
    """MeanSquaredError.get_metric (M/MeanSquaredError.py:26-42): mean((K_s^T alpha - y_test)^2)."""
    mu, _ = posterior(tree, hyp, noise, x, y, xs, scaled)
    return float(np.mean((mu.reshape(-1, 1) - np.asarray(ys).reshape(-1, 1)) ** 2))


def cv_folds(n: int, test_ratio: float = 0.2):
    """Fold indices of get_data_inputs (M/CrossValidation.py:16-44), drawn from numpy's GLOBAL
    generator exactly as the reference draws them: [(train_idx, test_idx)]."""
    n_test = int(round(n * test_ratio))
    epochs = int(np.floor(1 / test_ratio))
    idx = np.linspace(start=0, num=n, stop=n, endpoint=False, dtype=int)
    np.random.shuffle(idx)
    out, at = [], 0
    for _ in range(epochs):
        stop = n_test + at
        out.append((np.array(sorted(np.concatenate([idx[:at], idx[stop:]])), dtype=int),
                    np.array(sorted(idx[at:stop]), dtype=int)))
        at += n_test
    return out


def linear_cg(A, b, x):
    """linear_cg (A/LinearConjugateGradients.py:9-41): CG from x with the reference's stopping rule
    |max(r_k)| > 1e-2 (absolute value of the maximum) and its n-iteration guard."""
    n = A.shape[0]
    b = np.asarray(b, dtype=np.float64).reshape(-1, 1)
    x = np.asarray(x, dtype=np.float64).reshape(-1, 1).copy()
    r = A @ x - b
    p = -r
    k = 0
    first = True
    while first or abs(np.max(r)) > 1e-2:
        Ap = A @ p
        rr = float((r.T @ r)[0, 0])
        a = rr / float((p.T @ Ap)[0, 0])
        nx = x + a * p
        if np.any(np.isnan(nx)):
            return x
        x = nx
        r2 = r + a * Ap
        beta = float((r2.T @ r2)[0, 0]) / rr
        p = -r2 + beta * p
        r = r2
        k += 1
        first = False
        if k % (n / 4) == 0 and k > n:
            break
    return x


def nlml_with_alpha(alpha, y, logdet, n) -> float:
    """-LML from a given alpha and log-determinant (M/LogLikelihood.py:36-49)."""
    fit = float(np.asarray(y).reshape(-1) @ np.asarray(alpha).reshape(-1))
    return -((-0.5 * fit + -0.5 * logdet) + (-0.5 * (n * LOG_2PI)))


# ---------------------------------------------------------------- staged, threaded CPU baseline
def kernel_matrix_threaded(tree, hyp, x, x_, threads: int = 1, scaled: bool = False,
                           se_expanded: bool = False, row_chunk: int = 256) -> np.ndarray:
    """kernel_matrix with its row chunks evaluated on `threads` host threads (numpy's elementwise
    loops release the GIL), the way TF's intra-op pool (GP:38-39) spreads the reference's K build.
    Every element is computed by the same numpy expression as kernel_matrix: identical values."""
    if threads <= 1 or x.ndim != 2 or x.shape[0] <= row_chunk:
        return kernel_matrix(tree, hyp, x, x_, scaled, se_expanded)
    from concurrent.futures import ThreadPoolExecutor
    out = np.empty((x.shape[0], x_.shape[0]), dtype=np.float64)

    def part(i):
        out[i:i + row_chunk] = _kernel_matrix(tree, hyp, x[i:i + row_chunk], x_, scaled, se_expanded)

    with ThreadPoolExecutor(max_workers=threads) as ex:
        list(ex.map(part, range(0, x.shape[0], row_chunk)))
    return out


def nlml_stages(tree, hyp, noise, x, y, threads: int = 1, scaled: bool = False, lapack: str = "mkl"):
    """One CHOLESKY_BASED -LML evaluation (M/LogLikelihood.py:30-65) timed stage by stage on
    `threads` host threads: K build (+ noise on the diagonal, S/CovarianceMatrix.py:187-206),
    dpotrf (:250), the two triangular solves (:256-265) and the read-out (M/Metrics.py:152-154).
    lapack "mkl": torch's CPU LAPACK (MKL, OpenMP pool = `threads`); "openblas": scipy's.
    The CPU baseline of bench.py (test infrastructure; never the measured GPU path)."""
    import time
    from threadpoolctl import threadpool_limits
    y = np.asarray(y, dtype=np.float64).reshape(-1, 1)
    n = x.shape[-2]
    t = {}
    with threadpool_limits(limits=threads):
        t0 = time.perf_counter()
        A = kernel_matrix_threaded(tree, hyp, x, x, threads, scaled)
        A[np.diag_indices(n)] += noise
        t["kbuild"] = time.perf_counter() - t0
        if lapack == "mkl":
            import torch
            old = torch.get_num_threads()
            torch.set_num_threads(threads)
            try:
                t0 = time.perf_counter()
                At = torch.from_numpy(A)
                Lt = torch.linalg.cholesky(At)
                t["potrf"] = time.perf_counter() - t0
                t0 = time.perf_counter()
                yt = torch.from_numpy(y)
                z = torch.linalg.solve_triangular(Lt, yt, upper=False)
                alpha = torch.linalg.solve_triangular(Lt.mT, z, upper=True).numpy()
                t["trsv"] = time.perf_counter() - t0
                t0 = time.perf_counter()
                logdet = float(2.0 * torch.log(torch.diagonal(Lt)).sum())
            finally:
                torch.set_num_threads(old)
        else:
            t0 = time.perf_counter()
            L = cholesky_lower(A)
            t["potrf"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            alpha = l_alpha(L, y)
            t["trsv"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            logdet = float(2.0 * np.sum(np.log(np.diag(L))))
        fit = float((y.T @ alpha)[0, 0])
        ll = (-0.5 * fit + -0.5 * logdet) + (-0.5 * (n * LOG_2PI))
        t["readout"] = time.perf_counter() - t0
    t["total"] = sum(t.values())
    return -ll, t


# ---------------------------------------------------------------- synthetic configs
def make_inputs(cfg: str, n: int = None, seed: int = None) -> Tuple[np.ndarray, np.ndarray]:
    """Synthetic data generators of SURVEY §8(d) (numpy default_rng(seed))."""
    if cfg in ("C1", "C2", "C4", "metric"):
        d = 1
        seed = {"C1": 0, "C2": 1, "C4": 3, "metric": 5}[cfg] if seed is None else seed
        n = {"C1": 256, "C2": 4096, "C4": 4096, "metric": 8192}[cfg] if n is None else n
        rng = np.random.default_rng(seed)
        x = np.sort(rng.uniform(0.0, 1.0, n)).reshape(n, d)
        y = np.sin(4.0 * math.pi * x[:, 0]) + 0.1 * rng.standard_normal(n)
        return x, y
    if cfg == "C3":
        n = 8192 if n is None else n
        rng = np.random.default_rng(2 if seed is None else seed)
        x = rng.uniform(0.0, 1.0, (n, 4))
        y = np.sum(np.sin(2.0 * math.pi * x), axis=1) + 0.1 * rng.standard_normal(n)
        return x, y
    if cfg == "C5":
        n = 16384 if n is None else n
        rng = np.random.default_rng(4 if seed is None else seed)
        x = rng.uniform(0.0, 1.0, (n, 8))
        y = np.sum(np.sin(2.0 * math.pi * x), axis=1) + 0.1 * rng.standard_normal(n)
        return x, y
    raise ValueError(cfg)


def known_answers() -> List[Tuple[str, float, float]]:
    """Closed-form checks.  Returns (name, oracle value, exact value)."""
    out = []
    se = ("SE", {"ard": False})
    # N=1: NLL = y^2/(2(1+s2)) + log(1+s2)/2 + log(2pi)/2
    for y0, s2 in ((0.7, 0.01), (-1.3, 0.5)):
        got = nlml(se, [0.3], s2, np.array([[0.2]]), np.array([y0]))
        exp = 0.5 * y0 * y0 / (1 + s2) + 0.5 * math.log(1 + s2) + 0.5 * LOG_2PI
        out.append(("N1_y%.1f" % y0, got, exp))
    # N=2: K = [[1+s2, k],[k, 1+s2]], det = (1+s2)^2 - k^2, inverse closed form
    x = np.array([[0.1], [0.35]])
    yv = np.array([0.4, -0.9])
    l, s2 = 0.2, 0.05
    kk = math.exp(-0.5 * (0.25 ** 2) / (l * l))
    a = 1 + s2
    det = a * a - kk * kk
    quad = (a * yv[0] ** 2 - 2 * kk * yv[0] * yv[1] + a * yv[1] ** 2) / det
    exp = 0.5 * quad + 0.5 * math.log(det) + LOG_2PI
    out.append(("N2", nlml(se, [l], s2, x, yv), exp))
    # far separated points: K ~ I
    xf = np.arange(8, dtype=np.float64).reshape(-1, 1) * 100.0
    yf = np.linspace(-1, 1, 8)
    s2 = 0.1
    exp = 0.5 * float(np.sum(yf ** 2)) / (1 + s2) + 0.5 * 8 * math.log(1 + s2) + 0.5 * 8 * LOG_2PI
    out.append(("far", nlml(se, [0.5], s2, xf, yf), exp))
    # k(x, x) = 1 for SE / MAT / PER
    xp = np.array([[0.3, -1.2]])
    for tree, hyp in ((se, [0.7]), (("MAT52", {}), [0.7]), (("MAT32", {}), [0.7]), (("PER", {}), [0.7, 0.4])):
        out.append(("diag_" + tree[0], float(kernel_matrix(tree, hyp, xp, xp)[0, 0]), 1.0))
    # PER at d = p gives 1
    out.append(("per_d_eq_p", float(kernel_matrix(("PER", {}), [0.9, 0.5], np.array([[0.0]]), np.array([[0.5]]))[0, 0]), 1.0))
    # MAT52 at d = l/sqrt(5): (1 + 1 + 1/3) e^-1
    l = 0.8
    got = float(kernel_matrix(("MAT52", {}), [l], np.array([[0.0]]), np.array([[l / math.sqrt(5.0)]]))[0, 0])
    out.append(("mat52_unit", got, (2.0 + 1.0 / 3.0) * math.exp(-1.0)))
    # ARD identity: k_ARD(x, y; ls) == k_ref(x/ls, y/ls; l=1)
    rng = np.random.default_rng(7)
    xa, xb = rng.uniform(size=(5, 3)), rng.uniform(size=(4, 3))
    ls = [0.3, 0.6, 1.1]
    for name in ("SE", "MAT52", "MAT32"):
        k1 = kernel_matrix((name, {"ard": True}), [ls], xa, xb)
        k2 = kernel_matrix((name, {"ard": False}), [1.0], xa / ls, xb / ls)
        out.append(("ard_" + name, float(np.max(np.abs(k1 - k2))), 0.0))
    return out


# ----------------------------------------------------------------------------- approximations (§8f.4)
def tf_pinv(A: np.ndarray) -> np.ndarray:
    """tf.linalg.pinv with its default rcond = 10 max(rows, cols) eps: singular values s > rcond
    max(s) inverted, the rest dropped (Statistics/Nystroem_K.py:53 calls it on K_mm)."""
    rcond = 10.0 * max(A.shape) * np.finfo(np.float64).eps
    return np.linalg.pinv(A, rcond=rcond)


def nystroem_k_approx(tree, hyp, x, z, scaled=False, se_expanded=False):
    """K_hat = (K_nm pinv(K_mm)) K_nm^T (Statistics/Nystroem_K.py:36-64); z are the inducing
    inputs the reference passes as ``indices``."""
    knm = kernel_matrix(tree, hyp, x, z, scaled, se_expanded)
    kmm = kernel_matrix(tree, hyp, z, z, scaled, se_expanded)
    return (knm @ tf_pinv(kmm)) @ knm.T, knm, kmm


def nystroem_det(tree, hyp, noise, x, z, scaled=False, se_expanded=False) -> float:
    """get_K_approx_det (Statistics/Nystroem_K.py:92-108): (n - m) log(noise) +
    slogdet(noise I_m + K_nm^T (K_nm pinv(K_mm)))[1]."""
    _, knm, kmm = nystroem_k_approx(tree, hyp, x, z, scaled, se_expanded)
    n, m = knm.shape
    phi_t = knm @ tf_pinv(kmm)
    to_det = np.eye(m) * noise + knm.T @ phi_t
    return float((n - m) * math.log(noise) + np.linalg.slogdet(to_det)[1])


def nystroem_k_approx_inv(tree, hyp, noise, x, z, scaled=False, se_expanded=False) -> np.ndarray:
    """get_K_approx_inv (Statistics/Nystroem_K.py:73-90), the reference's Woodbury form op for op:
    (1 / noise) (I - K_nm (pinv(noise I_m + pinv(K_mm) K_nm^T K_nm) (pinv(K_mm) K_nm^T)))."""
    _, knm, kmm = nystroem_k_approx(tree, hyp, x, z, scaled, se_expanded)
    n, m = knm.shape
    dot_aux = tf_pinv(kmm) @ knm.T
    inner = tf_pinv(np.eye(m) * noise + dot_aux @ knm)
    return (1.0 / noise) * (np.eye(n) - knm @ (inner @ dot_aux))


def nystroem_nlml(tree, hyp, noise, x, y, z, handling: str = "CHOLESKY_BASED", lower_bound: bool = False,
                  jitter: float = 1e-8, scaled=False, se_expanded=False) -> float:
    """LogLikelihood.get_metric with BASIC_NYSTROEM / SKC_LOWER_BOUND (Metrics/LogLikelihood.py:30-65,
    Metrics/Metrics.py:77-150): the covariance matrix is K_hat + noise I, the log-determinant the
    Nystroem one; CHOLESKY_BASED keeps the EXACT alpha (get_alpha_cholesky reads the holistic
    covariance matrix), the other handlings solve with K_hat + noise I.  SKC_LOWER_BOUND subtracts
    trace(K_hat + noise I - K) / (2 p_cov_matrix_jitter) (:51-60)."""
    y = np.asarray(y, np.float64).reshape(-1, 1)
    n = y.shape[0]
    khat, _, _ = nystroem_k_approx(tree, hyp, x, z, scaled, se_expanded)
    khat_n = khat + np.eye(n) * noise
    if handling == "CHOLESKY_BASED":
        L = cholesky_lower(k_noised(tree, hyp, noise, x, scaled, se_expanded))
        alpha = l_alpha(L, y)
    elif handling == "LINEAR_CONJUGATE_GRADIENT":
        alpha = linear_cg(khat_n, y, np.zeros_like(y))
    elif handling == "PSEUDO_INVERSE":
        alpha = tf_pinv(khat_n) @ y
    else:
        alpha = np.linalg.inv(khat_n) @ y
    logdet = nystroem_det(tree, hyp, noise, x, z, scaled, se_expanded)
    ll = -0.5 * float(y.T @ alpha) - 0.5 * logdet - 0.5 * n * math.log(2 * math.pi)
    if lower_bound:
        k = kernel_matrix(tree, hyp, x, x, scaled, se_expanded)
        ll -= (1.0 / (2.0 * jitter)) * float(np.trace(khat_n - k))
    return -ll


def vsgd_step(alpha: np.ndarray, grad: np.ndarray, batch_size: float = 10.0, total: float = 10.0,
              decay: float = 0.95, max_lr: float = 1e-6) -> np.ndarray:
    """One tfp.optimizer.VariationalSGD(10, 10) step from zero moments in burn-in (iteration 0 <
    burnin = 25, so the learning-rate cap is burnin_max_learning_rate = 1e-6): first moment
    m = (1 - decay) g, second moment v = (1 - decay) (g - m)^2, per-coordinate learning rate
    min(2 batch_size / (total v), cap) (Mandt et al. 2017's preconditioned constant SGD), then
    alpha - lr g.  Restated from the published algorithm (TFP is absent here): parity unpinned."""
    m = (1.0 - decay) * grad
    v = (1.0 - decay) * (grad - m) ** 2
    with np.errstate(divide="ignore"):
        lr = np.where(v > 0, 2.0 * batch_size / (total * v), np.inf)
    lr = np.clip(lr, 0.0, max_lr)
    return alpha - lr * grad


def skc_upper_bound(tree, hyp, noise, x, y, z, scaled=False, se_expanded=False) -> float:
    """LogLikelihoodUpperBound.get_metric (Metrics/SkcLogLikelihood.py:26-69): alpha starts at ones;
    minimize(opt, alpha) differentiates the tuple (value, gradient) that opt returns, so the step
    uses grad = (K alpha - y) + K 1 (K = exact K + noise I); the value is
    1/2 alpha^T K alpha - alpha^T y - 1/2 nystroem_det - n/2 log 2 pi at the stepped alpha."""
    y = np.asarray(y, np.float64).reshape(-1, 1)
    n = y.shape[0]
    K = k_noised(tree, hyp, noise, x, scaled, se_expanded)
    a = np.ones((n, 1))
    g = (K @ a - y) + K @ np.ones((n, 1))
    a = vsgd_step(a, g)
    fit = 0.5 * float(a.T @ K @ a) - float(a.T @ y)
    det = nystroem_det(tree, hyp, noise, x, z, scaled, se_expanded)
    return fit - 0.5 * det - 0.5 * n * math.log(2 * math.pi)


def ski_inducing_indices(n: int, m: int) -> np.ndarray:
    """np.linspace(0, n, num=m, endpoint=False, dtype=int) (StructuredKernelInterpolation.py:14-16)."""
    return np.linspace(start=0, stop=n, num=m, endpoint=False, dtype=int)


def ski_weight_matrix(x: np.ndarray, z: np.ndarray) -> np.ndarray:
    """get_weight_matrix (Metrics/StructuredKernelInterpolation.py:31-49), op for op."""
    distances = euclidian_distance(x, z)
    reduce_min_1 = distances.min(axis=1).reshape(-1, 1)
    min_1_condition = distances == reduce_min_1
    mask_1_distances = distances.max() * min_1_condition.astype(np.float64)
    distances_masked = distances + mask_1_distances
    reduce_min_2 = distances_masked.min(axis=1).reshape(-1, 1)
    min_2_condition = distances_masked == reduce_min_2
    weight_i = 1 - reduce_min_1 / (reduce_min_1 + reduce_min_2)
    return (np.zeros_like(distances) + weight_i * min_1_condition.astype(np.float64)
            + (1 - weight_i) * min_2_condition.astype(np.float64))


def ski_matrix(tree, hyp, noise, x, m: int, scaled=False, se_expanded=False) -> np.ndarray:
    """get_ski_matrix (StructuredKernelInterpolation.py:10-28): W K_mm W^T + noise I with the
    inducing points x[linspace indices]."""
    idx = ski_inducing_indices(x.shape[0], m)
    z = x[idx]
    kmm = kernel_matrix(tree, hyp, z, z, scaled, se_expanded)
    w = ski_weight_matrix(x, z)
    return (w @ kmm) @ w.T + np.eye(x.shape[0]) * noise


def ski_nlml(tree, hyp, noise, x, y, m: int, handling: str = "CHOLESKY_BASED", scaled=False,
             se_expanded=False) -> float:
    """LogLikelihood.get_metric with SKI: only get_covariance_matrix changes (Metrics/Metrics.py:104-105),
    so CHOLESKY_BASED (alpha and log-det from the holistic covariance matrix) is the exact -LML and
    the other handlings use W K_mm W^T + noise I with slogdet."""
    y = np.asarray(y, np.float64).reshape(-1, 1)
    n = y.shape[0]
    if handling == "CHOLESKY_BASED":
        return nlml(tree, hyp, noise, x, y, scaled, se_expanded)
    K = ski_matrix(tree, hyp, noise, x, m, scaled, se_expanded)
    if handling == "LINEAR_CONJUGATE_GRADIENT":
        alpha = linear_cg(K, y, np.zeros_like(y))
    elif handling == "PSEUDO_INVERSE":
        alpha = tf_pinv(K) @ y
    else:
        alpha = np.linalg.inv(K) @ y
    logdet = np.linalg.slogdet(K)[1]
    return -(-0.5 * float(y.T @ alpha) - 0.5 * logdet - 0.5 * n * math.log(2 * math.pi))
