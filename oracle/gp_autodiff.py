"""CPU gradient oracle: reverse-mode autodiff (torch, fp64, CPU) of the reference's -LML op sequence.

TEST INFRASTRUCTURE ONLY (same rules as ``gp_oracle``: imported by ``tests/`` and nothing in
the product package).

The reference differentiates ``LogLikelihood.get_metric`` with ``tf.GradientTape`` inside
``VariationalSgdFitter.fit`` (gpbasics/Optimizer/Fitter.py:104-158; TensorFlow's autodiff through
``tf.linalg.cholesky`` / ``triangular_solve``).  TensorFlow cannot run here, so this module
restates the same forward op sequence as ``gp_oracle`` -- kernel formulas
(K/BaseKernels.py:277-294, :440-457, :702-720, :859-880), ADD/MUL folding with DFS
hyperparameter slicing (K/Operators.py:207-225, :306-326), noise on the diagonal
(S/CovarianceMatrix.py:197-206), Cholesky + two triangular solves (:247-265), log-determinant and
-LML assembly (M/Metrics.py:152-154, M/LogLikelihood.py:30-65) -- in torch and lets torch's
reverse mode produce the gradient, which is what GradientTape computes (including the
derivative of |l| as sign(l) in the Matern kernels).  Pinned in tests/test_oracle.py by (a) its
forward value == gp_oracle.nlml and (b) central finite differences of gp_oracle.nlml.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np
import torch

F64 = torch.float64
LOG_2PI = math.log(2.0 * math.pi)


def _n_hyp(tree, scaled: bool) -> int:
    op, arg = tree
    if op in ("ADD", "MUL"):
        return sum(_n_hyp(c, scaled) for c in arg)
    return (2 if op == "PER" else 1) + (1 if scaled else 0)


def _l1(a, b):
    return torch.sum(torch.abs(a[:, None, :] - b[None, :, :]), dim=-1)


def _sq(a, b):
    d = a[:, None, :] - b[None, :, :]
    return torch.sum(d * d, dim=-1)


def _base(op, opts, hyp, x, x_, scaled, se_expanded):
    ard = bool(opts.get("ard", False))
    if op == "SE":
        if ard:
            x, x_, l = x / hyp[0], x_ / hyp[0], None
        else:
            l = hyp[0]
        if se_expanded:
            na = torch.sum(x * x, -1, keepdim=True)
            nb = torch.sum(x_ * x_, -1, keepdim=True)
            dist = torch.sqrt((na - 2.0 * (x @ x_.T)) + nb.T)
            s = dist * dist
        else:
            s = _sq(x, x_)
        r = torch.exp(-0.5 * s) if l is None else torch.exp(-0.5 * (s / (l * l)))
        return hyp[1] * r if scaled else r
    if op in ("MAT32", "MAT52"):
        if ard:
            x, x_, l = x / hyp[0], x_ / hyp[0], None
        else:
            l = torch.abs(hyp[0])
        if opts.get("standard", False):
            s = _sq(x, x_)
            # sqrt at 0 has an infinite derivative; the distance itself does not depend on
            # the hyperparameters unless ARD, where d sqrt(s)/d l is finite away from s = 0
            dist = torch.sqrt(torch.clamp(s, min=1e-300)) * (s > 0)
        else:
            dist = _l1(x, x_)
        c = math.sqrt(5.0) if op == "MAT52" else math.sqrt(3.0)
        frac = (c * dist) if l is None else (c * dist) / l
        if op == "MAT52":
            third = (5.0 * (dist * dist)) / 3.0 if l is None else (5.0 * (dist * dist)) / (3.0 * (l * l))
            r = ((1.0 + frac) + third) * torch.exp(-frac)
        else:
            r = (1.0 + frac) * torch.exp(-frac)
        return hyp[1] * r if scaled else r
    if op == "PER":
        l, p = hyp[0], hyp[1]
        if opts.get("standard", False):
            dd = torch.abs(x[:, None, :] - x_[None, :, :])
            sd = torch.sin(math.pi * (dd / p))
            sine = torch.sum(sd * sd, dim=-1)
        else:
            sine = torch.sin(math.pi * (_l1(x, x_) / p))
            sine = sine * sine
        r = torch.exp((-2.0 * sine) / (l * l))
        return hyp[2] * r if scaled else r
    raise ValueError(op)


def _kmat(tree, hyp, x, x_, scaled, se_expanded):
    op, arg = tree
    if op in ("ADD", "MUL"):
        idx, res = 0, None
        for child in arg:
            k = _n_hyp(child, scaled)
            m = _kmat(child, hyp[idx:idx + k], x, x_, scaled, se_expanded)
            idx += k
            res = m if res is None else (res + m if op == "ADD" else res * m)
        return res
    return _base(op, arg, hyp, x, x_, scaled, se_expanded)


def nlml_and_grad(tree, hyp: List, noise: float, x: np.ndarray, y: np.ndarray, scaled: bool = False,
                  se_expanded: bool = False) -> Tuple[float, List[np.ndarray], float]:
    """(-LML, [d/d h for h in hyp] shaped like h, d/d noise) by torch reverse mode on the CPU."""
    params = [torch.tensor(np.asarray(h, dtype=np.float64), dtype=F64, requires_grad=True) for h in hyp]
    nz = torch.tensor(float(noise), dtype=F64, requires_grad=True)
    X = torch.as_tensor(np.asarray(x, dtype=np.float64))
    Y = torch.as_tensor(np.asarray(y, dtype=np.float64)).reshape(-1, 1)
    n = X.shape[0]
    K = _kmat(tree, params, X, X, scaled, se_expanded) + nz * torch.eye(n, dtype=F64)
    L = torch.linalg.cholesky(K)
    z = torch.linalg.solve_triangular(L, Y, upper=False)
    alpha = torch.linalg.solve_triangular(L.T, z, upper=True)
    fit = (Y.T @ alpha)[0, 0]
    logdet = 2.0 * torch.sum(torch.log(torch.diagonal(L)))
    nl = -((-0.5 * fit + -0.5 * logdet) + (-0.5 * (n * LOG_2PI)))
    grads = torch.autograd.grad(nl, params + [nz])
    return float(nl.detach()), [g.numpy() for g in grads[:-1]], float(grads[-1])


def finite_difference(f, hyp: Sequence, noise: float, h: float = 1e-5):
    """Central differences of f(hyp, noise) -> float over every scalar of hyp and noise."""
    flat = [np.atleast_1d(np.asarray(v, dtype=np.float64)).copy() for v in hyp]
    out = []
    for i, v in enumerate(flat):
        g = np.zeros_like(v)
        for j in range(v.size):
            step = h * max(1.0, abs(v[j]))
            vp, vm = [u.copy() for u in flat], [u.copy() for u in flat]
            vp[i][j] += step
            vm[i][j] -= step
            unpack = lambda vs: [u if np.ndim(hyp[k]) else float(u[0]) for k, u in enumerate(vs)]
            g[j] = (f(unpack(vp), noise) - f(unpack(vm), noise)) / (2 * step)
        out.append(g.reshape(np.shape(hyp[i])))
    step = h * max(1.0, abs(noise))
    unpack0 = [u if np.ndim(hyp[k]) else float(u[0]) for k, u in enumerate(flat)]
    gn = (f(unpack0, noise + step) - f(unpack0, noise - step)) / (2 * step)
    return out, gn


# ----------------------------------------------------------------------------- approximations (§8f.4)
def tf_pinv(A: torch.Tensor) -> torch.Tensor:
    """tf.linalg.pinv (Statistics/Nystroem_K.py:53) in torch, differentiable the way TensorFlow's is: SVD,
    singular values s > 10 max(shape) eps max(s) inverted, the rest dropped (their reciprocal masked
    without a NaN in the backward)."""
    U, s, Vh = torch.linalg.svd(A, full_matrices=False)
    rcond = 10.0 * max(A.shape) * float(np.finfo(np.float64).eps)
    keep = s > rcond * s.max()
    s_safe = torch.where(keep, s, torch.ones_like(s))
    s_inv = torch.where(keep, 1.0 / s_safe, torch.zeros_like(s))
    return (Vh.mT * s_inv) @ U.mT


def pinv_or_inv(A: torch.Tensor) -> torch.Tensor:
    """tf_pinv for a matrix whose singular values are all kept is inv(A); differentiate it as inv then.
    (K_hat + noise I has n - m eigenvalues equal to the noise: an SVD-based backward divides by their zero
    differences -- TensorFlow regularises that reciprocal -- while the derivative of the pseudo-inverse
    itself, which is inv's there, is finite.  The device returns that analytic derivative.)"""
    s = torch.linalg.svdvals(A.detach())
    rcond = 10.0 * max(A.shape) * float(np.finfo(np.float64).eps)
    if bool((s > rcond * s.max()).all()):
        return torch.linalg.inv(A)
    return tf_pinv(A)


def kernel_matrix_t(tree, hyp, x, x_, scaled: bool = False) -> torch.Tensor:
    """The kernel program in torch (differentiable in hyp and both inputs; direct squared distances for
    SE, so coincident points differentiate to 0 rather than TensorFlow's sqrt'(0) = inf times 0)."""
    return _kmat(tree, hyp, x, x_, scaled, False)


def nystroem_nlml_and_grad(tree, hyp: List, noise: float, x: np.ndarray, y: np.ndarray, z: np.ndarray,
                           handling: str = "CHOLESKY_BASED", lower_bound: bool = False, jitter: float = 1e-8,
                           scaled: bool = False, det_fresh: bool = True):
    """-LML of BASIC_NYSTROEM / SKC_LOWER_BOUND (gp_oracle.nystroem_nlml, op for op) and its reverse-mode
    gradient w.r.t. the hyperparameters, the noise and the inducing inputs z -- GradientTape through
    Optimizer/Fitter.py:124-132.  det_fresh=False treats the Nystroem log-determinant as the constant the
    reference's cache makes of it after an earlier call (Nystroem_K.py:92-93).
    Returns (nlml, [d/d h], d/d noise, d/d z or None)."""
    params = [torch.tensor(np.asarray(h, dtype=np.float64), dtype=F64, requires_grad=True) for h in hyp]
    nz = torch.tensor(float(noise), dtype=F64, requires_grad=True)
    Z = torch.tensor(np.asarray(z, dtype=np.float64), dtype=F64, requires_grad=True)
    X = torch.as_tensor(np.asarray(x, dtype=np.float64))
    Y = torch.as_tensor(np.asarray(y, dtype=np.float64)).reshape(-1, 1)
    n, m = X.shape[0], Z.shape[0]
    knm = kernel_matrix_t(tree, params, X, Z, scaled)
    kmm = kernel_matrix_t(tree, params, Z, Z, scaled)
    P = tf_pinv(kmm)
    khat = (knm @ P) @ knm.T
    eye = torch.eye(n, dtype=F64)
    if handling == "CHOLESKY_BASED":
        K = kernel_matrix_t(tree, params, X, X, scaled) + nz * eye
        L = torch.linalg.cholesky(K)
        alpha = torch.cholesky_solve(Y, L)
    elif handling == "PSEUDO_INVERSE":
        alpha = pinv_or_inv(khat + nz * eye) @ Y
    elif handling == "STRICT_INVERSE":
        alpha = torch.linalg.inv(khat + nz * eye) @ Y
    elif handling == "LINEAR_CONJUGATE_GRADIENT":
        alpha, _ = cg_torch(khat + nz * eye, Y)
    else:
        raise ValueError(handling)
    fit = (Y.T @ alpha)[0, 0]
    to_det = torch.eye(m, dtype=F64) * nz + knm.T @ (knm @ P)
    det = (n - m) * torch.log(nz) + torch.linalg.slogdet(to_det)[1]
    if not det_fresh:
        det = det.detach()
    ll = -0.5 * fit - 0.5 * det - 0.5 * n * LOG_2PI
    if lower_bound:
        kxx = kernel_matrix_t(tree, params, X, X, scaled)
        ll = ll - (1.0 / (2.0 * jitter)) * torch.trace(khat + nz * eye - kxx)
    nl = -ll
    grads = torch.autograd.grad(nl, params + [nz, Z], allow_unused=True)
    gz = grads[-1]
    return (float(nl.detach()), [g.numpy() if g is not None else np.zeros(np.shape(h)) for g, h in zip(grads[:-2], hyp)],
            float(grads[-2]), gz.numpy() if gz is not None else None)


def ski_nlml_and_grad(tree, hyp: List, noise: float, x: np.ndarray, y: np.ndarray, m: int,
                      handling: str = "STRICT_INVERSE", scaled: bool = False):
    """-LML of SKI with STRICT / PSEUDO inverse or linear CG (gp_oracle.ski_nlml) and its gradient w.r.t. the
    hyperparameters and the noise (the inducing points x[linspace] and the weights are constants)."""
    from . import gp_oracle as o
    params = [torch.tensor(np.asarray(h, dtype=np.float64), dtype=F64, requires_grad=True) for h in hyp]
    nz = torch.tensor(float(noise), dtype=F64, requires_grad=True)
    X = np.asarray(x, dtype=np.float64)
    Y = torch.as_tensor(np.asarray(y, dtype=np.float64)).reshape(-1, 1)
    n = X.shape[0]
    idx = o.ski_inducing_indices(n, m)
    Zt = torch.as_tensor(X[idx])
    W = torch.as_tensor(o.ski_weight_matrix(X, X[idx]))
    kmm = kernel_matrix_t(tree, params, Zt, Zt, scaled)
    A = (W @ kmm) @ W.T + nz * torch.eye(n, dtype=F64)
    if handling == "LINEAR_CONJUGATE_GRADIENT":
        alpha, _ = cg_torch(A, Y)
    else:
        alpha = (pinv_or_inv(A) if handling == "PSEUDO_INVERSE" else torch.linalg.inv(A)) @ Y
    fit = (Y.T @ alpha)[0, 0]
    logdet = torch.linalg.slogdet(A)[1]
    nl = -(-0.5 * fit - 0.5 * logdet - 0.5 * n * LOG_2PI)
    grads = torch.autograd.grad(nl, params + [nz])
    return float(nl.detach()), [g.numpy() for g in grads[:-1]], float(grads[-1])


def inverse_nlml_and_grad(tree, hyp: List, noise: float, x: np.ndarray, y: np.ndarray, handling: str,
                          scaled: bool = False):
    """-LML with STRICT_INVERSE (inv(K) y) / PSEUDO_INVERSE (pinv(K) y) and slogdet (M/Metrics.py:132-136,
    :146-147) and its reverse-mode gradient -- for any nonsingular K + noise I, positive definite or not."""
    params = [torch.tensor(np.asarray(h, dtype=np.float64), dtype=F64, requires_grad=True) for h in hyp]
    nz = torch.tensor(float(noise), dtype=F64, requires_grad=True)
    X = torch.as_tensor(np.asarray(x, dtype=np.float64))
    Y = torch.as_tensor(np.asarray(y, dtype=np.float64)).reshape(-1, 1)
    n = X.shape[0]
    K = kernel_matrix_t(tree, params, X, X, scaled) + nz * torch.eye(n, dtype=F64)
    alpha = (pinv_or_inv(K) if handling == "PSEUDO_INVERSE" else torch.linalg.inv(K)) @ Y
    nl = -(-0.5 * (Y.T @ alpha)[0, 0] - 0.5 * torch.linalg.slogdet(K)[1] - 0.5 * n * LOG_2PI)
    grads = torch.autograd.grad(nl, params + [nz])
    return float(nl.detach()), [g.numpy() for g in grads[:-1]], float(grads[-1])


def cg_torch(K: torch.Tensor, Y: torch.Tensor):
    """linear_cg(K, Y, 0) (Auxiliary/LinearConjugateGradients.py:9-41) op for op in torch, differentiable
    through the executed iterations as tf.GradientTape records them: the |max r| > 1e-2 stopping rule, the
    NaN early return, the n-iteration guard.  Returns (x, iterations)."""
    n = K.shape[0]
    xk = torch.zeros((n, 1), dtype=F64)
    r = K @ xk - Y
    p = -r
    k, first = 0, True
    while first or float(torch.abs(torch.max(r))) > 1e-2:
        Ap = K @ p
        a = (r.T @ r) / (p.T @ Ap)
        nxt = xk + a * p
        if bool(torch.any(torch.isnan(nxt))):
            break
        xk = nxt
        r1 = r + a * Ap
        beta = (r1.T @ r1) / (r.T @ r)
        p = -r1 + beta * p
        r = r1
        k += 1
        first = False
        if k % (n / 4) == 0 and k > n:
            break
    return xk, k


def lcg_nlml_and_grad(tree, hyp: List, noise: float, x: np.ndarray, y: np.ndarray, scaled: bool = False):
    """-LML with LINEAR_CONJUGATE_GRADIENT (alpha = linear_cg(K, y, 0), M/Metrics.py:141-144, the loop of
    Auxiliary/LinearConjugateGradients.py:9-41 restated op for op -- |max r| > 1e-2 stopping rule, NaN early
    return, the n-iteration guard) and slogdet (:146-147), with its reverse-mode gradient through the executed
    iterations, as tf.GradientTape records them.  Returns (nlml, [grad per hyperparameter], grad noise,
    iterations)."""
    params = [torch.tensor(np.asarray(h, dtype=np.float64), dtype=F64, requires_grad=True) for h in hyp]
    nz = torch.tensor(float(noise), dtype=F64, requires_grad=True)
    X = torch.as_tensor(np.asarray(x, dtype=np.float64))
    Y = torch.as_tensor(np.asarray(y, dtype=np.float64)).reshape(-1, 1)
    n = X.shape[0]
    K = kernel_matrix_t(tree, params, X, X, scaled) + nz * torch.eye(n, dtype=F64)
    xk, k = cg_torch(K, Y)
    nl = -(-0.5 * (Y.T @ xk)[0, 0] - 0.5 * torch.linalg.slogdet(K)[1] - 0.5 * n * LOG_2PI)
    grads = torch.autograd.grad(nl, params + [nz])
    return float(nl.detach()), [g.numpy() for g in grads[:-1]], float(grads[-1]), k


def batch_nlml_and_grad(tree, hyp: List, noise: float, xb: np.ndarray, yb: np.ndarray,
                        handling: str = "CHOLESKY_BASED", agg: str = "mean", scaled: bool = False):
    """BatchDataInput -LML (quirk Q7) and its gradient: CHOLESKY_BASED -agg_b(-1/2 fit_b - 1/2 sum_b' logdet_b'
    - c) (M/LogLikelihood.py:39-63 with M/Metrics.py:153-154's axis-free reduce_sum); STRICT / PSEUDO
    inverse: -agg over the [B, 1, B] broadcast of fit_b and slogdet_b' (gp_oracle.batch_nlml's sibling)."""
    params = [torch.tensor(np.asarray(h, dtype=np.float64), dtype=F64, requires_grad=True) for h in hyp]
    nz = torch.tensor(float(noise), dtype=F64, requires_grad=True)
    B, n = xb.shape[0], xb.shape[1]
    fits, logdets = [], []
    for b in range(B):
        X = torch.as_tensor(np.asarray(xb[b], dtype=np.float64))
        Y = torch.as_tensor(np.asarray(yb[b], dtype=np.float64)).reshape(-1, 1)
        K = kernel_matrix_t(tree, params, X, X, scaled) + nz * torch.eye(n, dtype=F64)
        L = torch.linalg.cholesky(K)
        fits.append((Y.T @ torch.cholesky_solve(Y, L))[0, 0])
        logdets.append(2.0 * torch.sum(torch.log(torch.diagonal(L))))
    fit, logdet = torch.stack(fits), torch.stack(logdets)
    c = 0.5 * n * LOG_2PI
    red = torch.mean if agg == "mean" else torch.sum
    if handling == "CHOLESKY_BASED":
        ll = -0.5 * fit - 0.5 * torch.sum(logdet) - c
    else:
        ll = (-0.5 * fit).reshape(B, 1, 1) + (-0.5 * logdet).reshape(1, 1, B) - c
    nl = -red(ll)
    grads = torch.autograd.grad(nl, params + [nz])
    return float(nl.detach()), [g.numpy() for g in grads[:-1]], float(grads[-1])


def skc_upper_nlml_and_grad(tree, hyp: List, noise: float, x: np.ndarray, y: np.ndarray, z: np.ndarray,
                            k_fresh: bool = True, det_fresh: bool = True, scaled: bool = False):
    """LogLikelihoodUpperBound.get_metric (gp_oracle.skc_upper_bound, Metrics/SkcLogLikelihood.py:26-69) and
    the gradient tf.GradientTape takes of it (Optimizer/Fitter.py:76-87): the VariationalSGD step writes
    alpha by a variable assignment, which the tape does not differentiate, so alpha is a constant for it
    and the value 1/2 alpha^T K alpha - alpha^T y - 1/2 det - n/2 log 2 pi is differentiated at the stepped
    alpha.  K (the metric's last_covariance_matrix) and the Nystroem determinant are cached across calls
    (the metric never resets): a cached one is a constant for the tape -- k_fresh / det_fresh say whether
    this call computed them.  Returns (value, [d/d h], d/d noise, d/d z or None)."""
    from . import gp_oracle as o
    params = [torch.tensor(np.asarray(h, dtype=np.float64), dtype=F64, requires_grad=True) for h in hyp]
    nz = torch.tensor(float(noise), dtype=F64, requires_grad=True)
    Z = torch.tensor(np.asarray(z, dtype=np.float64), dtype=F64, requires_grad=True)
    X = torch.as_tensor(np.asarray(x, dtype=np.float64))
    Y = torch.as_tensor(np.asarray(y, dtype=np.float64)).reshape(-1, 1)
    n, m = X.shape[0], Z.shape[0]
    K = kernel_matrix_t(tree, params, X, X, scaled) + nz * torch.eye(n, dtype=F64)
    Kd = K.detach()
    one = torch.ones((n, 1), dtype=F64)
    g = (Kd @ one - Y) + Kd @ one
    a = torch.as_tensor(o.vsgd_step(one.numpy(), g.numpy()))
    Ku = K if k_fresh else Kd
    fit = 0.5 * (a.T @ Ku @ a)[0, 0] - (a.T @ Y)[0, 0]
    knm = kernel_matrix_t(tree, params, X, Z, scaled)
    kmm = kernel_matrix_t(tree, params, Z, Z, scaled)
    P = tf_pinv(kmm)
    to_det = torch.eye(m, dtype=F64) * nz + knm.T @ (knm @ P)
    det = (n - m) * torch.log(nz) + torch.linalg.slogdet(to_det)[1]
    if not det_fresh:
        det = det.detach()
    val = fit - 0.5 * det - 0.5 * n * LOG_2PI
    grads = torch.autograd.grad(val, params + [nz, Z], allow_unused=True)
    gz = grads[-1]
    return (float(val.detach()), [gg.numpy() if gg is not None else np.zeros(np.shape(h)) for gg, h in zip(grads[:-2], hyp)],
            float(grads[-2]) if grads[-2] is not None else 0.0, gz.numpy() if gz is not None else None)
