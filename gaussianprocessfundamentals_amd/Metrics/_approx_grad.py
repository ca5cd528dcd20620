"""Reverse mode of the approximate -LML metrics (SURVEY §8f.1 with §8f.4): what tf.GradientTape computes
through LogLikelihood.get_metric under BASIC_NYSTROEM / SKC_LOWER_BOUND / SKI when the reference's only
live fitter differentiates it with respect to ``hyper_parameter + [indices]`` and the noise
(gpbasics/Optimizer/Fitter.py:76-87, :124-132, :155-156).

-LML = 1/2 fit + 1/2 logdet + 1/2 n log 2 pi  (+ trace(K_hat + noise I - K) / (2 p_cov_matrix_jitter) for
SKC_LOWER_BOUND, Metrics/LogLikelihood.py:51-60), with the pieces bound by Metric.__init__
(Metrics/Metrics.py:82-107):

  fit      CHOLESKY_BASED: y^T alpha with the EXACT alpha (get_alpha_cholesky reads the holistic matrix);
           STRICT / PSEUDO inverse: y^T (K_hat + noise I)^-1 y
  logdet   Nystroem: (n - m) log noise + slogdet(noise I_m + K_mn K_nm pinv(K_mm)) (Nystroem_K.py:92-108)
           -- cached by the Nystroem handler across get_metric calls: a value computed by an earlier call
           is a constant for the tape (the fitter's pre-fit evaluation, Fitter.py:120, computes it outside
           the tape), so it contributes to the gradient only in the call that computes it;
           SKI with STRICT / PSEUDO: slogdet(W K_mm W^T + noise I)

Device mapping: every piece hands back the adjoints of K_nm = k(X, Z) (dense [n, m]), of P = pinv(K_mm)
([m, m]) and of the noise; pinv's reverse mode is gpk_pinv_backward_scale on K_mm's eigendecomposition
(engine.pinv_backward) and the kernel matrices' reverse mode gpk_kernel_vjp, which also yields the
adjoint of the inducing inputs Z.  The exact fit's adjoint -alpha alpha^T goes to gpk_kernel_vjp as a
rank-1 weight (no n x n matrix).  Every product is gpk_dgemm (f64 MFMA), every inverse / log-determinant
the augmented Cholesky; torch only sums adjoint buffers.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from .. import engine
from .. import global_parameters as global_param


class NystroemAdjoint:
    """Accumulates the adjoints of K_nm, pinv(K_mm), the noise and the flat hyperparameters for one
    evaluation, then maps K_nm / K_mm adjoints to hyperparameters and inducing inputs."""

    def __init__(self, kernel, hyp: List, X: torch.Tensor, Z: Optional[torch.Tensor], noise: float):
        self.kernel, self.hyp, self.X, self.Z, self.noise = kernel, hyp, X, Z, float(noise)
        self.n = int(X.shape[0])
        d = int(X.shape[1])
        kd = engine.kernel_descriptor(kernel, d)
        dev = X.device
        self.hyp_bar = torch.zeros(kd.n_hyp, dtype=torch.float64, device=dev)
        self.noise_bar = torch.zeros((), dtype=torch.float64, device=dev)
        self.knm_bar = None
        self.t_bar = None
        self._nys = None

    # -- Nystroem pieces --------------------------------------------------------------------------
    def nystroem(self):
        """K_nm, eigendecomposition of K_mm, P = pinv(K_mm) (tf.linalg.pinv's cutoff), cached."""
        if self._nys is None:
            knm = engine.kernel_matrix(self.kernel, self.hyp, self.X, self.Z)
            kmm = engine.kernel_matrix(self.kernel, self.hyp, self.Z, self.Z)
            lam, V, _ = engine.eigh(kmm)
            U0, _, mu0 = engine.pinv_factor(lam, V, 0, return_mu=True)
            P = engine.dgemm(U0, V, trans_b=True)
            self._nys = (knm, lam, V, mu0, P)
        return self._nys

    def _acc_knm(self, M: torch.Tensor, w: float):
        if self.knm_bar is None:
            self.knm_bar = torch.zeros_like(M)
        self.knm_bar.add_(M, alpha=w)

    def _acc_knm_rank1(self, u: torch.Tensor, v: torch.Tensor, w: float):
        """K_nm adjoint += w u v^T (a K = 1 MFMA GEMM)."""
        knm = self.nystroem()[0]
        if self.knm_bar is None:
            self.knm_bar = torch.zeros_like(knm)
        engine.dgemm(u.reshape(-1, 1).contiguous(), v.reshape(1, -1).contiguous(), alpha=w, beta=1.0, C=self.knm_bar)

    def _acc_t(self, T: torch.Tensor, w: float):
        """adjoint of pinv(K_mm) in K_mm's eigenbasis (V^T Pbar V) += w T"""
        if self.t_bar is None:
            self.t_bar = torch.zeros_like(T)
        self.t_bar.add_(T, alpha=w)

    def _acc_p(self, M: torch.Tensor, w: float):
        """adjoint of pinv(K_mm) += w M (M in the standard basis)"""
        V = self.nystroem()[2]
        self._acc_t(engine.dgemm(engine.dgemm(V, M.contiguous(), trans_a=True), V), w)

    def exact_fit(self, alpha: torch.Tensor, w: float):
        """fit = y^T (K + noise I)^-1 y: d fit = -alpha^T dK alpha - d noise alpha^T alpha (rank-1 VJP)."""
        a = alpha.reshape(-1).contiguous()
        gh, _ = engine.kernel_vjp(self.kernel, self.hyp, self.X, self.X, gu=a, gv=a)
        self.hyp_bar.add_(gh, alpha=-w)
        self.noise_bar.add_(torch.dot(a, a), alpha=-w)

    def nystroem_logdet(self, w: float):
        """(n - m) log noise + log|det C|, C = noise S + D S~ D in K_mm's eigenbasis (S~ = V^T K_mn K_nm V,
        D = diag(|lam|^-1/2) on the kept eigenvalues, 0 on the dropped ones, S = diag(sign lam) with +1 on the
        dropped ones; log|det C| equals the reference's slogdet(noise I + K_mn K_nm pinv(K_mm))[1], Nystroem_K.py):
          d/d noise = (n - m) / noise + tr(C^-1 S),   d/d K_nm = 2 G C^-1 U^T   (U = V D, G = K_nm U),
          d/d pinv(K_mm) in the eigenbasis: (I + S~ F / noise)^-1 S~ / noise (F = D S D), written without its
          cancellation as D^-1 S (S - noise C^-1) S D^-1 on the kept block and D^-1 S C^-1 D S~ on the kept x
          dropped one (the dropped block is multiplied by 0 in pinv's reverse mode).  For a kernel matrix K_mm
          S = I and C = noise I + G^T G is positive definite (augmented Cholesky); an indefinite K_mm (the
          reference's L1 forms at D > 1) takes C^-1 from the eigendecomposition."""
        from ..Statistics.Nystroem_K import signed_pinv_factor, sym_inverse
        knm, lam, V, mu0, P = self.nystroem()
        n, m = self.n, int(V.shape[0])
        U1, sgn, n_neg, mu1 = signed_pinv_factor(lam, V)
        G = engine.dgemm(knm, U1)
        S = engine.dgemm(G, G, trans_a=True)
        if n_neg == 0:
            cinv = engine.DenseFactorization(m, inverse=True).run(S.contiguous(), self.noise)
            cinv.check_info()
            Ci = cinv.k_inv(0).to(torch.float64).contiguous()
            tr = torch.trace(Ci)
        else:
            C = S.clone()
            C.diagonal().add_(self.noise * sgn)
            Ci = sym_inverse(C).contiguous()
            tr = torch.sum(torch.diagonal(Ci) * sgn)
        self.noise_bar.add_((n - m) / self.noise + tr, alpha=w)
        self._acc_knm(engine.dgemm(engine.dgemm(G, Ci), U1, trans_b=True), 2.0 * w)
        kept = mu1 != 0
        dinv = torch.where(kept, 1.0 / torch.where(kept, mu1, torch.ones_like(mu1)), torch.zeros_like(mu1))
        ds = dinv * sgn
        T = -self.noise * Ci
        T.diagonal().add_(sgn)
        T = ds[:, None] * T * ds[None, :]
        if not bool(kept.all()):
            KV = engine.dgemm(knm, V)
            St = engine.dgemm(KV, KV, trans_a=True)
            Q = engine.dgemm((ds[:, None] * Ci * mu1[None, :]).contiguous(), St)
            Q = Q * (kept[:, None] & ~kept[None, :])
            T = T + Q + Q.T
        self._acc_t(T, w)

    def lowrank_matrix_adjoint(self, P: torch.Tensor, Q: torch.Tensor):
        """Adjoint Q P^T of the whole approximate matrix K_hat + noise I = K_nm pinv(K_mm) K_mn + noise I
        (from the CG iterations, [n, k] each): d/d K_nm = (Kbar + Kbar^T) K_nm P_m, d/d pinv(K_mm) =
        K_mn Kbar K_nm, d/d noise = tr Kbar -- all through the k-column factors, no n x n matrix."""
        if P.shape[1] == 0:
            return
        knm, _, _, _, Pm = self.nystroem()
        KP = engine.dgemm(knm, Pm)                              # K_nm P_m          [n, m]
        ptk = engine.dgemm(P, KP, trans_a=True)                 # P^T K_nm P_m      [k, m]
        qtk = engine.dgemm(Q, KP, trans_a=True)
        M = engine.dgemm(Q, ptk)
        engine.dgemm(P, qtk, beta=1.0, C=M)                     # Q P^T K P_m + P Q^T K P_m
        self._acc_knm(M, 1.0)
        a = engine.dgemm(Q, knm, trans_a=True)                  # Q^T K_nm          [k, m]
        b = engine.dgemm(P, knm, trans_a=True)
        self._acc_p(engine.dgemm(a, b, trans_a=True), 1.0)      # K_mn Q P^T K_nm
        self.noise_bar.add_(torch.sum(P * Q))

    def approx_fit(self, alpha_hat: torch.Tensor, w: float):
        """fit = y^T (K_hat + noise I)^-1 y with K_hat = K_nm P K_mn: d/d K_nm = -2 a (P K_mn a)^T,
        d/d P = -(K_mn a)(K_mn a)^T, d/d noise = -a^T a  (a = alpha_hat)."""
        knm, _, _, _, P = self.nystroem()
        a = alpha_hat.reshape(-1, 1).contiguous()
        t = engine.dgemm(knm, a, trans_a=True)            # K_mn a   [m, 1]
        Pt = engine.dgemm(P, t)
        self._acc_knm_rank1(a, Pt, -2.0 * w)
        self._acc_p(engine.dgemm(t, t, trans_b=True), -w)
        self.noise_bar.add_(torch.sum(a * a), alpha=-w)

    def trace_correction(self, w: float):
        """trace(K_nm P K_mn + noise I - K): d/d K_nm = 2 K_nm P, d/d P = K_mn K_nm, d/d noise = n, and
        -n d k(x, x) / d theta (stationary kernels: k(x, x) is the same for every x)."""
        knm, _, _, _, P = self.nystroem()
        self._acc_knm(engine.dgemm(knm, P), 2.0 * w)
        self._acc_p(engine.dgemm(knm, knm, trans_a=True), w)
        self.noise_bar.add_(torch.tensor(float(self.n), dtype=torch.float64, device=self.X.device), alpha=w)
        one = torch.ones(1, dtype=torch.float64, device=self.X.device)
        gh, _ = engine.kernel_vjp(self.kernel, self.hyp, self.X[:1], self.X[:1], gu=one, gv=one)
        self.hyp_bar.add_(gh, alpha=-w * self.n)

    def finish(self, want_z: bool):
        """Map the K_nm / P adjoints to (flat hyperparameter adjoint, noise adjoint, Z adjoint or None)."""
        gz = None
        if self.knm_bar is not None or self.t_bar is not None:
            knm, lam, V, mu0, P = self.nystroem()
            if self.knm_bar is not None:
                gh, gz1 = engine.kernel_vjp(self.kernel, self.hyp, self.X, self.Z, G=self.knm_bar, want_z=want_z)
                self.hyp_bar.add_(gh)
                gz = gz1
            if self.t_bar is not None:
                kbar = engine.pinv_backward(lam, V, mu0, T=self.t_bar)
                # K_mm = k(Z, Z) symmetric: weights Kbar + Kbar^T give the full Z adjoint, twice the hyp one
                gh, gz2 = engine.kernel_vjp(self.kernel, self.hyp, self.Z, self.Z, G=(2.0 * kbar).contiguous(),
                                            want_z=want_z)
                self.hyp_bar.add_(gh, alpha=0.5)
                gz = gz2 if gz is None else gz + gz2
        return self.hyp_bar, self.noise_bar, gz


def ski_adjoint(metric, hyp: List, noise, alpha_hat: torch.Tensor, Ainv: torch.Tensor):
    """SKI with STRICT / PSEUDO inverse: -LML = 1/2 y^T A^-1 y + 1/2 slogdet A + c, A = W K_zz W^T + noise I
    (Metrics/StructuredKernelInterpolation.py:10-28, Z = x_train[linspace] fixed): the adjoint of A is
    1/2 (A^-1 - a a^T), so K_zz's is W^T (.) W and the noise's its trace.  Returns (hyp adjoint, noise
    adjoint)."""
    a = alpha_hat.reshape(-1, 1).contiguous()
    Abar = (0.5 * Ainv).contiguous()
    engine.dgemm(a, a, trans_b=True, alpha=-0.5, beta=1.0, C=Abar)
    return ski_adjoint_from(metric, hyp, Abar)


def ski_adjoint_from(metric, hyp: List, Abar: torch.Tensor):
    """Map an adjoint Abar of the SKI matrix A = W K_zz W^T + noise I to (hyp adjoint, noise adjoint): K_zz's
    is W^T Abar W (symmetrised for the kernel VJP), the noise's tr Abar."""
    import numpy as np
    from .StructuredKernelInterpolation import get_weight_matrix
    di = metric.data_input
    n, m = int(di.n_train), int(di.n_inducting_train)
    idx = np.linspace(start=0, stop=n, num=m, endpoint=False, dtype=int)
    z = di.get_inducting_x_train(torch.as_tensor(idx, dtype=torch.int64))
    Wm = get_weight_matrix(di)
    kbar = engine.dgemm(engine.dgemm(Wm, Abar.contiguous(), trans_a=True), Wm)
    gh, _ = engine.kernel_vjp(metric.covariance_matrix.kernel, hyp, z, z, G=(kbar + kbar.T).contiguous())
    return 0.5 * gh, torch.trace(Abar)
