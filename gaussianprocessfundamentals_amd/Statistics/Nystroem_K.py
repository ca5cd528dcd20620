"""Nystroem approximation of the covariance matrix (gpbasics/Statistics/Nystroem_K.py:11-108) on
the device.

    K_hat        = (K_nm pinv(K_mm)) K_nm^T                               (:57-64)
    K_hat_noised = K_hat + noise I                                       (:66-71)
    det          = (n - m) log(noise) + slogdet(noise I_m + K_nm^T K_nm pinv(K_mm))[1]   (:92-108)

``indices`` are the inducing INPUTS (an [m, D] tensor), passed straight to the kernel as its second
argument exactly like the reference (:36-47; the fitters pass random points, Optimizer/Fitter.py:76-86).

Device mapping: the kernel blocks come from gpk_kernel_matrix; pinv(K_mm) is the tridiagonal eigendecomposition
(gpk_syevd, engine.eigh) with tf.linalg.pinv's cutoff (10 m eps max|lam|, gpk_pinv_factor) and one MFMA GEMM; the
products are gpk_dgemm.  The log-determinant uses a symmetric form.  With pinv(K_mm) = U S U^T, U = V diag(|lam|^-1/2)
over the kept eigenvalues, S = diag(sign lam) (+1 on the dropped ones) and G = K_nm U (Sylvester's determinant
identity; S^2 = I):

    slogdet(noise I_m + K_nm^T K_nm pinv(K_mm))[1] = log|det(noise S + G^T G)|.

For a kernel matrix K_mm (S = I) noise I + G^T G is positive definite and goes through the augmented Cholesky
(gpk_assemble_dense).  The reference's default L1 Matern / periodic forms give an INDEFINITE K_mm for D > 1
(DESIGN §2); TensorFlow's pinv + slogdet still return a value there, and so does this: noise S + G^T G is then a
symmetric indefinite matrix whose log|det| is the sum of log|eigenvalue| (gpk_syevd).

get_K_approx_inv returns (K_hat + noise I)^-1: from the dense factorisation for a positive-semidefinite K_mm, and for
an indefinite one by the reference's Woodbury form (:73-90) in the same symmetric terms,
(K_hat + noise I)^-1 = (I - G (noise S + G^T G)^-1 G^T) / noise -- equal to the reference's whenever its inner
matrix noise I + pinv(K_mm) K_nm^T K_nm is invertible (the same determinant up to the sign).

Caching follows the reference: K_approx_inv and K_approx_det are computed once and kept until
reset() / set_data_input() (Metric.get_metric(reset=True) does NOT reset them, :74, :93).
"""
from __future__ import annotations

import math
from typing import List

import torch

from .. import engine


class NystroemMatrix:
    def __init__(self, covariance_matrix):
        self.data_input = None
        self.covariance_matrix = covariance_matrix
        self.reset()

    def reset(self):
        self.Knm = None
        self.Kmm = None
        self.Kmm_pseudo_inv = None
        self.K_approx = None
        self.K_approx_noised = None
        self.K_approx_inv = None
        self.K_approx_det = None

    def set_data_input(self, data_input):
        self.data_input = data_input
        self.reset()

    @staticmethod
    def _inducing(indices) -> torch.Tensor:
        if indices is None:
            raise ValueError("the Nystroem approximation needs the inducing inputs (``indices``, [m, D])")
        z = engine.as_device_f64(indices)
        return z.reshape(-1, 1) if z.dim() == 1 else z

    def get_Knm(self, hyper_param: List, indices) -> torch.Tensor:
        self.Knm = self.covariance_matrix.kernel.get_tf_tensor(hyper_param, self.data_input.data_x_train,
                                                               self._inducing(indices))
        return self.Knm

    def get_Kmm(self, hyper_param: List, indices) -> torch.Tensor:
        z = self._inducing(indices)
        self.Kmm = self.covariance_matrix.kernel.get_tf_tensor(hyper_param, z, z)
        return self.Kmm

    def get_Kmm_pseudo_inv(self, hyper_parameter: List, indices) -> torch.Tensor:
        """tf.linalg.pinv(K_mm) (:49-55): tridiagonal eigendecomposition (gpk_syevd) + the reference's cutoff."""
        self.Kmm_pseudo_inv = engine.pinv_sym(self.get_Kmm(hyper_parameter, indices).contiguous())
        return self.Kmm_pseudo_inv

    def get_K_approx(self, hyper_parameter: List, indices) -> torch.Tensor:
        knm = self.get_Knm(hyper_parameter, indices).contiguous()
        pinv = self.get_Kmm_pseudo_inv(hyper_parameter, indices)
        self.K_approx = engine.dgemm(engine.dgemm(knm, pinv), knm, trans_b=True)
        return self.K_approx

    def get_K_approx_noised(self, hyper_parameter: List, noise, indices) -> torch.Tensor:
        self.get_K_approx(hyper_parameter, indices)
        self.K_approx_noised = engine.add_diagonal(self.K_approx.clone(), _noise_value(noise))
        return self.K_approx_noised

    def _signed_core(self, hyper_parameter: List, indices):
        """G = K_nm V diag(|lam|^-1/2) (kept eigenvalues of K_mm), the signs S of those eigenvalues (+1 on the
        dropped ones), G^T G and the number of kept negative eigenvalues (reads one count back)."""
        knm = self.get_Knm(hyper_parameter, indices).contiguous()
        kmm = self.get_Kmm(hyper_parameter, indices).contiguous()
        lam, V, _ = engine.eigh(kmm)
        U, sgn, n_neg, _ = signed_pinv_factor(lam, V)
        G = engine.dgemm(knm, U)
        return G, sgn, engine.dgemm(G, G, trans_a=True), n_neg

    def get_K_approx_inv(self, hyper_parameter: List, noise, indices) -> torch.Tensor:
        if self.K_approx_inv is None:
            nv = _noise_value(noise)
            G, sgn, GtG, n_neg = self._signed_core(hyper_parameter, indices)
            if n_neg == 0:
                # K_hat = K_nm U U^T K_nm^T = G G^T (S = I): no second kernel build and eigendecomposition
                a = engine.dgemm(G, G, trans_b=True)
                n = a.shape[0]
                f = engine.DenseFactorization(n, inverse=True).run(a, nv)
                f.check_info()
                self.K_approx_inv = f.k_inv(0).to(torch.float64)
            else:
                # Woodbury (:73-90): (I - G C^+ G^T) / noise, C = noise S + G^T G symmetric indefinite; the reference
                # takes tf.linalg.pinv of its inner matrix, so C^+ keeps pinv's cutoff (10 m eps max|lam|)
                C = GtG.clone()
                C.diagonal().add_(nv * sgn)
                Ci = sym_inverse(C, cutoff=True)
                out = engine.dgemm(engine.dgemm(G, Ci), G, trans_b=True, alpha=-1.0 / nv)
                self.K_approx_inv = engine.add_diagonal(out, 1.0 / nv)
        return self.K_approx_inv

    def get_K_approx_det(self, hyper_parameter: List, noise, indices) -> torch.Tensor:
        if self.K_approx_det is None:
            n = int(self.data_input.n_train)
            m = int(self.data_input.n_inducting_train)
            z = self._inducing(indices)
            if z.shape[0] != m:
                raise ValueError("%d inducing inputs given, n_inducting_train is %d (the reference's "
                                 "noise * eye(m) would not conform)" % (z.shape[0], m))
            nv = _noise_value(noise)
            _, sgn, GtG, n_neg = self._signed_core(hyper_parameter, indices)
            if n_neg == 0:
                f = engine.DenseFactorization(m).run(GtG, nv)
                f.check_info()
                det2 = f.logdet()[0]
            else:
                C = GtG.clone()
                C.diagonal().add_(nv * sgn)
                lam_c, _ = engine.syevd(C)
                det2 = torch.sum(torch.log(torch.abs(lam_c)))   # slogdet(.)[1] = log|det|
            self.K_approx_det = (n - m) * math.log(nv) + det2
        return self.K_approx_det


def signed_pinv_factor(lam: torch.Tensor, V: torch.Tensor):
    """pinv(A) = U diag(sgn) U^T of a symmetric A = V diag(lam) V^T with tf.linalg.pinv's cutoff: U = V diag(|lam|^-1/2)
    over the kept eigenvalues (gpk_pinv_factor mode 2), sgn = sign(lam) there and +1 on the dropped ones.  Returns
    (U, sgn, number of kept negative eigenvalues, mu = |lam|^-1/2 or 0) -- the count is read back (one small copy)."""
    U, _, mu = engine.pinv_factor(lam, V, 2, return_mu=True)
    sgn = torch.where((mu > 0) & (lam < 0), -torch.ones_like(lam), torch.ones_like(lam))
    return U, sgn, int((sgn < 0).sum()), mu


def sym_inverse(C: torch.Tensor, cutoff: bool = False) -> torch.Tensor:
    """Inverse of a symmetric (possibly indefinite) device matrix: V diag(1/lam) V^T from gpk_syevd, on the MFMA
    GEMM.  cutoff=False: every eigenvalue (the true inverse, e.g. d log|det C| / dC); cutoff=True: tf.linalg.pinv's
    (eigenvalues with |lam| <= 10 m eps max|lam| dropped), as the reference's pinv of the Woodbury inner matrix."""
    lam, V = engine.syevd(C.contiguous())
    U, _ = engine.pinv_factor(lam, V, 0) if cutoff else engine.pinv_factor(lam, V, 0, rcond=0.0)
    return engine.dgemm(U, V, trans_b=True)


def _noise_value(noise) -> float:
    t = noise if isinstance(noise, torch.Tensor) else torch.as_tensor(noise, dtype=torch.float64)
    if t.numel() != 1:
        raise ValueError("noise must be a scalar")
    return float(t)
