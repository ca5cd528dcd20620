"""Nystroem approximation of the covariance matrix (gpbasics/Statistics/Nystroem_K.py:11-108) on
the device.

    K_hat        = (K_nm pinv(K_mm)) K_nm^T                               (:57-64)
    K_hat_noised = K_hat + noise I                                       (:66-71)
    det          = (n - m) log(noise) + slogdet(noise I_m + K_nm^T K_nm pinv(K_mm))[1]   (:92-108)

``indices`` are the inducing INPUTS (an [m, D] tensor), passed straight to the kernel as its second
argument exactly like the reference (:36-47; the fitters pass random points, Optimizer/Fitter.py:76-86).

Device mapping: the kernel blocks come from gpk_kernel_matrix; pinv(K_mm) is the Jacobi
eigendecomposition (gpk_syevj) with tf.linalg.pinv's cutoff (10 m eps max|lam|, gpk_pinv_factor) and
one MFMA GEMM; the products are gpk_dgemm.  The log-determinant uses the similar symmetric matrix:
with U = V diag(lam^-1/2) over the kept eigenvalues and G = K_nm U,

    slogdet(noise I_m + K_nm^T K_nm pinv(K_mm)) = logdet(noise I_m + G^T G),

which is positive definite and goes through the augmented Cholesky (gpk_assemble_dense); a kept
NEGATIVE eigenvalue of K_mm (an indefinite K_mm beyond the cutoff, which a kernel matrix does not
produce) raises NotImplementedError.  get_K_approx_inv returns (K_hat + noise I)^-1 from the dense
factorisation -- the reference's Woodbury form (:73-90) equals it whenever its inner matrix
noise I + pinv(K_mm) K_nm^T K_nm is invertible, which noise > 0 guarantees.

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
        """tf.linalg.pinv(K_mm) (:49-55): Jacobi eigendecomposition + the reference's cutoff."""
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

    def get_K_approx_inv(self, hyper_parameter: List, noise, indices) -> torch.Tensor:
        if self.K_approx_inv is None:
            a = self.get_K_approx(hyper_parameter, indices).contiguous()
            n = a.shape[0]
            f = engine.DenseFactorization(n, inverse=True).run(a, _noise_value(noise))
            f.check_info()
            self.K_approx_inv = f.k_inv(0).to(torch.float64)
        return self.K_approx_inv

    def get_K_approx_det(self, hyper_parameter: List, noise, indices) -> torch.Tensor:
        if self.K_approx_det is None:
            knm = self.get_Knm(hyper_parameter, indices).contiguous()
            kmm = self.get_Kmm(hyper_parameter, indices).contiguous()
            n = int(self.data_input.n_train)
            m = int(self.data_input.n_inducting_train)
            if kmm.shape[0] != m:
                raise ValueError("%d inducing inputs given, n_inducting_train is %d (the reference's "
                                 "noise * eye(m) would not conform)" % (kmm.shape[0], m))
            nv = _noise_value(noise)
            lam, V, _ = engine.eigh(kmm)
            U, rank = engine.pinv_factor(lam, V, 1)
            if int(rank.cpu()[0]) < 0:
                raise NotImplementedError("K_mm has a negative eigenvalue above the pinv cutoff")
            G = engine.dgemm(knm, U)
            S = engine.dgemm(G, G, trans_a=True)
            f = engine.DenseFactorization(m).run(S, nv)
            f.check_info()
            self.K_approx_det = (n - m) * math.log(nv) + f.logdet()[0]
        return self.K_approx_det


def _noise_value(noise) -> float:
    t = noise if isinstance(noise, torch.Tensor) else torch.as_tensor(noise, dtype=torch.float64)
    if t.numel() != 1:
        raise ValueError("noise must be a scalar")
    return float(t)
