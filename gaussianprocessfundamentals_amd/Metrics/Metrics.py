"""Metric framework (gpbasics/Metrics/Metrics.py:17-154) on the device.

The reference binds ``get_alpha`` / ``get_log_determinant`` per numerical handling
(Metrics.py:82-107); the same binding happens here:

  CHOLESKY_BASED (default)   alpha = L^-T L^-1 y, logdet = 2 sum log diag L     (:138-139, :152-154)
  STRICT_INVERSE             alpha = inv(K) y: K^-1 from the identity-augmented factorisation,
                             one device GEMV; logdet = slogdet(K)                (:132-133, :148-149)
  PSEUDO_INVERSE             alpha = pinv(K) y: inv(K) y for a positive-definite K; otherwise the
                             eigendecomposition (gpk_syevd) with tf.linalg.pinv's cutoff (:135-136)
  LINEAR_CONJUGATE_GRADIENT  alpha = linear_cg(K, y, 0) (device GEMV per iteration) (:141-144)

slogdet(K)[1] is log|det K| = 2 sum log diag L for a positive-definite K (the device Cholesky) and
sum log|lam_i| from the eigenvalues (gpk_syevd) otherwise; STRICT_INVERSE of an indefinite nonsingular K
(LU in the reference) is V diag(1/lam) V^T.  The eigendecomposition fallback takes n <= 46340 (gpk_syevd).
Subset-of-data approximations (SOD_GRID, SOD_RANDOM) evaluate the exact path on the subset
(:60-68).  Matrix approximations (:77-126) swap get_covariance_matrix / get_log_determinant:

  BASIC_NYSTROEM, SKC_LOWER_BOUND  covariance K_hat + noise I, log-det of the Nystroem determinant
                                   (Statistics/Nystroem_K.py); CHOLESKY_BASED keeps the exact alpha
                                   because get_alpha_cholesky reads the holistic covariance matrix
  SKC_UPPER_BOUND                  exact covariance, Nystroem log-det (Metrics/SkcLogLikelihood.py)
  SKI                              covariance W K_mm W^T + noise I (Metrics/StructuredKernelInterpolation.py);
                                   with CHOLESKY_BASED nothing reads it, so the metric is the exact one

The STRICT / PSEUDO inverse and slogdet of an approximate covariance matrix factor it through the
augmented Cholesky (engine.DenseFactorization); linear CG multiplies it with gpk_gemv.
"""
from __future__ import annotations

from enum import Enum
from typing import List

import torch

from .. import global_parameters as global_param
from . import MatrixHandlingTypes as mht

global_param.ensure_init()


class MetricType(Enum):
    LL = 1
    MSE = 5
    BIC = 6
    blockwise_LL = 10
    blockwise_MSE = 50
    blockwise_BIC = 60


class AbstractMetric:
    """Metrics are given in minimise convention (Metrics.py:27)."""

    def get_metric(self, hyper_parameter: List, noise, indices=None) -> torch.Tensor:
        raise NotImplementedError

    def get_gradients(self, hyper_parameter: List, noise, reset: bool = True) -> torch.Tensor:
        """Metrics.py:31: an abstract stub in the reference (``pass``).  LogLikelihood overrides it with the
        device gradient (get_metric_and_gradient); metrics without one say so."""
        raise NotImplementedError("%s provides no gradient; LogLikelihood.get_gradients does"
                                  % type(self).__name__)


class Metric(AbstractMetric):
    def __init__(self, data_input, covariance_matrix, metric_type: MetricType, local_approx,
                 numerical_matrix_handling, subset_size: int = None):
        self.covariance_matrix = covariance_matrix
        self.local_approx = local_approx
        self.numerical_matrix_handling = numerical_matrix_handling
        self.subset_size = subset_size
        if self.local_approx is not mht.MatrixApproximations.NONE and self.subset_size is None:
            self.subset_size = int(data_input.n_train * global_param.p_nystroem_ratio)     # :54-55
        if self.subset_size is not None and self.subset_size >= data_input.n_train:
            self.local_approx = mht.MatrixApproximations.NONE                              # :57-58
        if isinstance(self.local_approx, mht.SubsetOfDataApproaches):                      # :60-66
            self.data_input = data_input.get_subset(subset_size=self.subset_size,
                                                    subset_of_data_approach=self.local_approx)
        else:
            self.data_input = data_input
        A = mht.MatrixApproximations
        if self.local_approx is not A.NONE:                                                # :70-72
            self.data_input.n_inducting_train = self.subset_size
            self.data_input.n_inducting_test = self.data_input.n_test / self.data_input.n_train * self.subset_size
        self.covariance_matrix.set_data_input(self.data_input)
        self.type = metric_type
        if self.local_approx in (A.SKC_LOWER_BOUND, A.BASIC_NYSTROEM, A.SKC_UPPER_BOUND):   # :77-80
            self.nystroem_matrix = self.get_nystroem_handler()
        self.last_covariance_matrix = None
        self._approx_fact = None
        h = mht.NumericalMatrixHandlingType
        if numerical_matrix_handling is h.PSEUDO_INVERSE:                                  # :82-94
            self.get_alpha, self.get_log_determinant = self.get_alpha_pseudo_inverse, self.get_log_determinant_slodget
        elif numerical_matrix_handling is h.CHOLESKY_BASED:
            self.get_alpha, self.get_log_determinant = self.get_alpha_cholesky, self.get_log_determinant_cholesky
        elif numerical_matrix_handling is h.LINEAR_CONJUGATE_GRADIENT:
            self.get_alpha, self.get_log_determinant = self.get_alpha_lcg, self.get_log_determinant_slodget
        else:
            self.get_alpha, self.get_log_determinant = self.get_alpha_strict_inverse, self.get_log_determinant_slodget
        if self.local_approx is A.SKC_UPPER_BOUND:                                         # :95-106
            self.get_covariance_matrix = self.get_default_covariance_matrix
            self.get_log_determinant = self.get_log_determinant_nystroem
        elif self.local_approx in (A.SKC_LOWER_BOUND, A.BASIC_NYSTROEM):
            self.get_covariance_matrix = self.get_nystroem_matrix
            self.get_log_determinant = self.get_log_determinant_nystroem
        elif self.local_approx is A.SKI:
            self.get_covariance_matrix = self.get_ski_matrix
        else:
            self.get_covariance_matrix = self.get_default_covariance_matrix

    def get_nystroem_handler(self):
        from ..Statistics.Nystroem_K import NystroemMatrix
        nyk = NystroemMatrix(self.covariance_matrix)
        nyk.set_data_input(self.data_input)
        return nyk

    def _approximate(self) -> bool:
        """True when get_covariance_matrix is an approximation (not the holistic K + noise I)."""
        return self.get_covariance_matrix.__func__ is not Metric.get_default_covariance_matrix

    def get_nystroem_matrix(self, hyper_parameter: List, noise, indices=None):
        """K_hat + noise I (Metrics.py:116-119)."""
        if self.last_covariance_matrix is None:
            self._require_plain()
            self.last_covariance_matrix = self.nystroem_matrix.get_K_approx_noised(hyper_parameter, noise, indices)
            self._approx_fact = None
        return self.last_covariance_matrix

    def get_ski_matrix(self, hyper_parameter: List, noise, indices=None):
        """W K_mm W^T + noise I (Metrics.py:121-125)."""
        if self.last_covariance_matrix is None:
            from .StructuredKernelInterpolation import get_ski_matrix
            self._require_plain()
            self.last_covariance_matrix = get_ski_matrix(hyper_parameter, self.data_input,
                                                         self.covariance_matrix.kernel, noise)
            self._approx_fact = None
        return self.last_covariance_matrix

    def get_log_determinant_nystroem(self, hyper_parameter: List, noise, indices=None):
        """get_K_approx_det (Metrics.py:149-150): cached by the Nystroem handler (quirk kept)."""
        return self.nystroem_matrix.get_K_approx_det(hyper_parameter, noise, indices)

    def _approx_factorization(self, hyper_parameter: List, noise, indices=None):
        """Identity-augmented dense factorisation of the approximate covariance matrix (its inverse,
        log-determinant and info), cached until the matrix is rebuilt."""
        from .. import engine
        A = self.get_covariance_matrix(hyper_parameter, noise, indices).contiguous()
        if self._approx_fact is None:
            self._approx_fact = engine.DenseFactorization(A.shape[0], inverse=True).run(A, 0.0)
        return self._approx_fact

    def get_default_covariance_matrix(self, hyper_parameter: List, noise, indices=None):
        if self.last_covariance_matrix is None:
            self.last_covariance_matrix = self.covariance_matrix.get_K_noised(hyper_parameter, noise)
        return self.last_covariance_matrix

    def _y(self, y):
        return (self.data_input.get_detrended_y_train() if y is None else y).reshape(-1, 1).to(torch.float64)

    def _require_plain(self):
        if self.data_input.data_x_train.dim() == 3:
            raise NotImplementedError("numerical handling %s is provided for DataInput, not BatchDataInput"
                                      % self.numerical_matrix_handling)

    def get_alpha_cholesky(self, hyper_parameter: List, noise, y=None, indices=None):
        """get_alpha_cholesky (Metrics.py:138-139)."""
        return self.covariance_matrix.get_L_alpha(hyper_parameter, noise)

    def get_alpha_strict_inverse(self, hyper_parameter: List, noise, y=None, indices=None):
        """inv(K) y (Metrics.py:132-133): the explicit inverse, then one device GEMV."""
        from .. import engine
        self._require_plain()
        if not self._positive_definite(hyper_parameter, noise, indices):
            # tf.linalg.inv is LU-based: an indefinite but nonsingular K is inverted, a singular one raises
            lam, V = self._eigen(hyper_parameter, noise, indices)
            if bool((lam == 0).any()):
                raise engine.CholeskyError("inv: the covariance matrix is singular")
            U, _ = engine.pinv_factor(lam, V, 0, rcond=0.0)
            return engine.dgemm(U, engine.dgemm(V, self._y(y), trans_a=True))
        if self._approximate():
            f = self._approx_factorization(hyper_parameter, noise, indices)
            return engine.gemv(f.k_inv(0).contiguous(), self._y(y))
        return engine.gemv(self.covariance_matrix.get_K_inv(hyper_parameter, noise).contiguous(), self._y(y))

    # largest n for the eigendecomposition fallback of a matrix that is not positive definite (gpk_syevd's cap: its
    # kernels index the m x m matrix with 32-bit products, m^2 < 2^31; n = 46340 is 17 GB per m x m buffer)
    EIGEN_FALLBACK_MAX_N = 46340

    def _positive_definite(self, hyper_parameter: List, noise, indices=None) -> bool:
        f = (self._approx_factorization(hyper_parameter, noise, indices) if self._approximate()
             else self.covariance_matrix.factorization(hyper_parameter, noise))
        return int(f.info.abs().max()) == 0

    def _eigen(self, hyper_parameter: List, noise, indices=None):
        """Eigendecomposition (gpk_syevd) of the covariance matrix the handling works on, for the
        handlings' non-positive-definite cases; cached with that matrix."""
        from .. import engine
        K = self.get_covariance_matrix(hyper_parameter, noise, indices)
        if getattr(self, "_eig_src", None) is not K:
            n = K.shape[0]
            if n > self.EIGEN_FALLBACK_MAX_N:
                raise NotImplementedError("the covariance matrix is not positive definite and n = %d exceeds the "
                                          "eigendecomposition fallback (n <= %d)" % (n, self.EIGEN_FALLBACK_MAX_N))
            lam, V, _ = engine.eigh(K.contiguous())
            self._eig, self._eig_src = (lam, V), K
        return self._eig

    def get_alpha_pseudo_inverse(self, hyper_parameter: List, noise, y=None, indices=None):
        """pinv(K) y (Metrics.py:135-136): inv(K) y for a positive-definite K; otherwise the
        eigendecomposition route of tf.linalg.pinv (gpk_syevd, cutoff 10 n eps max|lam|)."""
        from .. import engine
        self._require_plain()
        if self._positive_definite(hyper_parameter, noise, indices):
            return self.get_alpha_strict_inverse(hyper_parameter, noise, y, indices)
        lam, V = self._eigen(hyper_parameter, noise, indices)
        U, _ = engine.pinv_factor(lam, V, 0)
        return engine.dgemm(U, engine.dgemm(V, self._y(y), trans_a=True))

    def get_alpha_lcg(self, hyper_parameter: List, noise, y=None, indices=None):
        """linear_cg(K, y, 0) (Metrics.py:141-144; Auxiliary/LinearConjugateGradients.py)."""
        from ..Auxiliary.LinearConjugateGradients import linear_cg
        self._require_plain()
        yv = self._y(y)
        return linear_cg(self.get_covariance_matrix(hyper_parameter, noise, indices).contiguous(), yv,
                         torch.zeros_like(yv))

    def get_log_determinant_cholesky(self, hyper_parameter: List, noise, indices=None):
        """2 * reduce_sum(log(diag L)) (Metrics.py:152-154); summed over the whole batch for
        BatchDataInput, exactly like the reference's axis-free reduce_sum (quirk Q7)."""
        f = self.covariance_matrix.factorization(hyper_parameter, noise)
        return torch.sum(f.logdet())

    def get_log_determinant_slodget(self, hyper_parameter: List, noise, indices=None):
        """slogdet(K)[1] = log|det K| (Metrics.py:146-147): 2 sum log diag L from the device Cholesky
        for a positive-definite K, sum log|lam_i| from the eigenvalues otherwise (-inf if singular)."""
        self._require_plain()
        f = (self._approx_factorization(hyper_parameter, noise, indices) if self._approximate()
             else self.covariance_matrix.factorization(hyper_parameter, noise))
        if int(f.info.abs().max()) == 0:
            return torch.sum(f.logdet())
        lam, _ = self._eigen(hyper_parameter, noise, indices)
        return torch.sum(torch.log(torch.abs(lam)))
