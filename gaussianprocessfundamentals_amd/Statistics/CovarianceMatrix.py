"""Covariance-matrix plugin (gpbasics/Statistics/CovarianceMatrix.py:15-286) on the MI355X engine.

``HolisticCovarianceMatrix`` keeps the reference's contract: it owns and memoises every matrix it
hands out until :meth:`reset` / :meth:`set_data_input` (CovarianceMatrix.py:37-62); callers reset
when hyperparameters change.  Underneath, the factorisation is ONE augmented Cholesky in libgpk
(include/gpk.h): L, z = L^-1 y, the log-determinant and the data-fit term come out of the same
launches, and alpha = L^-T z is a device triangular solve.  Nothing is computed on the host.

Errors: "No Data Input given" (CovarianceMatrix.py:195); a noise that is not rank-0 raises
(:198-206); a matrix that is not positive definite raises ``CholeskyError`` when the factor is
requested (TensorFlow raises InvalidArgumentError at :250).
"""
from __future__ import annotations

from enum import Enum
from typing import List, Optional

import torch

from .. import engine
from .. import global_parameters as global_param

global_param.ensure_init()


class CovarianceMatrixType(Enum):
    HOLISTIC = 0
    SEGMENTED = 1
    GLOBALIZED_SEGMENTED = 2


def _is_scalar(noise) -> bool:
    return noise is not None and torch.as_tensor(noise).shape == torch.Size([])


def noise_vector(noise) -> torch.Tensor:
    """Rank-0 noise as a 1-element fp64 device vector (no host round trip for device tensors)."""
    t = noise if isinstance(noise, torch.Tensor) else torch.tensor(float(noise), dtype=torch.float64)
    return t.detach().to(device=engine.device(), dtype=torch.float64).reshape(1)


class CovarianceMatrix:
    _CACHES = ("K", "noised_K", "K_ss", "noised_K_ss", "L_K_ss", "L_K", "L_inv_K", "K_inv", "K_s", "L_alpha")

    def __init__(self, matrix_type: CovarianceMatrixType, kernel):
        self.kernel = kernel
        self.data_input = None
        self.type = matrix_type
        for c in self._CACHES:
            setattr(self, c, None)

    def reset(self):
        """Drop every memoised matrix (CovarianceMatrix.py:37-53)."""
        for c in self._CACHES:
            setattr(self, c, None)

    def set_data_input(self, data_input):
        self.data_input = data_input
        self.reset()

    def is_segmented(self) -> bool:
        return self.type == CovarianceMatrixType.SEGMENTED


class HolisticCovarianceMatrix(CovarianceMatrix):
    """The usual, unapproximated covariance matrix of a GP (CovarianceMatrix.py:178-286)."""

    def __init__(self, kernel):
        super().__init__(CovarianceMatrixType.HOLISTIC, kernel)
        self._fact: Optional[engine.AugmentedFactorization] = None   # y only (the LML)
        self._fact_key = None
        self._inv_fact: Optional[engine.AugmentedFactorization] = None  # identity rows (inverses)

    def reset(self):
        super().reset()
        self._fact_key = None
        self._inv_fact = None

    # -- helpers --------------------------------------------------------------------------------
    def _require_data(self):
        if self.data_input is None:
            raise Exception("No Data Input given")

    def _xy(self):
        di = self.data_input
        y = di.get_detrended_y_train()
        return di.data_x_train, y

    def _shape(self, x):
        if x.dim() == 3:
            return int(x.shape[0]), int(x.shape[1]), int(x.shape[2])
        return 1, int(x.shape[0]), int(x.shape[1])

    def _run(self, fact, hyper_parameter, noise, E=None):
        x, y = self._xy()
        batch, n, d = self._shape(x)
        kd = engine.kernel_descriptor(self.kernel, d)
        hyp = engine.pack_hyper_parameter(hyper_parameter, kd.n_hyp)
        x = x.contiguous()
        yv = y.reshape(batch, n).to(torch.float64).contiguous()
        fact.run(kd, hyp, 0, noise_vector(noise), 0, x, n * d if batch > 1 else 0, yv, n if batch > 1 else 0,
                 E=E, e_bstride=0)
        self.kernel._record_hyper_parameter(list(hyper_parameter))
        return fact

    def factorization(self, hyper_parameter: List, noise) -> engine.AugmentedFactorization:
        """The augmented factorisation carrying y (memoised until reset)."""
        self._require_data()
        if not _is_scalar(noise):
            raise Exception("No Data Input given or Noise unspecified")
        if self._fact_key is None:
            x, _ = self._xy()
            batch, n, d = self._shape(x)
            shape = (batch, n, d, global_param.p_dtype)
            if self._fact is None or self._fact.shape_key != shape:
                f = engine.AugmentedFactorization(n, d, 0, batch, global_param.p_dtype)
                f.shape_key = shape
                self._fact = f
            self._run(self._fact, hyper_parameter, noise)
            self._fact_key = True
        return self._fact

    # -- reference surface ------------------------------------------------------------------------
    def get_K(self, hyper_parameter: List) -> torch.Tensor:
        self._require_data()
        if self.K is None:
            x = self.data_input.data_x_train
            if x.dim() == 3:
                self.K = torch.stack([self.kernel.get_tf_tensor(hyper_parameter, xb, xb) for xb in x])
            else:
                self.K = self.kernel.get_tf_tensor(hyper_parameter, x, x)
        return self.K

    def get_K_noised(self, hyper_parameter: List, noise) -> torch.Tensor:
        if _is_scalar(noise) and self.data_input is not None:
            if self.noised_K is None:
                x = self.data_input.data_x_train
                nv = float(torch.as_tensor(noise))
                if x.dim() == 3:
                    self.noised_K = torch.stack([engine.kernel_matrix(self.kernel, hyper_parameter, xb, xb, nv) for xb in x])
                else:
                    self.noised_K = engine.kernel_matrix(self.kernel, hyper_parameter, x, x, nv)
            return self.noised_K
        raise Exception("No Data Input given or Noise unspecified")

    def get_L_K(self, hyper_parameter: List, noise) -> torch.Tensor:
        """Lower Cholesky factor of K + noise I (CovarianceMatrix.py:247-254)."""
        self._require_data()
        if self.L_K is None:
            f = self.factorization(hyper_parameter, noise)
            f.check_info()
            if f.batch == 1 and self.data_input.data_x_train.dim() == 2:
                self.L_K = f.cholesky(0).to(torch.float64)
            else:
                self.L_K = torch.stack([f.cholesky(b).to(torch.float64) for b in range(f.batch)])
        return self.L_K

    def get_L_alpha(self, hyper_parameter: List, noise) -> torch.Tensor:
        """alpha = L^-T (L^-1 y) as [N, 1] (CovarianceMatrix.py:256-265)."""
        self._require_data()
        if self.L_alpha is None:
            f = self.factorization(hyper_parameter, noise)
            f.check_info()
            if f.batch == 1 and self.data_input.data_x_train.dim() == 2:
                self.L_alpha = f.alpha(0).reshape(-1, 1)
            else:
                self.L_alpha = torch.stack([f.alpha(b).reshape(-1, 1) for b in range(f.batch)])
        return self.L_alpha

    def _inverse_factorization(self, hyper_parameter, noise):
        """Augment with identity rows: extra rows -> L^-T, corner -> -K^-1 (one factorisation)."""
        self._require_data()
        if self.data_input.data_x_train.dim() == 3:
            raise NotImplementedError("explicit inverses are not provided for BatchDataInput")
        if self._inv_fact is None:
            self._inv_fact = self.inverse_factorization(hyper_parameter, noise, gradient=False)
            self._inv_fact.check_info()
        return self._inv_fact

    def inverse_factorization(self, hyper_parameter, noise, gradient: bool = True):
        """One factorisation with identity extra rows (engine.InverseFactorization): -LML, K^-1,
        L^-1, alpha and (gradient=True) d(-LML)/d(hyperparameters, noise) for every member of a
        DataInput (batch 1) or BatchDataInput (one member per batch entry).  Not memoised."""
        self._require_data()
        if not _is_scalar(noise):
            raise Exception("No Data Input given or Noise unspecified")
        x, y = self._xy()
        batch, n, d = self._shape(x)
        kd = engine.kernel_descriptor(self.kernel, d)
        hyp = engine.pack_hyper_parameter(hyper_parameter, kd.n_hyp)
        f = engine.InverseFactorization(n, d, batch, global_param.p_dtype)
        yv = y.reshape(batch, n).to(torch.float64).contiguous()
        f.run(kd, hyp, 0, noise_vector(noise), 0, x.contiguous(), n * d if batch > 1 else 0, yv,
              n if batch > 1 else 0, gradient=gradient)
        self.kernel._record_hyper_parameter(list(hyper_parameter))
        return f

    def get_L_inv_K(self, hyper_parameter: List, noise) -> torch.Tensor:
        """inv(L) (CovarianceMatrix.py:267-275), without an explicit inverse: the identity rows of
        the augmented matrix come out as L^-T."""
        if self.L_inv_K is None:
            f = self._inverse_factorization(hyper_parameter, noise)
            self.L_inv_K = f.l_inv(0).to(torch.float64).contiguous()
        return self.L_inv_K

    def get_K_inv(self, hyper_parameter: List, noise) -> torch.Tensor:
        """inv(K + noise I) (CovarianceMatrix.py:208-216) from the Schur complement corner."""
        if self.K_inv is None:
            f = self._inverse_factorization(hyper_parameter, noise)
            self.K_inv = f.k_inv(0).to(torch.float64)
        return self.K_inv

    def get_K_s(self, hyper_parameter: List) -> torch.Tensor:
        """k(X_train, X_test) [N, M] (CovarianceMatrix.py:277-286)."""
        self._require_data()
        if self.K_s is None:
            di = self.data_input
            self.K_s = self.kernel.get_tf_tensor(hyper_parameter, di.data_x_train, di.data_x_test)
        return self.K_s

    def get_K_ss(self, hyper_parameter: List) -> torch.Tensor:
        """k(X_test, X_test) without noise (CovarianceMatrix.py:218-225)."""
        self._require_data()
        if self.K_ss is None:
            xt = self.data_input.data_x_test
            self.K_ss = self.kernel.get_tf_tensor(hyper_parameter, xt, xt)
        return self.K_ss

    def get_K_ss_noised(self, hyper_parameter: List, noise) -> torch.Tensor:
        if _is_scalar(noise) and self.data_input is not None:
            if self.noised_K_ss is None:
                xt = self.data_input.data_x_test
                self.noised_K_ss = engine.kernel_matrix(self.kernel, hyper_parameter, xt, xt, float(torch.as_tensor(noise)))
            return self.noised_K_ss
        raise Exception("No Data Input given or noise unspecified")

    def get_L_K_ss(self, hyper_parameter: List, noise) -> torch.Tensor:
        """Cholesky of K_ss + noise I (CovarianceMatrix.py:238-245)."""
        self._require_data()
        if self.L_K_ss is None:
            xt = self.data_input.data_x_test
            m, d = int(xt.shape[0]), int(xt.shape[1])
            f = engine.AugmentedFactorization(m, d, 0, 1, global_param.p_dtype)
            kd = engine.kernel_descriptor(self.kernel, d)
            hyp = engine.pack_hyper_parameter(hyper_parameter, kd.n_hyp)
            zeros = torch.zeros(1, m, dtype=torch.float64, device=engine.device())
            f.run(kd, hyp, 0, noise_vector(noise), 0, xt.contiguous(), 0, zeros, 0)
            f.check_info()
            self.L_K_ss = f.cholesky(0).to(torch.float64)
        return self.L_K_ss
