"""Mean squared error of the posterior mean on the test set (gpbasics/Metrics/MeanSquaredError.py:14-81).

``get_posterior_mu`` (mu = K_s^T alpha, :33-42) comes from ONE device factorisation of the
augmented matrix with the test points as extra rows; the blockwise form factors every segment
together in one ragged batch.  MSE = mean((mu - detrended y_test)^2).
"""
from __future__ import annotations

from typing import List

import torch

from .. import engine
from .. import global_parameters as global_param
from ..Statistics.CovarianceMatrix import noise_vector
from .LogLikelihood import blockwise_hyper_parameter_offset
from .Metrics import AbstractMetric, Metric, MetricType

global_param.ensure_init()


class AbstractMSE(Metric):
    pass


def posterior_mu(kernel, hyper_parameter: List, noise, data_input) -> torch.Tensor:
    """mu = K_s^T alpha for one DataInput, [n_test] (MeanSquaredError.py:33-42)."""
    x, xt = data_input.data_x_train, data_input.data_x_test
    n, d, m = int(x.shape[0]), int(x.shape[1]), int(xt.shape[0])
    y = data_input.get_detrended_y_train().reshape(1, n).to(torch.float64).contiguous()
    f = engine.AugmentedFactorization(n, d, m, 1, global_param.p_dtype)
    kd = engine.kernel_descriptor(kernel, d)
    hyp = engine.pack_hyper_parameter(hyper_parameter, kd.n_hyp)
    f.run(kd, hyp, 0, noise_vector(noise), 0, x.contiguous(), 0, y, 0, Xs=xt.contiguous(), xs_bstride=0)
    kernel._record_hyper_parameter(list(hyper_parameter))
    f.check_info()
    return f.posterior_mu(0).clone()


class MeanSquaredError(AbstractMSE):
    def __init__(self, data_input, covariance_matrix, aux_gp, local_approx, numerical_matrix_handling,
                 subset_size: int = None):
        super().__init__(data_input, covariance_matrix, MetricType.MSE, local_approx, numerical_matrix_handling,
                         subset_size)
        self.aux_gp = aux_gp

    def get_metric(self, hyper_parameter: List, noise, indices=None) -> torch.Tensor:
        self.aux_gp.reset()
        self.covariance_matrix.reset()
        mu = self.get_posterior_mu(hyper_parameter, noise, indices).reshape(-1, 1)
        yt = self.data_input.get_detrended_y_test().reshape(-1, 1).to(torch.float64)
        return torch.mean((mu - yt) ** 2)

    def get_posterior_mu(self, hyper_parameter: List, noise, indices=None):
        """K_s^T alpha (MeanSquaredError.py:33-42).  CHOLESKY_BASED: one augmented factorisation with
        the test rows; the other handlings: their alpha (Metrics.get_alpha) and one device GEMV."""
        from .. import engine
        from . import MatrixHandlingTypes as mht
        if self.numerical_matrix_handling is mht.NumericalMatrixHandlingType.CHOLESKY_BASED:
            return posterior_mu(self.covariance_matrix.kernel, hyper_parameter, noise, self.data_input)
        alpha = self.get_alpha(hyper_parameter, noise, None, indices)
        ks_t = self.covariance_matrix.get_K_s(hyper_parameter).transpose(0, 1).contiguous()
        return engine.gemv(ks_t, alpha.reshape(-1)).reshape(-1)


class BlockwiseMeanSquaredError(AbstractMetric):
    def __init__(self, _gp, local_approx, numerical_matrix_handling, subset_size: int = None):
        self.local_approx = local_approx
        self.numerical_matrix_handling = numerical_matrix_handling
        self.subset_size = subset_size
        self.aux_gp = _gp.aux
        self._gp = _gp
        self.data_input = _gp.data_input

    def get_metric(self, hyper_parameter: List, noise, indices=None) -> torch.Tensor:
        """Per-segment posterior means (hyperparameters sliced from offset 0, the reference's
        quirk, see blockwise_hyper_parameter_offset) against the segments' detrended test targets,
        both concatenated in segment order (MeanSquaredError.py:63-81)."""
        from ..Statistics.Auxiliary import segment_posterior_mu
        index = blockwise_hyper_parameter_offset(self._gp)
        kernels, slices, dis = [], [], []
        for sub in self._gp.constituent_gps:
            kern = sub.covariance_matrix.kernel
            nh = kern.get_number_of_hyper_parameter()
            kernels.append(kern)
            slices.append(list(hyper_parameter[index:index + nh]))
            dis.append(sub.data_input)
            index += nh
        mu = segment_posterior_mu(kernels, slices, dis, noise).reshape(-1, 1)
        yt = torch.cat([d.get_detrended_y_test().reshape(-1, 1).to(torch.float64) for d in dis], dim=0)
        return torch.mean((mu - yt) ** 2)
