"""Negative log marginal likelihood (gpbasics/Metrics/LogLikelihood.py:15-65) on the device.

``get_metric`` returns -LML (minimise convention), a [1, 1] fp64 tensor for a DataInput and a
scalar for a BatchDataInput, as the reference does.  One augmented factorisation in libgpk
(``gpk_assemble`` + ``gpk_potrf_aug`` + ``gpk_finalize``) produces the data-fit term y^T alpha
(= z^T z with z = L^-1 y) and the log-determinant; assembling

    ll = (-1/2 y^T alpha - 1/2 logdet) - 1/2 N log(2 pi)        (LogLikelihood.py:39-49)

happens on the device as well.  Batch quirk (Q7): the data fit is averaged by
p_batch_metric_aggregator while the log-determinant is summed over the batch
(LogLikelihood.py:62-63 with Metrics.py:153-154).
"""
from __future__ import annotations

import math
from typing import List

import torch

from .. import global_parameters as global_param
from . import MatrixHandlingTypes as mht
from .Metrics import AbstractMetric, Metric, MetricType

global_param.ensure_init()

LOG_2PI = math.log(2.0 * math.pi)


class AbstractLogLikelihood(Metric):
    def get_metric(self, hyper_parameter: List, noise, indices=None, reset: bool = True) -> torch.Tensor:
        raise NotImplementedError


class LogLikelihood(AbstractLogLikelihood):
    def __init__(self, data_input, covariance_matrix, local_approx, numerical_matrix_handling,
                 subset_size: int = None):
        super().__init__(data_input, covariance_matrix, MetricType.LL, local_approx,
                         numerical_matrix_handling, subset_size)
        if local_approx is mht.MatrixApproximations.SKC_UPPER_BOUND:
            raise Exception("SKC Upper Bound cannot be handled via default likelihood class")

    def get_metric(self, hyper_parameter: List, noise, indices=None, reset: bool = True) -> torch.Tensor:
        if reset:
            self.covariance_matrix.reset()
            self.last_covariance_matrix = None
        f = self.covariance_matrix.factorization(hyper_parameter, noise)
        if self.data_input.data_x_train.dim() == 3:
            n = float(self.data_input.n_train)
            logdet_total = torch.sum(f.logdet())
            ll = (-0.5 * f.fit() + -0.5 * logdet_total) + (-0.5 * (n * LOG_2PI))
            ll = torch.where(f.info == 0, ll, torch.full_like(ll, -math.inf))
            agg = global_param.p_batch_metric_aggregator or torch.mean
            return -agg(ll)
        return f.nlml().reshape(1, 1)

    def get_metric_checked(self, hyper_parameter: List, noise, reset: bool = True) -> torch.Tensor:
        """get_metric that raises CholeskyError when K + noise I is not positive definite
        (the reference's TensorFlow raises from tf.linalg.cholesky); synchronises."""
        out = self.get_metric(hyper_parameter, noise, reset=reset)
        self.covariance_matrix.factorization(hyper_parameter, noise).check_info()
        return out


class BlockwiseLogLikelihood(AbstractMetric):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("blockwise likelihood is SURVEY §8f 'next' (variable-size batched potrf)")
