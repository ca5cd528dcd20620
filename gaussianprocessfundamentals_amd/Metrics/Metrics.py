"""Metric framework (gpbasics/Metrics/Metrics.py:17-154), CHOLESKY_BASED strategy on the device.

The reference binds ``get_alpha`` / ``get_log_determinant`` per numerical handling
(Metrics.py:82-107).  The device engine implements the default pair, CHOLESKY_BASED with no
approximation (Metrics.py:85-87, :138-139, :152-154); the other strategies raise
``NotImplementedError`` naming SURVEY §8f.
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
        raise NotImplementedError("LML gradients are SURVEY §8f 'next'")


class Metric(AbstractMetric):
    def __init__(self, data_input, covariance_matrix, metric_type: MetricType, local_approx,
                 numerical_matrix_handling, subset_size: int = None):
        if local_approx is not mht.MatrixApproximations.NONE and not (
                subset_size is not None and subset_size >= data_input.n_train):
            raise NotImplementedError("approximation %s is SURVEY §8f 'next'; the device engine is exact" % local_approx)
        if numerical_matrix_handling is not mht.NumericalMatrixHandlingType.CHOLESKY_BASED:
            raise NotImplementedError("numerical handling %s is SURVEY §8f 'next'; use CHOLESKY_BASED"
                                      % numerical_matrix_handling)
        self.covariance_matrix = covariance_matrix
        self.local_approx = mht.MatrixApproximations.NONE
        self.numerical_matrix_handling = numerical_matrix_handling
        self.subset_size = subset_size
        self.data_input = data_input
        self.covariance_matrix.set_data_input(self.data_input)
        self.type = metric_type
        self.last_covariance_matrix = None

    def get_covariance_matrix(self, hyper_parameter: List, noise, indices=None):
        if self.last_covariance_matrix is None:
            self.last_covariance_matrix = self.covariance_matrix.get_K_noised(hyper_parameter, noise)
        return self.last_covariance_matrix

    def get_alpha(self, hyper_parameter: List, noise, y=None, indices=None):
        """get_alpha_cholesky (Metrics.py:138-139)."""
        return self.covariance_matrix.get_L_alpha(hyper_parameter, noise)

    def get_log_determinant(self, hyper_parameter: List, noise, indices=None):
        """2 * reduce_sum(log(diag L)) (Metrics.py:152-154); summed over the whole batch for
        BatchDataInput, exactly like the reference's axis-free reduce_sum (quirk Q7)."""
        f = self.covariance_matrix.factorization(hyper_parameter, noise)
        return torch.sum(f.logdet())
