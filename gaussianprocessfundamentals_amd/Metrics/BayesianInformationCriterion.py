"""Bayesian information criterion (gpbasics/Metrics/BayesianInformationCriterion.py:14-63).

BIC = -2 LML + |theta| log n_train, in the minimise convention: LML = -(the log-likelihood
metric), so BIC = 2 * (-LML metric) + n_hyp * log(n).  The log-likelihood comes from the device
factorisation (LogLikelihood / BlockwiseLogLikelihood); the rest is a scalar epilogue.
"""
from __future__ import annotations

import math
from typing import List

import torch

from .. import global_parameters as global_param
from .LogLikelihood import AbstractLogLikelihood, BlockwiseLogLikelihood
from .Metrics import AbstractMetric, Metric, MetricType

global_param.ensure_init()


class AbstractBIC(Metric):
    pass


def _bic(neg_ll: torch.Tensor, n_hyp: int, n_train: int) -> torch.Tensor:
    # -2 * log_likelihood + |M| * log n (BayesianInformationCriterion.py:27-38)
    log_likelihood = -1.0 * neg_ll
    return (-2.0 * log_likelihood) + float(n_hyp) * math.log(float(n_train))


class BIC(AbstractBIC):
    def __init__(self, data_input, covariance_matrix, log_likelihood: AbstractLogLikelihood):
        super().__init__(data_input, covariance_matrix, MetricType.BIC, log_likelihood.local_approx,
                         log_likelihood.numerical_matrix_handling, log_likelihood.subset_size)
        self.log_likelihood = log_likelihood

    def get_metric(self, hyper_parameter: List, noise, indices=None, reset: bool = True) -> torch.Tensor:
        nl = self.log_likelihood.get_metric(hyper_parameter, noise, indices, reset)
        return _bic(nl, self.covariance_matrix.kernel.get_number_of_hyper_parameter(), self.data_input.n_train)


class BlockwiseBIC(AbstractMetric):
    def __init__(self, _gp, local_approx, numerical_matrix_handling, subset_size: int = None):
        self.local_approx = local_approx
        self.numerical_matrix_handling = numerical_matrix_handling
        self.subset_size = subset_size
        self._gp = _gp

    def get_metric(self, hyper_parameter: List, noise, indices=None) -> torch.Tensor:
        ll = BlockwiseLogLikelihood(self._gp, self.local_approx, self.numerical_matrix_handling, self.subset_size)
        nl = ll.get_metric(hyper_parameter, noise, indices)
        return _bic(nl, self._gp.covariance_matrix.kernel.get_number_of_hyper_parameter(), self._gp.data_input.n_train)
