"""Upper bound of the log likelihood with the Nystroem log-determinant
(gpbasics/Metrics/SkcLogLikelihood.py:14-69) on the device.

The reference minimises over alpha with one tfp.optimizer.VariationalSGD(batch_size=10,
total_num_examples=10) step started at alpha = 1 (:57-69), then returns

    optimizable(alpha) = 1/2 alpha^T K alpha - alpha^T y - 1/2 det_nystroem - n/2 log(2 pi)   (:26-52)

(K = the exact K + noise I, get_default_covariance_matrix).  Two details of that call decide the
result and are kept: ``minimize(opt, alpha)`` differentiates the TUPLE (value, gradient) that
tfp.math.value_and_gradient returns, so the step uses (K alpha - y) + K 1; and the optimizer is in
burn-in (iteration 0 < 25), so its per-coordinate learning rate 2 B / (N v) is capped at
burnin_max_learning_rate = 1e-6, with the moments started at zero (m = 0.05 g, v = 0.05 (g - m)^2).
TensorFlow Probability is not available here: the optimizer step is restated from its published
algorithm (Mandt et al. 2017) -- parity unpinned.  The metric never resets its caches (the
reference's get_metric has no reset): K and the Nystroem determinant of the first call are reused.
"""
from __future__ import annotations

import math
from typing import List

import torch

from .. import engine
from . import MatrixHandlingTypes as mht
from .Metrics import Metric, MetricType

LOG_2PI = math.log(2.0 * math.pi)


def variational_sgd_step(alpha: torch.Tensor, grad: torch.Tensor, batch_size: float = 10.0,
                         total_num_examples: float = 10.0, decay: float = 0.95,
                         max_learning_rate: float = 1e-6) -> torch.Tensor:
    """One VariationalSGD step from zero moments in burn-in (see the module docstring)."""
    m = (1.0 - decay) * grad
    v = (1.0 - decay) * (grad - m) ** 2
    lr = torch.where(v > 0, 2.0 * batch_size / (total_num_examples * v), torch.full_like(v, math.inf))
    lr = torch.clamp(lr, 0.0, max_learning_rate)
    return alpha - lr * grad


class LogLikelihoodUpperBound(Metric):
    def __init__(self, data_input, covariance_matrix, nystroem_k):
        super().__init__(data_input, covariance_matrix, MetricType.LL,
                         local_approx=mht.MatrixApproximations.SKC_UPPER_BOUND,
                         numerical_matrix_handling=mht.NumericalMatrixHandlingType.LINEAR_CONJUGATE_GRADIENT)
        self.nyK = nystroem_k
        self.hyper_parameter = None
        self.noise = None
        self.indices = None

    def optimizable(self, alpha: torch.Tensor) -> torch.Tensor:
        y = self.data_input.get_detrended_y_train().reshape(-1, 1).to(torch.float64)
        n = int(self.data_input.n_train)
        alpha = alpha.reshape(n, 1)
        K = self.get_covariance_matrix(self.hyper_parameter, self.noise, self.indices).contiguous()
        ka = engine.gemv(K, alpha)
        data_fit = 0.5 * torch.sum(alpha * ka) - torch.sum(alpha * y)
        det = self.nyK.get_K_approx_det(self.hyper_parameter, self.noise, self.indices)
        return data_fit + (-0.5 * det) + (-0.5 * n) * LOG_2PI

    def get_metric(self, hyper_parameter: List, noise, indices=None) -> torch.Tensor:
        self.hyper_parameter = hyper_parameter
        self.noise = noise
        self.indices = indices
        n = int(self.data_input.n_train)
        y = self.data_input.get_detrended_y_train().reshape(-1, 1).to(torch.float64)
        K = self.get_covariance_matrix(hyper_parameter, noise, indices).contiguous()
        alpha = torch.ones((n, 1), dtype=torch.float64, device=K.device)
        k1 = engine.gemv(K, alpha)
        grad = (k1 - y) + k1
        alpha = variational_sgd_step(alpha, grad)
        return self.optimizable(alpha)
