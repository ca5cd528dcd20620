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

Gradient (what the reference's fitter gets from tf.GradientTape through get_metric, Optimizer/Fitter.py:
76-87): the step writes alpha by a variable assignment, which the tape does not differentiate, so alpha is
a constant and the gradient is that of 1/2 a^T K a - a^T y - 1/2 det at the stepped a -- 1/2 a a^T
through the kernel's reverse mode (gpk_kernel_vjp, rank-1 weight) and 1/2 a^T a for the noise, plus
-1/2 the Nystroem determinant's adjoint (hyperparameters, noise, inducing inputs; Metrics/_approx_grad.py).
A K or determinant taken from the caches is a constant for the tape: it contributes only in the call that
computes it.  Checked against oracle/gp_autodiff.skc_upper_nlml_and_grad (pinned by finite differences).
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
        from .LogLikelihood import _as_tensor, _wants_grad
        if _wants_grad(hyper_parameter, noise, indices):
            return _SkcUpperBound.apply(self, indices, _as_tensor(noise), *[_as_tensor(h) for h in hyper_parameter])
        return self._value_and_alpha(hyper_parameter, noise, indices)[0]

    def _value_and_alpha(self, hyper_parameter: List, noise, indices=None):
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
        return self.optimizable(alpha), alpha


class _SkcUpperBound(torch.autograd.Function):
    """The SKC upper bound as an autograd node (module docstring: alpha constant, cached K / determinant
    constant)."""

    @staticmethod
    def forward(ctx, metric, indices, noise, *hyper_parameter):
        hyp = [h.detach() for h in hyper_parameter]
        ind = indices.detach() if isinstance(indices, torch.Tensor) else indices
        ctx.k_fresh = metric.last_covariance_matrix is None and metric.covariance_matrix.noised_K is None
        ctx.det_fresh = metric.nyK.K_approx_det is None
        value, alpha = metric._value_and_alpha(hyp, noise.detach(), ind)
        ctx.metric, ctx.hyp, ctx.ind, ctx.noise, ctx.alpha = metric, hyp, ind, float(noise), alpha
        ctx.want_z = isinstance(indices, torch.Tensor) and indices.requires_grad
        ctx.meta = [(h.device, h.dtype, h.shape) for h in (noise,) + hyper_parameter]
        ctx.z_meta = (indices.device, indices.dtype, indices.shape) if isinstance(indices, torch.Tensor) else None
        return value.reshape(1, 1).clone()

    @staticmethod
    def backward(ctx, gout):
        from . import _approx_grad as ag
        from .LogLikelihood import _split_like
        m, hyp = ctx.metric, ctx.hyp
        X = m.data_input.data_x_train
        kernel = m.covariance_matrix.kernel
        kd = engine.kernel_descriptor(kernel, int(X.shape[1]))
        gh = torch.zeros(kd.n_hyp, dtype=torch.float64, device=X.device)
        gn = torch.zeros((), dtype=torch.float64, device=X.device)
        gz = None
        if ctx.k_fresh:
            a = ctx.alpha.reshape(-1).contiguous()
            gk, _ = engine.kernel_vjp(kernel, hyp, X, X, gu=a, gv=a)
            gh = gh + 0.5 * gk
            gn = gn + 0.5 * torch.dot(a, a)
        if ctx.det_fresh:
            Z = m.nyK._inducing(ctx.ind)
            adj = ag.NystroemAdjoint(kernel, hyp, X, Z, ctx.noise)
            adj.nystroem_logdet(-0.5)
            h2, n2, gz = adj.finish(ctx.want_z)
            gh = gh + h2
            gn = gn + n2
        s = gout.reshape(())
        out = [None]
        if ctx.z_meta is None or gz is None or not ctx.want_z:
            out.append(None)
        else:
            dev, dt, shp = ctx.z_meta
            out.append((gz * s).reshape(shp).to(device=dev, dtype=dt))
        dev, dt, shp = ctx.meta[0]
        out.append((gn * s).reshape(shp).to(device=dev, dtype=dt))
        for g, (dev, dt, shp) in zip(_split_like(gh, hyp), ctx.meta[1:]):
            out.append((g * s).reshape(shp).to(device=dev, dtype=dt))
        return tuple(out)
