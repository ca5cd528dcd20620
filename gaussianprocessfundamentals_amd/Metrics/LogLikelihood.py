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
        approx = self.local_approx in _MATRIX_APPROX
        H = mht.NumericalMatrixHandlingType
        if approx and _wants_grad(hyper_parameter, noise, indices) and not (
                self.local_approx is mht.MatrixApproximations.SKI and self.numerical_matrix_handling is H.CHOLESKY_BASED):
            # what the reference's tape sees through the approximate metric (Optimizer/Fitter.py:76-87,
            # :124-132, :155-156): hyperparameters, noise and -- Nystroem -- the inducing inputs; under
            # LINEAR_CONJUGATE_GRADIENT through the executed CG iterations on the approximate matrix
            if self.data_input.data_x_train.dim() == 3:
                raise NotImplementedError("approximate metrics are provided for DataInput, not BatchDataInput")
            z = indices if isinstance(indices, torch.Tensor) else None
            return _ApproxNegLogLikelihood.apply(self, z, _as_tensor(noise), *[_as_tensor(h) for h in hyper_parameter])
        if _wants_grad(hyper_parameter, noise):
            # differentiable form: what the reference's tf.GradientTape sees through get_metric
            # (Optimizer/Fitter.py:104-158); backward() uses the analytic device gradient.  The value
            # comes from the selected handling (STRICT / PSEUDO inverse: the exact gradient is theirs)
            return _NegLogLikelihood.apply(self, _as_tensor(noise), *[_as_tensor(h) for h in hyper_parameter])
        if approx or self.numerical_matrix_handling is not mht.NumericalMatrixHandlingType.CHOLESKY_BASED:
            return self._get_metric_by_strategy(hyper_parameter, noise, indices)
        f = self.covariance_matrix.factorization(hyper_parameter, noise)
        if self.data_input.data_x_train.dim() == 3:
            n = float(self.data_input.n_train)
            logdet_total = torch.sum(f.logdet())
            ll = (-0.5 * f.fit() + -0.5 * logdet_total) + (-0.5 * (n * LOG_2PI))
            agg = global_param.p_batch_metric_aggregator or torch.mean
            res = -agg(ll)
            # one member that is not positive definite makes the whole aggregate +inf (its NaN
            # log-determinant would otherwise reach every member through the summed penalty, Q7);
            # the reference raises from tf.linalg.cholesky (get_metric_checked does)
            return torch.where(torch.any(f.info != 0), torch.full_like(res, math.inf), res)
        # (no copy: every evaluation writes a fresh read-out buffer, engine.AugmentedFactorization._fresh_out)
        return f.nlml().reshape(1, 1)

    def _get_metric_by_strategy(self, hyper_parameter: List, noise, indices=None) -> torch.Tensor:
        """The reference's formula with the bound get_alpha / get_log_determinant (LogLikelihood.py:36-49)
        for the STRICT / PSEUDO inverse and linear-CG handlings."""
        H = mht.NumericalMatrixHandlingType
        if (self.data_input.data_x_train.dim() == 3 and self.local_approx is mht.MatrixApproximations.NONE
                and self.numerical_matrix_handling in (H.STRICT_INVERSE, H.PSEUDO_INVERSE)):
            return self._batch_inverse_metric(hyper_parameter, noise)
        y = self.data_input.get_detrended_y_train().reshape(-1, 1).to(torch.float64)
        alpha = self.get_alpha(hyper_parameter, noise, y, indices).reshape(-1, 1)
        fit = torch.sum(y * alpha)
        logdet = self.get_log_determinant(hyper_parameter, noise, indices)
        n = float(self.data_input.n_train)
        ll = (-0.5 * fit + -0.5 * logdet) + (-0.5 * (n * LOG_2PI))
        if self.local_approx is mht.MatrixApproximations.SKC_LOWER_BOUND:
            # Titsias' correction trace(K_hat + noise I - K) / (2 p_cov_matrix_jitter) (:51-60)
            diff = torch.diagonal(self.get_covariance_matrix(hyper_parameter, noise, indices)) - \
                torch.diagonal(self.covariance_matrix.get_K(hyper_parameter))
            ll = ll - (1.0 / (2.0 * float(global_param.p_cov_matrix_jitter))) * torch.sum(diff)
        return -ll.reshape(1, 1)

    def _batch_inverse_metric(self, hyper_parameter: List, noise) -> torch.Tensor:
        """STRICT / PSEUDO inverse over a BatchDataInput.  In the reference the data fit is [B, 1, 1]
        (one y^T alpha per member) and slogdet gives [B], so their sum broadcasts to [B, 1, B] before
        p_batch_metric_aggregator reduces it (LogLikelihood.py:39-63) -- with the default mean: the
        mean data fit plus the MEAN log-determinant (the Cholesky path sums the log-determinants, Q7).
        K^-1 of every member comes from one batched identity-augmented factorisation; members must be
        positive definite (pinv = inv there)."""
        from .. import engine
        cm = self.covariance_matrix
        f = cm._inverse_factorization(hyper_parameter, noise)
        y = self.data_input.get_detrended_y_train().to(torch.float64)
        B = f.batch
        yb = y.reshape(B, -1)
        fit = torch.stack([torch.dot(yb[b], engine.gemv(f.k_inv(b).contiguous(), yb[b].contiguous()))
                           for b in range(B)])
        logdet = f.logdet()
        n = float(self.data_input.n_train)
        T = (-0.5 * fit).reshape(B, 1, 1) + (-0.5 * logdet).reshape(1, 1, B) + (-0.5 * (n * LOG_2PI))
        agg = global_param.p_batch_metric_aggregator or torch.mean
        return -agg(T)

    def get_metric_and_gradient(self, hyper_parameter: List, noise, reset: bool = True):
        """(-LML [1, 1], [d(-LML)/d h for h in hyper_parameter] (each shaped like h), d(-LML)/d noise).

        One device factorisation with identity extra rows yields K^-1 and alpha; one fused pass
        over the lower triangle evaluates 1/2 sum_ij ((K^-1)_ij - alpha_i alpha_j) dK_ij/d theta
        for every hyperparameter (gpk_nlml_grad).  This is the gradient the reference obtains by
        tf.GradientTape through get_metric (Optimizer/Fitter.py:104-158).  Gradients are NaN when
        K + noise I is not positive definite (the metric is +inf)."""
        if reset:
            self.covariance_matrix.reset()
            self.last_covariance_matrix = None
        H = mht.NumericalMatrixHandlingType
        if self.local_approx in _MATRIX_APPROX and not (self.local_approx is mht.MatrixApproximations.SKI and
                                                        self.numerical_matrix_handling is H.CHOLESKY_BASED):
            raise NotImplementedError("approximate metrics: differentiate get_metric(hyper_parameter, noise, "
                                      "indices) with autograd (inducing-input gradients included)")
        if self.numerical_matrix_handling is H.LINEAR_CONJUGATE_GRADIENT:
            if self.data_input.data_x_train.dim() == 3:
                raise NotImplementedError("LINEAR_CONJUGATE_GRADIENT gradients are provided for DataInput")
            return self._lcg_metric_and_gradient(hyper_parameter, noise)
        if self.data_input.data_x_train.dim() == 3:
            return self._batch_metric_and_gradient(hyper_parameter, noise)
        if self.numerical_matrix_handling in (H.STRICT_INVERSE, H.PSEUDO_INVERSE) and \
                not self._positive_definite(hyper_parameter, noise):
            return self._eigen_metric_and_gradient(hyper_parameter, noise)
        f = self.covariance_matrix.inverse_factorization(hyper_parameter, noise, gradient=True)
        g = f.gradient()[0]   # (fresh buffers per evaluation: no copies needed)
        return f.nlml().reshape(1, 1), _split_like(g[:-1], hyper_parameter), g[-1]

    def _batch_metric_and_gradient(self, hyper_parameter: List, noise):
        """BatchDataInput (quirk Q7).  CHOLESKY_BASED: -LML = -agg_b(-1/2 fit_b - 1/2 sum_b' logdet_b' - c):
        with agg = mean, 1/2 mean fit + 1/2 sum logdet + c, whose gradient is the sum over members of the
        per-member gradient with y scaled by 1 / sqrt(B) (alpha alpha^T weighted 1 / B); with agg = sum,
        B times that.  STRICT / PSEUDO inverse ([B, 1, B] broadcast, Metrics/LogLikelihood.py:39-63): mean
        fit + mean log-determinant, i.e. the mean of the per-member gradients (sum: B^2 entries, B times
        their sum).  One batched identity-augmented factorisation + gradient pass (gpk_nlml_grad)."""
        H = mht.NumericalMatrixHandlingType
        agg = global_param.p_batch_metric_aggregator or torch.mean
        if agg is not torch.mean and agg is not torch.sum:
            raise NotImplementedError("batch gradients for p_batch_metric_aggregator in (torch.mean, torch.sum)")
        B = int(self.data_input.data_x_train.shape[0])
        chol = self.numerical_matrix_handling is H.CHOLESKY_BASED
        value = self.get_metric([_as_tensor(h).detach() for h in hyper_parameter], _as_tensor(noise).detach(),
                                reset=True)
        f = self.covariance_matrix.inverse_factorization(hyper_parameter, noise, gradient=True,
                                                         y_scale=(1.0 / math.sqrt(B)) if chol else 1.0)
        # a member that is not positive definite has no gradient here (the reference raises from
        # tf.linalg.cholesky under CHOLESKY_BASED; the batched STRICT / PSEUDO value needs K^-1 of every
        # member as well): raise CholeskyError instead of returning NaN gradients beside an +inf value
        f.check_info()
        g = f.gradient().sum(0)
        if chol:
            g = g * (float(B) if agg is torch.sum else 1.0)
        else:
            g = g * (float(B) if agg is torch.sum else 1.0 / B)
        return value, _split_like(g[:-1], hyper_parameter), g[-1]

    def _eigen_metric_and_gradient(self, hyper_parameter: List, noise):
        """STRICT / PSEUDO inverse of a K + noise I that is not positive definite (eigendecomposition route of
        Metrics.py): -LML = 1/2 y^T f(K) y + 1/2 sum_i log|lam_i| + c with f = 1/lam (STRICT: every
        eigenvalue; PSEUDO: tf.linalg.pinv's kept ones).  Adjoint of K: 1/2 V diag(1/lam) V^T (slogdet) plus
        pinv's reverse mode of 1/2 y y^T (gpk_pinv_backward_scale; = -1/2 alpha alpha^T without truncation);
        then gpk_kernel_vjp for the hyperparameters and its trace for the noise."""
        from .. import engine
        H = mht.NumericalMatrixHandlingType
        value = self._get_metric_by_strategy(hyper_parameter, noise).reshape(1, 1)
        lam, V = self._eigen(hyper_parameter, noise)
        rcond = 0.0 if self.numerical_matrix_handling is H.STRICT_INVERSE else -1.0
        _, _, mu_all = engine.pinv_factor(lam, V, 0, rcond=0.0, return_mu=True)
        _, _, mu = engine.pinv_factor(lam, V, 0, rcond=rcond, return_mu=True)
        y = self._y(None)
        vy = engine.dgemm(V, y, trans_a=True)                             # V^T y
        T = engine.dgemm(vy, vy, trans_b=True, alpha=0.5)                 # V^T (1/2 y y^T) V
        kbar = engine.pinv_backward(lam, V, mu, T=T)
        kbar = kbar + 0.5 * engine.dgemm(V * mu_all[None, :], V, trans_b=True)
        x = self.data_input.data_x_train
        gh, _ = engine.kernel_vjp(self.covariance_matrix.kernel, hyper_parameter, x, x,
                                  G=(kbar + kbar.T).contiguous())
        return value, _split_like(0.5 * gh, hyper_parameter), torch.trace(kbar)

    def _lcg_metric_and_gradient(self, hyper_parameter: List, noise):
        """LINEAR_CONJUGATE_GRADIENT (Metrics.py:141-147): -LML = 1/2 y^T x_cg + 1/2 slogdet(K) + c with x_cg the
        reference's CG iterate (tolerance 1e-2), differentiated as tf.GradientTape does -- through the executed
        iterations (Auxiliary.LinearConjugateGradients.linear_cg_backward: one GEMV per iteration in reverse),
        not as the exact solve.  Adjoint of K: Q P^T from the loop (seeded with 1/2 y) plus 1/2 K^-1 from the
        log-determinant (identity-augmented factorisation; the eigendecomposition when K is not positive
        definite); then gpk_kernel_vjp for the hyperparameters and its trace for the noise."""
        from .. import engine
        from ..Auxiliary.LinearConjugateGradients import linear_cg, linear_cg_backward
        K = self.get_covariance_matrix(hyper_parameter, noise, None).contiguous()
        y = self._y(None)
        tape = []
        x = linear_cg(K, y, torch.zeros_like(y), tape=tape)
        n = float(self.data_input.n_train)
        logdet = self.get_log_determinant(hyper_parameter, noise, None)
        value = (-((-0.5 * torch.sum(y * x) + -0.5 * logdet) + (-0.5 * (n * LOG_2PI)))).reshape(1, 1)
        P, Q = linear_cg_backward(K, tape, 0.5 * y)
        if self._positive_definite(hyper_parameter, noise):
            f = self.covariance_matrix.inverse_factorization(hyper_parameter, noise, gradient=False)
            G = (0.5 * f.k_inv(0).to(torch.float64)).contiguous()
        else:
            lam, V = self._eigen(hyper_parameter, noise)
            _, _, mu_all = engine.pinv_factor(lam, V, 0, rcond=0.0, return_mu=True)
            G = 0.5 * engine.dgemm(V * mu_all[None, :], V, trans_b=True)
        if P.shape[1] > 0:
            G = engine.dgemm(Q, P, trans_b=True, beta=1.0, C=G)
        xin = self.data_input.data_x_train
        gh, _ = engine.kernel_vjp(self.covariance_matrix.kernel, hyper_parameter, xin, xin, G=G)
        return value, _split_like(gh, hyper_parameter), torch.trace(G)

    def get_gradients(self, hyper_parameter: List, noise, reset: bool = True) -> torch.Tensor:
        """Metrics.py:31 (AbstractMetric.get_gradients; the reference's gradient_function of
        Optimizer/ConjugateGradient.py:28-31 calls it): d(-LML)/d(hyperparameters) as one flat vector in
        DFS order (the serialised layout of BasicGPComponent.serialize_hyper_parameter) -- the device
        gradient of get_metric_and_gradient."""
        _, grads, _ = self.get_metric_and_gradient(hyper_parameter, noise, reset=reset)
        return torch.cat([g.reshape(-1) for g in grads]) if grads else torch.zeros(0, dtype=torch.float64)

    def get_metric_checked(self, hyper_parameter: List, noise, reset: bool = True) -> torch.Tensor:
        """get_metric that raises CholeskyError when K + noise I is not positive definite
        (the reference's TensorFlow raises from tf.linalg.cholesky); synchronises."""
        out = self.get_metric(hyper_parameter, noise, reset=reset)
        self.covariance_matrix.factorization(hyper_parameter, noise).check_info()
        return out


_MATRIX_APPROX = (mht.MatrixApproximations.BASIC_NYSTROEM, mht.MatrixApproximations.SKC_LOWER_BOUND,
                  mht.MatrixApproximations.SKI)


def _as_tensor(h) -> torch.Tensor:
    return h if isinstance(h, torch.Tensor) else torch.as_tensor(h, dtype=torch.float64)


def _wants_grad(hyper_parameter, noise, indices=None) -> bool:
    if not torch.is_grad_enabled():
        return False
    return any(isinstance(h, torch.Tensor) and h.requires_grad for h in list(hyper_parameter) + [noise, indices])


def _split_like(flat: torch.Tensor, hyper_parameter) -> List[torch.Tensor]:
    """Split a flat DFS-ordered vector into pieces shaped like the hyperparameter entries."""
    out, i = [], 0
    for h in hyper_parameter:
        t = _as_tensor(h)
        k = max(1, t.numel())
        out.append(flat[i:i + k].reshape(t.shape))
        i += k
    return out


class _NegLogLikelihood(torch.autograd.Function):
    """-LML as an autograd node whose backward is the analytic device gradient."""

    @staticmethod
    def forward(ctx, metric, noise, *hyper_parameter):
        H = mht.NumericalMatrixHandlingType
        nl, grads, gnoise = metric.get_metric_and_gradient(list(hyper_parameter), noise, reset=False)
        if metric.numerical_matrix_handling is not H.CHOLESKY_BASED and metric.data_input.data_x_train.dim() == 2:
            # the value of the selected handling (STRICT / PSEUDO inverse of a positive-definite K: the
            # gradient is the Cholesky one; otherwise both come from the eigendecomposition route)
            nl = metric._get_metric_by_strategy(list(hyper_parameter), noise).reshape(1, 1)
        ctx.save_for_backward(gnoise, *grads)
        ctx.meta = [(h.device, h.dtype) for h in (noise,) + hyper_parameter]
        return nl.clone()

    @staticmethod
    def backward(ctx, gout):
        saved = ctx.saved_tensors
        s = gout.reshape(())
        res = [None]
        for g, (dev, dt) in zip(saved, ctx.meta):
            res.append((g * s).to(device=dev, dtype=dt))
        return tuple(res)


class _ApproxNegLogLikelihood(torch.autograd.Function):
    """-LML under BASIC_NYSTROEM / SKC_LOWER_BOUND / SKI (STRICT / PSEUDO) as an autograd node: forward is
    the device metric, backward the device reverse mode of Metrics/_approx_grad.py (adjoints of the
    hyperparameters, the noise and the inducing inputs).  The Nystroem log-determinant contributes only when
    this call computes it (the reference caches it across calls, so a cached value is a constant for the
    tape)."""

    @staticmethod
    def forward(ctx, metric, z, noise, *hyper_parameter):
        A = mht.MatrixApproximations
        H = mht.NumericalMatrixHandlingType
        hyp = [h.detach() for h in hyper_parameter]
        zd = z.detach() if isinstance(z, torch.Tensor) else z
        nys = metric.local_approx in (A.BASIC_NYSTROEM, A.SKC_LOWER_BOUND)
        ctx.fresh_det = nys and metric.nystroem_matrix.K_approx_det is None
        ctx.lcg = None
        if metric.numerical_matrix_handling is H.LINEAR_CONJUGATE_GRADIENT:
            nl, ctx.lcg = _approx_lcg_value(metric, hyp, noise.detach(), zd)
        else:
            nl = metric._get_metric_by_strategy(hyp, noise.detach(), zd).reshape(1, 1)
        ctx.metric, ctx.hyp, ctx.z, ctx.noise = metric, hyp, zd, noise.detach()
        ctx.want_z = isinstance(z, torch.Tensor) and z.requires_grad
        ctx.meta = [(h.device, h.dtype, h.shape) for h in (noise,) + hyper_parameter]
        ctx.z_meta = (z.device, z.dtype, z.shape) if isinstance(z, torch.Tensor) else None
        return nl.clone()

    @staticmethod
    def backward(ctx, gout):
        from . import _approx_grad as ag
        from .. import engine
        A = mht.MatrixApproximations
        H = mht.NumericalMatrixHandlingType
        m, hyp, noise = ctx.metric, ctx.hyp, ctx.noise
        nv = float(noise)
        X = m.data_input.data_x_train
        kernel = m.covariance_matrix.kernel
        lcg_adj = None
        if ctx.lcg is not None:
            # the fit's adjoint of the approximate matrix through the executed CG iterations: Q P^T
            # (Auxiliary.LinearConjugateGradients.linear_cg_backward, seeded with 1/2 y)
            from ..Auxiliary.LinearConjugateGradients import linear_cg_backward
            Khat, tape, y = ctx.lcg
            lcg_adj = linear_cg_backward(Khat, tape, 0.5 * y)
            ctx.lcg = None
        if m.local_approx is A.SKI:
            Ainv = m._approx_factorization(hyp, noise, ctx.z).k_inv(0).to(torch.float64).contiguous()
            if lcg_adj is not None:
                # A-bar = Q P^T (fit) + 1/2 A^-1 (slogdet of the SKI matrix)
                P, Q = lcg_adj
                Abar = (0.5 * Ainv).contiguous()
                if P.shape[1] > 0:
                    engine.dgemm(Q, P, trans_b=True, beta=1.0, C=Abar)
                gh, gn = ag.ski_adjoint_from(m, hyp, Abar)
            else:
                alpha_hat = m.get_alpha(hyp, noise, None, ctx.z)
                gh, gn = ag.ski_adjoint(m, hyp, noise, alpha_hat, Ainv)
            gz = None
        else:
            Z = engine.as_device_f64(ctx.z)
            Z = Z.reshape(-1, 1) if Z.dim() == 1 else Z
            adj = ag.NystroemAdjoint(kernel, hyp, X, Z, nv)
            if lcg_adj is not None:
                adj.lowrank_matrix_adjoint(*lcg_adj)
            elif m.numerical_matrix_handling is H.CHOLESKY_BASED:
                adj.exact_fit(m.covariance_matrix.get_L_alpha(hyp, noise), 0.5)
            else:
                adj.approx_fit(m.get_alpha(hyp, noise, None, ctx.z), 0.5)
            if ctx.fresh_det:
                adj.nystroem_logdet(0.5)
            if m.local_approx is A.SKC_LOWER_BOUND:
                adj.trace_correction(1.0 / (2.0 * float(global_param.p_cov_matrix_jitter)))
            gh, gn, gz = adj.finish(ctx.want_z)
        s = gout.reshape(())
        out = [None]
        if ctx.z_meta is None:
            out.append(None)
        elif gz is None or not ctx.want_z:
            out.append(None)
        else:
            dev, dt, shp = ctx.z_meta
            out.append((gz * s).reshape(shp).to(device=dev, dtype=dt))
        dev, dt, shp = ctx.meta[0]
        out.append((gn * s).reshape(shp).to(device=dev, dtype=dt))
        for g, (dev, dt, shp) in zip(_split_like(gh, hyp), ctx.meta[1:]):
            out.append((g * s).reshape(shp).to(device=dev, dtype=dt))
        return tuple(out)


def _approx_lcg_value(metric, hyp, noise, z):
    """-LML of an approximate metric under LINEAR_CONJUGATE_GRADIENT (LogLikelihood.py:36-60 with
    Metrics.py:141-147): alpha = linear_cg(K_hat, y, 0) on the approximate matrix (its iterations recorded for
    the reverse mode), the bound log-determinant (Nystroem determinant, or slogdet of the SKI matrix), the
    SKC lower bound's trace correction.  Returns ([1, 1] value, (K_hat, tape, y))."""
    from ..Auxiliary.LinearConjugateGradients import linear_cg
    metric._require_plain()
    Khat = metric.get_covariance_matrix(hyp, noise, z).contiguous()
    y = metric._y(None)
    tape = []
    x = linear_cg(Khat, y, torch.zeros_like(y), tape=tape)
    logdet = metric.get_log_determinant(hyp, noise, z)
    n = float(metric.data_input.n_train)
    ll = (-0.5 * torch.sum(y * x) + -0.5 * logdet) + (-0.5 * (n * LOG_2PI))
    if metric.local_approx is mht.MatrixApproximations.SKC_LOWER_BOUND:
        diff = torch.diagonal(Khat) - torch.diagonal(metric.covariance_matrix.get_K(hyp))
        ll = ll - (1.0 / (2.0 * float(global_param.p_cov_matrix_jitter))) * torch.sum(diff)
    return -ll.reshape(1, 1), (Khat, tape, y)


def blockwise_hyper_parameter_offset(_gp) -> int:
    """Offset of the first constituent's hyperparameters in a blockwise metric's hyperparameter
    list.  Quirk kept: the reference tests ``hasattr(_gp, 'change_point_positions')``
    on the GP object (LogLikelihood.py:80-83, MeanSquaredError.py:64-67), which no GP object has,
    so the offset is always 0 -- even for a change-point kernel whose change points lead its list."""
    return len(_gp.covariance_matrix.kernel.change_point_positions) if hasattr(_gp, "change_point_positions") else 0


class BlockwiseLogLikelihood(AbstractMetric):
    """Sum of the constituent GPs' -LML (LogLikelihood.py:68-104).

    The reference evaluates one LogLikelihood per segment, one TensorFlow Cholesky after another;
    here all segments are factored by ONE ragged device batch (engine.RaggedFactorization), each
    segment with its own kernel, hyperparameter slice and detrended targets.  Segments without
    training points contribute 0 (an empty Cholesky).  Returns a [1, 1] tensor like LogLikelihood."""

    def __init__(self, _gp, local_approx, numerical_matrix_handling, subset_size: int = None):
        self.local_approx = local_approx
        self.numerical_matrix_handling = numerical_matrix_handling
        self.subset_size = subset_size
        self._gp = _gp

    def segment_factorization(self, hyper_parameter: List, noise):
        from ..Statistics.CovarianceMatrix import factor_segments
        index = blockwise_hyper_parameter_offset(self._gp)
        kernels, slices, dis = [], [], []
        for sub in self._gp.constituent_gps:
            kern = sub.covariance_matrix.kernel
            nh = kern.get_number_of_hyper_parameter()
            kernels.append(kern)
            slices.append(list(hyper_parameter[index:index + nh]))
            dis.append(sub.data_input)
            index += nh
        return factor_segments(kernels, slices, dis, noise)

    def get_metric(self, hyper_parameter: List, noise, indices=None, reset: bool = True) -> torch.Tensor:
        if (self.local_approx is not mht.MatrixApproximations.NONE or
                self.numerical_matrix_handling is not mht.NumericalMatrixHandlingType.CHOLESKY_BASED):
            return self._per_segment(hyper_parameter, noise, indices)
        f, _ = self.segment_factorization(hyper_parameter, noise)
        for sub in self._gp.constituent_gps:
            sub.covariance_matrix.reset()
            sub.aux.reset()
        if f is None:
            return torch.zeros((1, 1), dtype=torch.float64, device=_device())
        return torch.sum(f.nlml()).reshape(1, 1)


    def _per_segment(self, hyper_parameter: List, noise, indices=None) -> torch.Tensor:
        """One LogLikelihood per segment with the requested approximation / handling, as the
        reference does for every strategy (LogLikelihood.py:86-104); segments without training
        points contribute 0."""
        index = blockwise_hyper_parameter_offset(self._gp)
        total = torch.zeros((1, 1), dtype=torch.float64, device=_device())
        for sub in self._gp.constituent_gps:
            kern = sub.covariance_matrix.kernel
            nh = kern.get_number_of_hyper_parameter()
            if int(sub.data_input.n_train) > 0:
                sub_ll = LogLikelihood(sub.data_input, sub.covariance_matrix, self.local_approx,
                                       self.numerical_matrix_handling, self.subset_size)
                total = total + sub_ll.get_metric(list(hyper_parameter[index:index + nh]), noise, indices).reshape(1, 1)
            index += nh
            sub.covariance_matrix.reset()
            sub.aux.reset()
        return total


def _device():
    from .. import engine
    return engine.device()
