"""Posterior properties (gpbasics/Statistics/Auxiliary.py:14-103).

The reference computes mu = K_s^T alpha and Sigma = K_ss - v^T v with v = inv(L) K_s, an explicit
N^3 inverse (Auxiliary.py:57-93).  Here the test points become extra rows of the augmented
matrix and ONE device factorisation yields V^T = K_s^T L^-T in those rows and the Schur
complement K_ss - V^T V in the corner, together with mu = V^T z (include/gpk.h).  Returned
shapes follow the reference: mu [M], variance the full [M, M] matrix, sd its elementwise sqrt
(quirk Q8: NaN where an off-diagonal covariance is negative).
"""
from __future__ import annotations

from typing import List

import torch

from .. import engine
from .. import global_parameters as global_param
from .CovarianceMatrix import noise_vector

global_param.ensure_init()


class AuxiliaryGpProperties:
    def __init__(self, covariance_matrix, mean_function):
        self.covariance_matrix = covariance_matrix
        self.data_input = None
        self.mean_function = mean_function
        self.reset()

    def reset(self):
        self.detrended_y_train = None
        self.inv_L_K_dot_K_s = None
        self.posterior_mu = None
        self.posterior_var = None
        self.posterior_sd = None
        self._post = None

    def set_data_input(self, data_input):
        self.data_input = data_input
        self.reset()


class HolisticAuxiliaryGpProperties(AuxiliaryGpProperties):
    def _posterior_factorization(self, hyper_parameter: List, noise) -> engine.AugmentedFactorization:
        if self._post is None:
            di = self.data_input
            if di.data_x_train.dim() != 2:
                raise NotImplementedError("posterior of BatchDataInput is not provided")
            cm = self.covariance_matrix
            x, xt = di.data_x_train, di.data_x_test
            n, d, m = int(x.shape[0]), int(x.shape[1]), int(xt.shape[0])
            y = di.get_detrended_y_train().reshape(1, n).to(torch.float64).contiguous()
            f = engine.AugmentedFactorization(n, d, m, 1, global_param.p_dtype)
            kd = engine.kernel_descriptor(cm.kernel, d)
            hyp = engine.pack_hyper_parameter(hyper_parameter, kd.n_hyp)
            f.run(kd, hyp, 0, noise_vector(noise), 0, x.contiguous(), 0, y, 0, Xs=xt.contiguous(), xs_bstride=0)
            cm.kernel._record_hyper_parameter(list(hyper_parameter))
            f.check_info()
            self._post = f
        return self._post

    def get_inverse_cholesky_k_times_k_s(self, hyper_parameter: List, noise):
        """v = inv(L) K_s [N, M] (Auxiliary.py:57-66)."""
        if self.data_input is None:
            return None
        if self.inv_L_K_dot_K_s is None:
            f = self._posterior_factorization(hyper_parameter, noise)
            self.inv_L_K_dot_K_s = f.extra_rows(0).to(torch.float64).transpose(0, 1).contiguous()
        return self.inv_L_K_dot_K_s

    def get_posterior_mu(self, hyper_parameter: List, noise):
        """mu = K_s^T alpha, shape [M] (Auxiliary.py:68-81)."""
        if self.data_input is None:
            return None
        if self.posterior_mu is None:
            self.posterior_mu = self._posterior_factorization(hyper_parameter, noise).posterior_mu(0).clone()
        return self.posterior_mu

    def get_posterior_var(self, hyper_parameter: List, noise):
        """K_ss - v^T v, full [M, M] (Auxiliary.py:83-93)."""
        if self.data_input is None:
            return None
        if self.posterior_var is None:
            self.posterior_var = self._posterior_factorization(hyper_parameter, noise).corner(0).to(torch.float64)
        return self.posterior_var

    def get_posterior_var_diag(self, hyper_parameter: List, noise):
        """Diagonal of the posterior covariance [M] (build extension; no M x M read-back)."""
        if self.data_input is None:
            return None
        return self._posterior_factorization(hyper_parameter, noise).posterior_var_diag(0).clone()

    def get_posterior_sd(self, hyper_parameter: List, noise):
        """Elementwise sqrt of the full posterior covariance (Auxiliary.py:95-103)."""
        if self.data_input is None:
            return None
        if self.posterior_sd is None:
            self.posterior_sd = torch.sqrt(self.get_posterior_var(hyper_parameter, noise))
        return self.posterior_sd


def _segment_posterior(kernels, hyper_parameters, data_inputs, noise):
    from .CovarianceMatrix import factor_segments
    f, index = factor_segments(kernels, hyper_parameters, data_inputs, noise, with_test=True)
    if f is not None:
        f.check_info()
    return f, index


def segment_posterior_mu(kernels, hyper_parameters, data_inputs, noise) -> torch.Tensor:
    """Posterior means of independent segments concatenated in segment order [sum M_i]
    (the constituent-GP loop of GaussianProcess.predict, gpbasics/Statistics/GaussianProcess.py:64-77),
    from ONE ragged factorisation with the test points as extra rows.  A segment without training
    points has K_s of shape [0, M_i] and so a zero mean."""
    f, index = _segment_posterior(kernels, hyper_parameters, data_inputs, noise)
    parts = [torch.zeros(di.n_test, dtype=torch.float64, device=engine.device()) for di in data_inputs]
    for j, i in enumerate(index):
        parts[i] = f.posterior_mu(j).clone()
    return torch.cat(parts) if parts else torch.zeros(0, dtype=torch.float64, device=engine.device())


class BlockwiseAuxiliaryGpProperties(HolisticAuxiliaryGpProperties):
    """Posterior of a segmented GP (Auxiliary.py:106-107 inherits the holistic formulas, which over
    a SegmentedCovarianceMatrix amount to the per-segment posteriors in segment order).  All segments
    come out of one ragged factorisation: mu concatenated, the covariance block-diagonal."""

    def _segments(self, hyper_parameter, noise):
        if self._post is None:
            cm = self.covariance_matrix
            self._post = _segment_posterior(cm.kernel.child_nodes, cm._slices(hyper_parameter),
                                            self.data_input.data_inputs, noise)
        return self._post

    def get_posterior_mu(self, hyper_parameter: List, noise):
        if self.data_input is None:
            return None
        if self.posterior_mu is None:
            cm = self.covariance_matrix
            self.posterior_mu = segment_posterior_mu(cm.kernel.child_nodes, cm._slices(hyper_parameter),
                                                     self.data_input.data_inputs, noise)
        return self.posterior_mu

    def get_posterior_var(self, hyper_parameter: List, noise):
        if self.data_input is None:
            return None
        if self.posterior_var is None:
            f, index = self._segments(hyper_parameter, noise)
            dis = self.data_input.data_inputs
            blocks = []
            for i, di in enumerate(dis):
                if i in index:
                    blocks.append(f.corner(index.index(i)).to(torch.float64))
                else:  # no training points: the prior K_ss
                    cm = self.covariance_matrix
                    blocks.append(cm.kernel.child_nodes[i].get_tf_tensor(cm._slices(hyper_parameter)[i],
                                                                        di.data_x_test, di.data_x_test)
                                  if di.n_test > 0 else None)
            self.posterior_var = self.covariance_matrix._block_diag(blocks)
        return self.posterior_var

    def get_posterior_var_diag(self, hyper_parameter: List, noise):
        return torch.diagonal(self.get_posterior_var(hyper_parameter, noise)).clone()

    def get_inverse_cholesky_k_times_k_s(self, hyper_parameter: List, noise):
        """inv(L) K_s over a SegmentedCovarianceMatrix (Auxiliary.py:57-66 inherited): block-diagonal
        [sum n_i, sum m_i] of the segments' V_i = L_i^-1 K_s,i, read (transposed) from the extra rows of
        the one ragged factorisation; a segment without training (test) points has an n_i x 0
        (0 x m_i) block."""
        if self.data_input is None:
            return None
        if self.inv_L_K_dot_K_s is None:
            f, index = self._segments(hyper_parameter, noise)
            blocks = []
            for i, di in enumerate(self.data_input.data_inputs):
                if i in index:
                    blocks.append(f.extra_rows(index.index(i)).to(torch.float64).transpose(0, 1))
                else:
                    blocks.append(torch.zeros((int(di.n_train), int(di.n_test)), dtype=torch.float64,
                                              device=engine.device()))
            self.inv_L_K_dot_K_s = torch.block_diag(*blocks).contiguous()
        return self.inv_L_K_dot_K_s
