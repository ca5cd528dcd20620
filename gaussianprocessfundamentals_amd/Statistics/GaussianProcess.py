"""Gaussian process objects (gpbasics/Statistics/GaussianProcess.py:20-206).

:class:`GaussianProcess` is the holistic GP of the hot path.  :class:`BlockwiseGaussianProcess`
(a change-point operator) and :class:`PartitionedGaussianProcess` (a partition operator) hold one
constituent GaussianProcess per segment; their likelihood and posterior are computed for all
segments at once by one ragged device factorisation (Statistics/CovarianceMatrix.factor_segments).
"""
from __future__ import annotations

import logging
from typing import List, Tuple

import torch

from .. import engine
from .. import global_parameters as global_param
from . import Auxiliary as ax
from . import CovarianceMatrix as cm

global_param.ensure_init()


class AbstractGaussianProcess:
    def __init__(self, kernel, mean_function):
        self.mean_function = mean_function
        self.kernel = kernel
        self.covariance_matrix = None
        self.aux = None
        self.data_input = None
        self.inducing_points = None

    def set_inducing_points(self, inducing_points):
        self.inducing_points = inducing_points

    def set_data_input(self, data_input):
        """A new data input obsoletes every memoised matrix (GaussianProcess.py:35-40)."""
        self.data_input = data_input
        self.covariance_matrix.set_data_input(data_input)
        self.aux.set_data_input(data_input)

    def predict(self, kernel_hyper_param: List = None, mean_function_hyper_param: List = None,
                noise=None) -> Tuple:
        """(mean + posterior mu, mean, posterior mu), each [M] (GaussianProcess.py:42-85).
        noise defaults to the jitter p_cov_matrix_jitter, not to kernel.get_noise() (:48-49)."""
        self.aux.reset()
        self.covariance_matrix.reset()
        if noise is None:
            noise = global_param.p_cov_matrix_jitter
        logging.debug("GP Predict: Retrieving covariance and mean function hyper parameters.")
        if mean_function_hyper_param is None:
            mean_function_hyper_param = self.mean_function.get_last_hyper_parameter()
            if mean_function_hyper_param is None:
                mean_function_hyper_param = self.mean_function.get_default_hyper_parameter()
        if kernel_hyper_param is None:
            kernel_hyper_param = self.kernel.get_last_hyper_parameter()
            if kernel_hyper_param is None:
                kernel_hyper_param = self.kernel.get_default_hyper_parameter(self.data_input.get_x_range(),
                                                                             self.data_input.n_train)
        mean_mu = self.mean_function.get_tf_tensor(mean_function_hyper_param, self.data_input.data_x_test)
        if isinstance(self, (PartitionedGaussianProcess, BlockwiseGaussianProcess)):
            # per-segment posterior means concatenated in segment order (GaussianProcess.py:64-77);
            # a change-point kernel's change points precede the children's hyperparameters.  (The
            # reference reads them from self.covariance_matrix.change_point_positions, an attribute
            # SegmentedCovarianceMatrix does not have -- it raises AttributeError there; the kernel's
            # change points are the intended offset, as in SegmentedCovarianceMatrix.get_K_blocks.)
            index = len(self.kernel.change_point_positions) if isinstance(self, BlockwiseGaussianProcess) else 0
            kernels, slices = [], []
            for sub in self.constituent_gps:
                nh = sub.kernel.get_number_of_hyper_parameter()
                kernels.append(sub.kernel)
                slices.append(list(kernel_hyper_param[index:index + nh]))
                index += nh
            post_mu = ax.segment_posterior_mu(kernels, slices, [g.data_input for g in self.constituent_gps], noise)
        else:
            post_mu = self.aux.get_posterior_mu(kernel_hyper_param, noise)
        return mean_mu + post_mu, mean_mu, post_mu

    def get_n_prior_functions(self, n: int, hyper_param, noise, generator=None):
        """n prior function draws at the test points, [n_test, n] (GaussianProcess.py:87-95):
        L_K_ss N, N ~ normal(mean(y_train), std(y_train)) -- the reference's draw, whose mean and
        spread come from the training targets (np.mean / np.std, population std), not N(0, 1).
        L_K_ss is the device Cholesky of K_ss + noise I, the product the f64 MFMA dgemm;
        ``generator`` (a torch.Generator on the device) only makes the draw reproducible."""
        L = self.covariance_matrix.get_L_K_ss(hyper_param, noise)
        y = engine.as_device_f64(self.data_input.data_y_train)
        z = torch.randn((int(L.shape[0]), int(n)), dtype=torch.float64, device=L.device, generator=generator)
        z = z * torch.std(y, unbiased=False) + torch.mean(y)
        return engine.dgemm(L.contiguous(), z)

    def get_n_posterior_functions(self, n: int, hyper_param, noise, generator=None):
        """n posterior function draws, [n_test, n] (GaussianProcess.py:97-110): mu + chol(Sigma +
        p_cov_matrix_jitter I) N(0, 1), Sigma the full posterior covariance (Auxiliary.py:83-93),
        its Cholesky on the device (DenseFactorization; CholeskyError if Sigma + jitter I is not PD,
        where the reference's tf.linalg.cholesky raises InvalidArgumentError)."""
        sigma = self.aux.get_posterior_var(hyper_param, noise).to(torch.float64).contiguous()
        m = int(sigma.shape[0])
        f = engine.DenseFactorization(m)
        f.run(sigma, float(torch.as_tensor(global_param.p_cov_matrix_jitter)))
        f.check_info()
        L = f.cholesky(0).to(torch.float64).contiguous()
        z = torch.randn((m, int(n)), dtype=torch.float64, device=L.device, generator=generator)
        mu = self.aux.get_posterior_mu(hyper_param, noise).to(torch.float64).reshape(-1, 1)
        return engine.dgemm(L, z, beta=1.0, C=mu.expand(m, int(n)).contiguous())

    def copy(self):
        raise NotImplementedError


class GaussianProcess(AbstractGaussianProcess):
    def __init__(self, kernel, mean_function):
        super().__init__(kernel, mean_function)
        self.covariance_matrix = cm.HolisticCovarianceMatrix(self.kernel)
        self.aux = ax.HolisticAuxiliaryGpProperties(self.covariance_matrix, self.mean_function)

    def copy(self):
        g = GaussianProcess(self.kernel, self.mean_function)
        g.set_inducing_points(self.inducing_points)
        return g



class PredefinedGaussianProcess(AbstractGaussianProcess):
    """A GP around a given covariance-matrix object (GaussianProcess.py:134-143)."""

    def __init__(self, covariance_matrix, mean_function):
        super().__init__(covariance_matrix.kernel, mean_function)
        self.covariance_matrix = covariance_matrix
        self.aux = ax.HolisticAuxiliaryGpProperties(self.covariance_matrix, self.mean_function)

    def copy(self):
        g = PredefinedGaussianProcess(self.covariance_matrix, self.mean_function)
        g.set_inducing_points(self.inducing_points)
        return g


class _SegmentedGaussianProcess(AbstractGaussianProcess):
    _WHAT = "Partitioned GP"

    def __init__(self, kernel, mean_function):
        super().__init__(kernel, mean_function)
        self.constituent_gps: List[GaussianProcess] = [GaussianProcess(cn, self.mean_function)
                                                       for cn in kernel.child_nodes]
        self.covariance_matrix = cm.SegmentedCovarianceMatrix(kernel)
        self.aux = ax.BlockwiseAuxiliaryGpProperties(self.covariance_matrix, self.mean_function)

    def set_data_input(self, data_input):
        assert len(data_input.data_inputs) == len(self.constituent_gps), \
            "Data Input does not fit constituent GPs of %s" % self._WHAT
        self.data_input = data_input
        self.covariance_matrix.set_data_input(data_input)
        self.aux.set_data_input(data_input)
        for sub, di in zip(self.constituent_gps, data_input.data_inputs):
            sub.set_data_input(di)

    def copy(self):
        g = type(self)(self.kernel, self.mean_function)
        g.set_inducing_points(self.inducing_points)
        return g


class BlockwiseGaussianProcess(_SegmentedGaussianProcess):
    """Globally segmented GP over a ChangePointOperator (GaussianProcess.py:146-175)."""
    _WHAT = "blockwise GP"


class PartitionedGaussianProcess(_SegmentedGaussianProcess):
    """GP over a PartitionOperator (GaussianProcess.py:178-206)."""
    _WHAT = "Partitioned GP"
