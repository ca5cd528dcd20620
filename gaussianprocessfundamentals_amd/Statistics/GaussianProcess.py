"""Gaussian process objects (gpbasics/Statistics/GaussianProcess.py:20-125).

Only the holistic :class:`GaussianProcess` is on the hot path; the blockwise / partitioned /
predefined variants are SURVEY §8f "next".
"""
from __future__ import annotations

import logging
from typing import List, Tuple

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
        post_mu = self.aux.get_posterior_mu(kernel_hyper_param, noise)
        return mean_mu + post_mu, mean_mu, post_mu

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
