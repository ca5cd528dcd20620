"""Structured kernel interpolation (gpbasics/Metrics/StructuredKernelInterpolation.py:10-62) on the
device.

    K_ski = (W K_mm) W^T + noise I                                        (:10-28)

with the inducing inputs x_train[linspace(0, n, m, endpoint=False)] (m = n_inducting_train) and the
interpolation weights of get_weight_matrix (:31-49, gpk_ski_weights: the reference's expanded-norm
euclidean distances, ties included).  The products are gpk_dgemm, the noise gpk_add_diagonal.

get_approx_logdet (:52-62) is not called by any metric in the reference; it is provided with the
eigenvalues from gpk_syevj (tf.linalg.eigvals of the symmetric K_mm)."""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from .. import engine


def _check_noise(noise) -> float:
    if noise is None:
        raise Exception("SKI: Invalid noise")
    t = noise if isinstance(noise, torch.Tensor) else torch.as_tensor(noise, dtype=torch.float64)
    if t.dim() != 0:
        raise Exception("SKI: Invalid noise")
    return float(t)


def get_ski_matrix(hyper_parameter: List, data_input, kernel, noise) -> torch.Tensor:
    nv = _check_noise(noise)
    n, m = int(data_input.n_train), int(data_input.n_inducting_train)
    indices = np.linspace(start=0, stop=n, num=m, endpoint=False, dtype=int)
    z = data_input.get_inducting_x_train(torch.as_tensor(indices, dtype=torch.int64))
    k_mm = kernel.get_tf_tensor(hyper_parameter, z, z).contiguous()
    w = get_weight_matrix(data_input)
    k_ski = engine.dgemm(engine.dgemm(w, k_mm), w, trans_b=True)
    return engine.add_diagonal(k_ski, nv)


def get_weight_matrix(data_input) -> torch.Tensor:
    return engine.ski_weights(data_input.data_x_train, data_input.inducting_x_train)


def get_approx_logdet(K_mm, n, m, noise) -> torch.Tensor:
    nv = _check_noise(noise)
    lam, _, _ = engine.eigh(engine.as_device_f64(K_mm))
    return (n / m) * torch.sum(torch.log((n / m) * lam + nv))
