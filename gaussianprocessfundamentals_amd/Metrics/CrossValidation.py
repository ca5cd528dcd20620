"""Cross-validated metrics (gpbasics/Metrics/CrossValidation.py:16-134).

Folds are drawn exactly as the reference draws them -- ``np.random.shuffle`` of the record
indices with numpy's global generator, then consecutive test slices of round(n * test_ratio)
records (CrossValidation.py:16-44) -- so a seeded numpy yields the reference's folds.  The
reference then evaluates the metric fold after fold; here every fold of a holistic GP is one
member of ONE ragged device factorisation (the folds are independent problems of (nearly) equal
size), with the test points as extra rows when the metric needs the posterior mean.  Blockwise
metrics evaluate fold after fold, each fold itself one ragged batch over its segments.
"""
from __future__ import annotations

import math
import typing
from typing import List

import numpy as np
import torch

from .. import global_parameters as global_param
from ..DataHandling import DataInput as di
from . import Auxiliary as met_aux
from . import MatrixHandlingTypes as mht
from . import Metrics as met

global_param.ensure_init()


def get_data_inputs(data_input, test_ratio: float = 0.2) -> List:
    """floor(1 / test_ratio) train / test splits of the training data (CrossValidation.py:16-44)."""
    n_samples = data_input.n_train
    idx_test = 0
    n_test = int(round(n_samples * test_ratio))
    epochs = int(np.floor(1 / test_ratio))
    indices = np.linspace(start=0, num=n_samples, stop=n_samples, endpoint=False, dtype=int)
    np.random.shuffle(indices)
    out = []
    for _ in range(epochs):
        stop = n_test + idx_test
        te = sorted(indices[idx_test:stop])
        tr = sorted(np.concatenate([indices[:idx_test], indices[stop:]]))
        dev = data_input.data_x_train.device
        tr_t = torch.as_tensor(np.asarray(tr, dtype=np.int64), device=dev)
        te_t = torch.as_tensor(np.asarray(te, dtype=np.int64), device=dev)
        fold = di.DataInput(data_input.data_x_train[tr_t], data_input.data_y_train[tr_t],
                            data_input.data_x_train[te_t], data_input.data_y_train[te_t])
        fold.set_mean_function(data_input.mean_function)
        out.append(fold)
        idx_test += n_test
    return out


class CrossValidation:
    def __init__(self, gaussian_process, data_input, local_approx, numerical_matrix_handling,
                 subset_size: int = None, metric_type: met.MetricType = met.MetricType.MSE, random_restarts: int = 1):
        from ..Statistics import GaussianProcess as gp
        self.metric_type = metric_type
        self.local_approx = local_approx
        self.numerical_matrix_handling = numerical_matrix_handling
        self.subset_size = subset_size
        if self.local_approx is not mht.MatrixApproximations.NONE and self.subset_size is None:
            self.subset_size = int(data_input.n_train * global_param.p_nystroem_ratio)
        if isinstance(gaussian_process, gp.GaussianProcess):
            self.gaussian_process = gp.GaussianProcess(gaussian_process.kernel.deepcopy(),
                                                       gaussian_process.mean_function.deepcopy())
        else:
            self.gaussian_process = gp.BlockwiseGaussianProcess(gaussian_process.kernel.deepcopy(),
                                                                gaussian_process.mean_function.deepcopy())
        self.data_input = data_input
        self.random_restarts = max(1, random_restarts)

    def cross_validation(self, test_ratio: float = 0.2) -> float:
        from ..Statistics import GaussianProcess as gp
        segmented = isinstance(self.gaussian_process, (gp.BlockwiseGaussianProcess, gp.PartitionedGaussianProcess))
        if self.metric_type.value >= 10 and isinstance(self.data_input, di.PartitionedDataInput) and segmented:
            folds = self.get_partitioned_data_inputs(self.data_input, test_ratio)
        else:
            folds = get_data_inputs(self.data_input, test_ratio)
        kernel = self.gaussian_process.kernel
        hyp, noise = kernel.get_last_hyper_parameter(), kernel.get_noise()
        if isinstance(self.gaussian_process, gp.GaussianProcess) and self.metric_type in (
                met.MetricType.LL, met.MetricType.BIC, met.MetricType.MSE) and \
                self.local_approx is mht.MatrixApproximations.NONE and \
                self.numerical_matrix_handling is mht.NumericalMatrixHandlingType.CHOLESKY_BASED:
            return float(np.mean(self.batched_fold_metrics(folds, hyp, noise)))
        results: typing.List[float] = []
        for fold in folds:
            self.gaussian_process.set_data_input(fold)
            metric = met_aux.get_metric_by_type(self.metric_type, self.gaussian_process, local_approx=self.local_approx,
                                                numerical_matrix_handling=self.numerical_matrix_handling,
                                                subset_size=self.subset_size)
            results.append(float(metric.get_metric(hyp, noise)))
        return float(np.mean(results))

    def batched_fold_metrics(self, folds, hyper_parameter, noise) -> List[float]:
        """The metric of every fold from ONE ragged factorisation (one member per fold)."""
        from ..Statistics.CovarianceMatrix import factor_segments
        kernel = self.gaussian_process.kernel
        need_mu = self.metric_type is met.MetricType.MSE
        f, index = factor_segments([kernel] * len(folds), [list(hyper_parameter)] * len(folds), folds, noise,
                                   with_test=need_mu)
        out = []
        if self.metric_type is met.MetricType.MSE:
            f.check_info()
            for j, fold in enumerate(folds):
                mu = f.posterior_mu(j).reshape(-1, 1)
                yt = fold.get_detrended_y_test().reshape(-1, 1).to(torch.float64)
                out.append(float(torch.mean((mu - yt) ** 2)))
            return out
        nl = f.nlml().detach().cpu().tolist()
        for j, fold in enumerate(folds):
            if self.metric_type is met.MetricType.LL:
                out.append(nl[j])
            else:  # BIC (BayesianInformationCriterion.py:27-38)
                out.append(2.0 * nl[j] + kernel.get_number_of_hyper_parameter() * math.log(fold.n_train))
        return out

    def get_partitioned_data_inputs(self, partitioned_data_input, test_ratio: float = 0.2):
        """Folds of every partition, zipped into one PartitionedDataInput per fold
        (CrossValidation.py:96-134)."""
        per_partition = []
        n_inputs = -1
        for d in partitioned_data_input.data_inputs:
            inputs = get_data_inputs(d, test_ratio)
            if n_inputs == -1:
                n_inputs = len(inputs)
            else:
                assert len(inputs) == n_inputs, \
                    "All data_inputs of partitioned data inputs need to have the same amount of permutations"
            per_partition.append(inputs)
        out = []
        for i in range(n_inputs):
            parts = [p[i] for p in per_partition]
            pdi = di.PartitionedDataInput(torch.cat([p.data_x_train for p in parts]),
                                          torch.cat([p.data_y_train for p in parts]),
                                          torch.cat([p.data_x_test for p in parts]),
                                          torch.cat([p.data_y_test for p in parts]), parts)
            pdi.set_mean_function(self.data_input.mean_function)
            out.append(pdi)
        return out
