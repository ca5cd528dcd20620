"""Metric factory (gpbasics/Metrics/Auxiliary.py:13-51)."""
from __future__ import annotations

import logging

from . import MatrixHandlingTypes as mht
from .LogLikelihood import LogLikelihood
from .Metrics import MetricType


def get_metric_by_type(metric_type: MetricType, _gp,
                       local_approx: mht.GlobalApproximationsType = mht.MatrixApproximations.NONE,
                       numerical_matrix_handling: mht.NumericalMatrixHandlingType =
                       mht.NumericalMatrixHandlingType.CHOLESKY_BASED,
                       subset_size: int = None):
    """MetricType.LL -> LogLikelihood over the GP's covariance matrix (default CHOLESKY_BASED,
    Auxiliary.py:16).  BIC / MSE / blockwise metrics are SURVEY §8f 'next'."""
    if metric_type is MetricType.LL:
        return LogLikelihood(_gp.data_input, _gp.covariance_matrix, local_approx, numerical_matrix_handling, subset_size)
    if metric_type in (MetricType.BIC, MetricType.MSE, MetricType.blockwise_LL, MetricType.blockwise_BIC,
                       MetricType.blockwise_MSE):
        raise NotImplementedError("metric %s is SURVEY §8f 'next'" % metric_type)
    logging.error("Invalid MetricType: %s" % str(metric_type))
    return None


def get_blockwise_metric_for_standard_metric(metric_type: MetricType) -> MetricType:
    mapping = {MetricType.LL: MetricType.blockwise_LL, MetricType.BIC: MetricType.blockwise_BIC,
               MetricType.MSE: MetricType.blockwise_MSE}
    if metric_type.value >= 10:
        logging.warning("get_blockwise_metric_for_standard_metric received blockwise metric and thus had no effect.")
        return metric_type
    return mapping.get(metric_type, metric_type)
