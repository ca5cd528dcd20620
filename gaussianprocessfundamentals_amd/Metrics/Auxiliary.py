"""Metric factory (gpbasics/Metrics/Auxiliary.py:13-66)."""
from __future__ import annotations

import logging

from . import MatrixHandlingTypes as mht
from .BayesianInformationCriterion import BIC, BlockwiseBIC
from .LogLikelihood import BlockwiseLogLikelihood, LogLikelihood
from .MeanSquaredError import BlockwiseMeanSquaredError, MeanSquaredError
from .Metrics import MetricType


def get_metric_by_type(metric_type: MetricType, _gp,
                       local_approx: mht.GlobalApproximationsType = mht.MatrixApproximations.NONE,
                       numerical_matrix_handling: mht.NumericalMatrixHandlingType =
                       mht.NumericalMatrixHandlingType.CHOLESKY_BASED,
                       subset_size: int = None):
    """Metric object for ``metric_type`` over ``_gp`` (default CHOLESKY_BASED, Auxiliary.py:16);
    SKC_UPPER_BOUND gives the Nystroem upper bound of Metrics/SkcLogLikelihood.py."""
    from ..Statistics import GaussianProcess as gp
    if metric_type is MetricType.LL:
        if local_approx is mht.MatrixApproximations.SKC_UPPER_BOUND:                          # :19-22
            from ..Statistics.Nystroem_K import NystroemMatrix
            from .SkcLogLikelihood import LogLikelihoodUpperBound
            nyk = NystroemMatrix(_gp.covariance_matrix)
            nyk.set_data_input(_gp.data_input)
            return LogLikelihoodUpperBound(_gp.data_input, _gp.covariance_matrix, nystroem_k=nyk)
        return LogLikelihood(_gp.data_input, _gp.covariance_matrix, local_approx, numerical_matrix_handling,
                             subset_size)
    if metric_type is MetricType.BIC:
        ll = LogLikelihood(_gp.data_input, _gp.covariance_matrix, local_approx, numerical_matrix_handling, subset_size)
        return BIC(_gp.data_input, _gp.covariance_matrix, ll)
    if metric_type is MetricType.MSE:
        return MeanSquaredError(_gp.data_input, _gp.covariance_matrix, _gp.aux, local_approx,
                                numerical_matrix_handling, subset_size)
    segmented = isinstance(_gp, (gp.BlockwiseGaussianProcess, gp.PartitionedGaussianProcess))
    if metric_type is MetricType.blockwise_MSE:
        assert segmented, "Blockwise MSE may only be determined for blockwise Gaussian Process."
        return BlockwiseMeanSquaredError(_gp, local_approx, numerical_matrix_handling, subset_size)
    if metric_type is MetricType.blockwise_BIC:
        assert segmented, "Blockwise BIC may only be determined for blockwise Gaussian Process."
        return BlockwiseBIC(_gp, local_approx, numerical_matrix_handling, subset_size)
    if metric_type is MetricType.blockwise_LL:
        assert segmented, "Blockwise Log Likelihood may only be determined for blockwise Gaussian Process."
        return BlockwiseLogLikelihood(_gp, local_approx, numerical_matrix_handling, subset_size)
    logging.error("Invalid MetricType: %s" % str(metric_type))
    return None


def get_blockwise_metric_for_standard_metric(metric_type: MetricType) -> MetricType:
    if metric_type.value >= 10:
        logging.warning("get_blockwise_metric_for_standard_metric received blockwise metric and thus had no effect.")
        return metric_type
    mapping = {MetricType.LL: MetricType.blockwise_LL, MetricType.BIC: MetricType.blockwise_BIC,
               MetricType.MSE: MetricType.blockwise_MSE}
    if metric_type not in mapping:
        logging.warning("There is no blockwise version for metric %s." % str(metric_type))
    return mapping.get(metric_type, metric_type)
