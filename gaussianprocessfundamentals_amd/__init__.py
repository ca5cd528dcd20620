"""gaussianprocessfundamentals_amd -- an MI355X-native exact-GP likelihood engine.

A drop-in for the hot path of gpbasics (Bernsai/GaussianProcessFundamentals): the module layout
and the class / method names of the kernel, covariance-matrix, metric and GP plugins are kept
(``KernelBasics.BaseKernels``, ``KernelBasics.Operators``, ``Statistics.CovarianceMatrix``,
``Statistics.GaussianProcess``, ``Metrics.LogLikelihood``, ``Metrics.Auxiliary``,
``DataHandling.DataInput``, ``MeanFunctionBasics.BaseMeanFunctions``), while every matrix is
built, factored and solved by hand-written HIP for gfx950 in ``libgpk.so`` behind the C ABI of
``include/gpk.h``.  There is no CPU fallback.

Usage mirrors the reference::

    import gaussianprocessfundamentals_amd.global_parameters as gp
    gp.init(0)                                   # before importing the other modules
    from gaussianprocessfundamentals_amd.KernelBasics.BaseKernels import SquaredExponentialKernel
    ...

``install_gpbasics_alias()`` additionally registers the package under the name ``gpbasics`` so
that unmodified ``import gpbasics.…`` statements resolve to it.
"""
from __future__ import annotations

import importlib
import sys

__version__ = "0.1.0"

_SUBMODULES = (
    "global_parameters", "engine", "sweep",
    "Auxiliary", "Auxiliary.BasicGPComponent", "Auxiliary.Distances", "Auxiliary.LinearConjugateGradients",
    "KernelBasics", "KernelBasics.Kernel", "KernelBasics.BaseKernels", "KernelBasics.Operators",
    "KernelBasics.PartitioningModel", "KernelBasics.PartitionOperator",
    "MeanFunctionBasics", "MeanFunctionBasics.MeanFunction", "MeanFunctionBasics.BaseMeanFunctions",
    "DataHandling", "DataHandling.DataInput", "DataHandling.AbstractDataInput", "DataHandling.BatchDataInput",
    "Statistics", "Statistics.CovarianceMatrix", "Statistics.Auxiliary", "Statistics.GaussianProcess", "Statistics.ApproximationType",
    "Metrics", "Metrics.MatrixHandlingTypes", "Metrics.Metrics", "Metrics.LogLikelihood", "Metrics.Auxiliary",
    "Metrics.BayesianInformationCriterion", "Metrics.MeanSquaredError", "Metrics.CrossValidation",
)


def install_gpbasics_alias():
    """Make ``import gpbasics.X`` resolve to ``gaussianprocessfundamentals_amd.X`` (call after
    ``global_parameters.init``)."""
    sys.modules.setdefault("gpbasics", sys.modules[__name__])
    for name in _SUBMODULES:
        mod = importlib.import_module(__name__ + "." + name)
        sys.modules.setdefault("gpbasics." + name, mod)
