"""Strategy enums of gpbasics/Metrics/MatrixHandlingTypes.py (same names and values).

Every strategy runs on the device (Metrics/Metrics.py documents the binding); the fast path is
MatrixApproximations.NONE with NumericalMatrixHandlingType.CHOLESKY_BASED.
"""
from enum import Enum


class GlobalApproximationsType(Enum):
    """Common base of the approximation enums (an empty Enum can be subclassed)."""


MatrixApproximations = GlobalApproximationsType(
    "MatrixApproximations", dict(NONE=0, SKC_LOWER_BOUND=1, SKC_UPPER_BOUND=2, BASIC_NYSTROEM=3, SKI=4))
SubsetOfDataApproaches = GlobalApproximationsType(
    "SubsetOfDataApproaches", dict(SOD_RANDOM=5, SOD_GRID=6, SOD_SMOOTHED_GRID=7))
NumericalMatrixHandlingType = Enum(
    "NumericalMatrixHandlingType",
    dict(STRICT_INVERSE=0, PSEUDO_INVERSE=1, CHOLESKY_BASED=2, LINEAR_CONJUGATE_GRADIENT=3))
