"""Constant / zero mean functions (gpbasics/MeanFunctionBasics/BaseMeanFunctions.py:12-79).

Only the zero mean is on the hot path: detrending with it is the identity
(gpbasics/DataHandling/DataInput.py:253-254), so y reaches the factorisation untouched.
The linear / exponential / logit means and the mean-function operators are O(N) host work,
out of scope.
"""
from __future__ import annotations

from typing import List

import torch

from .. import global_parameters as global_param
from . import MeanFunction as mf

global_param.ensure_init()


class BaseMeanFunction(mf.MeanFunction):
    def __init__(self, manifestation, input_dimensionality: int):
        super().__init__(mf.MeanFunctionType.BASE_MEAN_FUNCTION, manifestation, input_dimensionality)

    def get_number_base_mean_function(self) -> int:
        return 1

    def set_last_hyper_parameter(self, last_hyper_parameter: List):
        assert len(last_hyper_parameter) == self.get_number_of_hyper_parameter(), \
            "Wrong size/shape of given 'last_hyper_param'"
        self.last_hyper_parameter = last_hyper_parameter

    def get_number_of_hyper_parameter(self) -> int:
        return len(self.get_default_hyper_parameter())

    def get_string_representation(self) -> str:
        return self.manifestation.name

    def get_string_representation_weight(self) -> int:
        return self.manifestation.value - 100


class ConstantMeanFunction(BaseMeanFunction):
    """m(x) = c for every row of x (BaseMeanFunctions.py:37-63)."""

    def __init__(self, input_dimensionality: int):
        super().__init__(mf.MeanFunctionManifestation.C, input_dimensionality)

    def get_tf_tensor(self, hyper_parameter: List, x_vector) -> torch.Tensor:
        assert x_vector is not None, "Input vector x uninitialized: " + str(self)
        assert len(hyper_parameter) == self.get_number_of_hyper_parameter(), "Invalid hyper_param size: " + str(self)
        from ..engine import device
        c = torch.as_tensor(hyper_parameter[0], dtype=torch.float64).to(device())
        self.last_hyper_parameter = hyper_parameter
        return torch.zeros(x_vector.shape[0], dtype=torch.float64, device=device()) + c

    def get_default_hyper_parameter(self) -> List:
        return [torch.tensor(0.01, dtype=torch.float64)]

    def get_hyper_parameter_dimensionalities(self) -> List[list]:
        return [[]]

    def deepcopy(self):
        c = type(self)(self.input_dimensionality)
        c.set_last_hyper_parameter(self.last_hyper_parameter)
        return c


class ZeroMeanFunction(ConstantMeanFunction):
    """m(x) = 0 (BaseMeanFunctions.py:66-79)."""

    def get_string_representation(self) -> str:
        return "ZERO_MEAN"

    def get_default_hyper_parameter(self) -> List:
        return [torch.tensor(0.0, dtype=torch.float64)]

    def deepcopy(self):
        return ZeroMeanFunction(self.input_dimensionality)
