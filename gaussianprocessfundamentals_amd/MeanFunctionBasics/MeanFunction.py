"""Mean-function interface (gpbasics/MeanFunctionBasics/MeanFunction.py)."""
from __future__ import annotations

from enum import Enum
from typing import List

from ..Auxiliary import BasicGPComponent as bgpc

MeanFunctionType = Enum("MeanFunctionType", {"BASE_MEAN_FUNCTION": 1, "OPERATOR": 2})
MeanFunctionManifestation = Enum("MeanFunctionManifestation",
                                 dict(C=101, LIN=102, EXP=103, LOGIT=104, ADD=201, MUL=202, CP=203))


class MeanFunction(bgpc.Component):
    def __init__(self, mean_function_type, manifestation, input_dimensionality: int):
        assert input_dimensionality >= 1, "input_dimensionality for a mean function ought to be 1 or larger"
        self.type = mean_function_type
        self.manifestation = manifestation
        self.last_hyper_parameter = None
        self.input_dimensionality = input_dimensionality

    def get_tf_tensor(self, hyper_parameter: List, x_vector):
        raise NotImplementedError

    def get_mean_function_type(self):
        return self.type

    def get_mean_function_manifestation(self):
        return self.manifestation

    def get_last_hyper_parameter(self):
        return self.last_hyper_parameter

    def set_last_hyper_parameter(self, last_hyper_parameter: List):
        self.last_hyper_parameter = last_hyper_parameter

    def get_default_hyper_parameter(self) -> List:
        raise NotImplementedError
