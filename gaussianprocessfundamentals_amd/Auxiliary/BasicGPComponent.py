"""Component base class (gpbasics/Auxiliary/BasicGPComponent.py) with torch tensors."""
from __future__ import annotations

from typing import List, Tuple

import torch


class Component:
    def get_hyper_parameter_bounds(self, xrange: List[List[float]], n: int) -> List[Tuple]:
        pass

    def get_hyper_parameter_dimensionalities(self) -> List[list]:
        pass

    def get_hyper_parameter_distribution_definition(self, xrange: List[List[float]], n: int) -> List[dict]:
        pass

    @staticmethod
    def serialize_hyper_parameter(hyper_parameter: List) -> torch.Tensor:
        """Concatenate every hyperparameter reshaped to [-1] (BasicGPComponent.py:16-23)."""
        return torch.cat([torch.as_tensor(h, dtype=torch.float64).reshape(-1) for h in hyper_parameter])

    @staticmethod
    def deserialize_hyper_parameter(hyper_parameter: torch.Tensor, dimensionalities: List[list]) -> List:
        """Split a flat vector by dimensionalities.  Quirk kept: like the reference
        (BasicGPComponent.py:26-42) every slice starts at offset 0."""
        out = []
        for dim in dimensionalities:
            size = 1 if len(dim) == 0 else dim[0]
            out.append(hyper_parameter[0:size].reshape(dim))
        return out
