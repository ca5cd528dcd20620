"""Kernel plugin interface (gpbasics/KernelBasics/Kernel.py).

``Kernel.get_tf_tensor(hyper_parameter, x_vector, x_vector_)`` keeps the reference's name and
argument meaning (K/Kernel.py:51-52) and returns an [n, m] fp64 device tensor computed by the
HIP kernel-matrix build (libgpk ``gpk_kernel_matrix``); ``get_tensor`` is an alias.
Subclasses add ``_emit``: the flattening of the tree into the device's postfix program.
"""
from __future__ import annotations

from enum import Enum
from typing import List

import torch

from ..Auxiliary import BasicGPComponent as bgpc


# enum values follow the reference (K/Kernel.py:10-37); built functionally
ConstantHyperParamType = Enum("ConstantHyperParamType", {"NONE_CONSTANT": 0, "JUST_CONSTANT_BASE_KERNELS": 1,
                                                         "JUST_CONSTANT_CP": 2, "ALL_CONSTANT": 3})
KernelType = Enum("KernelType", {"BASE_KERNEL": 1, "OPERATOR": 2})
KernelManifestation = Enum("KernelManifestation", dict(
    C=101, LIN=102, RQ=103, PER=104, SE=105, WN=106, MAT32=107, MAT52=108, ADD=201, MUL=202, CP=203, PART=204))


def _abstract(obj, name):
    return NotImplementedError("%s.%s is provided by the concrete kernel" % (type(obj).__name__, name))


class Kernel(bgpc.Component):
    """Abstract kernel: a node of a kernel expression tree."""

    def __init__(self, kernel_type: KernelType, manifestation: KernelManifestation, input_dimensionality: int):
        assert input_dimensionality >= 1, "input_dimensionality for a kernel ought to be one or larger"
        self.kernel_type = kernel_type
        self.manifestation = manifestation
        self.last_hyper_parameter = None
        self.input_dimensionality = input_dimensionality
        self.noise = None

    # -- evaluation -------------------------------------------------------------------------
    def get_tf_tensor(self, hyper_parameter: List, x_vector, x_vector_) -> torch.Tensor:
        assert x_vector is not None and x_vector_ is not None, "Input vectors x and x_ uninitialized: " + str(self)
        assert len(hyper_parameter) == self.get_number_of_hyper_parameter(), "Invalid hyper_param size: " + str(self)
        from .. import engine
        K = engine.kernel_matrix(self, hyper_parameter, x_vector, x_vector_)
        self._record_hyper_parameter(list(hyper_parameter))
        return K

    get_tensor = get_tf_tensor

    def _record_hyper_parameter(self, hyper_parameter: List):
        """The reference's get_tf_tensor stores its argument in last_hyper_parameter."""
        self.last_hyper_parameter = hyper_parameter

    def _emit(self, nodes: list, offset: int, ard_slots: list, dim: int) -> int:
        raise NotImplementedError("%s has no device form" % type(self).__name__)

    # -- tree / hyperparameter plumbing -----------------------------------------------------
    def get_kernel_type(self) -> KernelType:
        return self.kernel_type

    def get_kernel_manifestation(self) -> KernelManifestation:
        return self.manifestation

    def get_number_of_hyper_parameter(self) -> int:
        raise _abstract(self, 'get_number_of_hyper_parameter')

    def get_string_representation(self) -> str:
        raise _abstract(self, 'get_string_representation')

    def get_number_base_kernels(self) -> int:
        raise _abstract(self, 'get_number_base_kernels')

    def get_default_hyper_parameter(self, xrange: List[List[float]], n: int, from_distribution: bool = False) -> List:
        raise _abstract(self, 'get_default_hyper_parameter')

    def set_last_hyper_parameter(self, last_hyper_parameter: List):
        raise _abstract(self, 'set_last_hyper_parameter')

    def get_last_hyper_parameter(self, scaling_x_param=None):
        raise _abstract(self, 'get_last_hyper_parameter')

    def set_noise(self, noise):
        """noise must be a rank-0 value (K/Kernel.py:79-83)."""
        if torch.as_tensor(noise).shape == torch.Size([]):
            self.noise = noise
        else:
            raise Exception("Invalid Noise set for Kernel")

    def get_noise(self):
        return self.noise

    def deepcopy(self):
        raise _abstract(self, 'deepcopy')

    def get_string_representation_weight(self) -> float:
        return 0

    def sort_child_nodes(self):
        pass

    def get_json(self) -> dict:
        raise _abstract(self, 'get_json')

    def get_number_of_child_nodes(self) -> int:
        raise _abstract(self, 'get_number_of_child_nodes')

    def get_derivative_matrices(self, hyper_parameter: List, x_vector, x_vector_) -> List:
        # not rebuilt: nothing in the reference calls them (its fitter differentiates through
        # tf.linalg.cholesky), SE's is wrong (K/BaseKernels.py:383-399), and the LML gradient is computed by
        # the fused device pass of gpk_nlml_grad without any dK/dtheta matrix (LogLikelihood.get_metric_and_gradient)
        raise NotImplementedError("analytic derivative matrices are not provided: use "
                                  "LogLikelihood.get_metric_and_gradient or autograd through get_metric")

    def get_hyper_parameter_names(self, kernel_id: int = -1) -> List[str]:
        raise _abstract(self, 'get_hyper_parameter_names')

    def get_dimensionality(self):
        return self.input_dimensionality

    def set_dimensionality(self, input_dimensionality: int):
        self.input_dimensionality = input_dimensionality

    def get_simplified_version(self):
        return self

    def type_compare_to(self, other):
        return self == other

    def get_hash_tuple(self):
        flat = []
        if isinstance(self.last_hyper_parameter, list):
            for h in self.last_hyper_parameter:
                v = torch.as_tensor(h).detach().reshape(-1).tolist()
                flat.extend(float(x) for x in v)
        noise = None if self.noise is None else float(torch.as_tensor(self.noise, dtype=torch.float64))
        return self.manifestation.value, noise, tuple(flat)

    def __hash__(self):
        return hash(self.get_hash_tuple())
