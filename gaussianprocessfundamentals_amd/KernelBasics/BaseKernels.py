"""Base kernels SE / PER / MAT32 / MAT52 (gpbasics/KernelBasics/BaseKernels.py) on the device.

One table-driven class body serves the four kernels on the hot path; each subclass only states
its op code, its shape hyperparameters and its string name.  Semantics (formulae, DFS
hyperparameter order, default values, bounds, names, |l| normalisation in
``set_last_hyper_parameter``) follow the reference:

  SE     hyp [l, (sg)]      BaseKernels.py:272-432
  PER    hyp [l, p, (sg)]   BaseKernels.py:435-634
  MAT32  hyp [l, (sg)]      BaseKernels.py:697-851
  MAT52  hyp [l, (sg)]      BaseKernels.py:854-1011

``sg`` exists only when ``global_parameters.p_scaled_base_kernel`` is True.

Build extension: ``ard=True`` on SE / MAT32 / MAT52 makes the length scale a vector
of ``input_dimensionality`` values; the kernel then equals the reference kernel with l = 1 on
inputs divided elementwise by that vector.

Build option (``standard=True`` per kernel, or ``global_parameters.p_stationary_distance =
"standard"``): Matern kernels on the Euclidean distance and PER as the per-dimension product
exp(-2 sum_d sin^2(pi |x_d - y_d| / p) / l^2).  Both equal the reference's L1 forms
(BaseKernels.py:446, :708, :865) when D == 1; for D > 1 those L1 forms are not positive
definite (their Cholesky fails on the SURVEY C3 / C5 inputs).  The default stays the reference form.

Out of scope: LinearKernel, ConstantKernel (raises in the reference), WhiteNoiseKernel.
"""
from __future__ import annotations

import logging
import math
from typing import List, Tuple

import torch

from .. import _native as nat
from .. import global_parameters as global_param
from . import Kernel as k

global_param.ensure_init()


def _abs_tensor(h):
    return torch.abs(torch.as_tensor(h, dtype=torch.float64))


class BaseKernel(k.Kernel):
    # per-kernel table (set by subclasses)
    _OP: int = 0
    _SHAPE: Tuple[str, ...] = ("l",)      # shape hyperparameters, in reference order
    _ARD_CAPABLE: bool = True

    def __init__(self, manifestation, input_dimensionality: int, ard: bool = False, standard=None):
        super().__init__(k.KernelType.BASE_KERNEL, manifestation, input_dimensionality)
        if self.manifestation.value > 199:
            logging.critical("Invalid manifestation for BaseKernel: %s", manifestation)
        if ard and not self._ARD_CAPABLE:
            raise ValueError("%s has no ARD form" % type(self).__name__)
        self.ard = bool(ard)
        # None: follow global_parameters.p_stationary_distance at evaluation time
        self.standard = standard
        self.latest_cov_mat = None

    def uses_standard_form(self) -> bool:
        if self._OP == nat.OP_SE:
            return False
        if self.standard is None:
            return global_param.p_stationary_distance == "standard"
        return bool(self.standard)

    # -- device program -----------------------------------------------------------------------
    def _emit(self, nodes: list, offset: int, ard_slots: list, dim: int) -> int:
        flags = 0
        if global_param.p_scaled_base_kernel:
            flags |= nat.NODE_SCALED
        slot = -1
        if self.ard:
            flags |= nat.NODE_ARD
            slot = len(ard_slots)
            ard_slots.append(offset)
        if self._OP == nat.OP_SE and global_param.p_se_expanded_norm:
            flags |= nat.NODE_SE_EXPANDED
        if self.uses_standard_form():
            flags |= nat.NODE_STANDARD
        nodes.append((self._OP, offset, slot, flags))
        return offset + self._n_values(dim)

    def _n_values(self, dim: int) -> int:
        n = len(self._SHAPE) + (dim - 1 if self.ard else 0)
        return n + (1 if global_param.p_scaled_base_kernel else 0)

    # -- hyperparameters ----------------------------------------------------------------------
    def get_number_base_kernels(self) -> int:
        return 1

    def get_number_of_child_nodes(self) -> int:
        return 1

    def get_number_of_hyper_parameter(self) -> int:
        return len(self._SHAPE) + (1 if global_param.p_scaled_base_kernel else 0)

    def get_hyper_parameter_dimensionalities(self) -> List[list]:
        dims = [[self.input_dimensionality] if (self.ard and name == "l") else [] for name in self._SHAPE]
        if global_param.p_scaled_base_kernel:
            dims.append([])
        return dims

    def _shape_value(self, name, width):
        return torch.full([self.input_dimensionality] if (self.ard and name == "l") else [],
                          width / 10.0, dtype=torch.float64)

    def get_default_hyper_parameter(self, xrange: List[List[float]], n: int, from_distribution: bool = False):
        """Fixed defaults: every shape parameter = range width / 10, sg = 0.1
        (e.g. BaseKernels.py:323-332, :490-501); random defaults draw |N(width/10, 0.2)|
        (:334-350), with torch's generator instead of TensorFlow's."""
        width = xrange[0][1] - xrange[0][0]
        if from_distribution:
            out = []
            for name in self._SHAPE:
                shape = [self.input_dimensionality] if (self.ard and name == "l") else []
                if name == "p":
                    avg = min(r[1] - r[0] for r in xrange) / n
                    out.append(torch.empty(shape, dtype=torch.float64).uniform_(avg * 5, avg * (n / 2)))
                else:
                    out.append(torch.abs(torch.normal(width / 10.0, 0.2, size=shape, dtype=torch.float64)))
            if global_param.p_scaled_base_kernel:
                out.append(torch.abs(torch.normal(0.1, 0.2, size=[], dtype=torch.float64)))
            return out
        out = [self._shape_value(name, width) for name in self._SHAPE]
        if global_param.p_scaled_base_kernel:
            out.append(torch.tensor(0.1, dtype=torch.float64))
        return out

    def get_default_hyper_parameter_fixed(self, xrange: List[List[float]], n: int) -> List:
        """The fixed branch of get_default_hyper_parameter (e.g. BaseKernels.py:323-332)."""
        return self.get_default_hyper_parameter(xrange, n, from_distribution=False)

    def get_default_hyper_parameter_distribution(self, xrange: List[List[float]], n: int) -> List:
        """The random branch of get_default_hyper_parameter (e.g. BaseKernels.py:334-350)."""
        return self.get_default_hyper_parameter(xrange, n, from_distribution=True)

    def get_hyper_parameter_distribution_definition(self, xrange: List[List[float]], n: int) -> List[dict]:
        width = xrange[0][1] - xrange[0][0]
        out = []
        for dim, name in zip(self.get_hyper_parameter_dimensionalities(), self._SHAPE):
            if name == "p":
                avg = min(r[1] - r[0] for r in xrange) / n
                out.append({"shape": dim, "minval": avg * 5, "maxval": avg * (n / 2), "type": "random_uniform"})
            else:
                out.append({"shape": dim, "mean": width / 10, "stddev": 0.2, "type": "random_normal"})
        if global_param.p_scaled_base_kernel:
            out.append({"shape": [], "mean": 0.1, "stddev": 0.2, "type": "random_normal"})
        return out

    def get_hyper_parameter_bounds(self, xrange: List[List[float]], n: int) -> List[tuple]:
        """l in [5 range / n, range / 3]; PER p in [log(10 range / n), log(range / 5)];
        sg in [100 jitter, inf) (BaseKernels.py:296-306, :459-473)."""
        rl = xrange[0][1] - xrange[0][0]
        f64 = torch.float64
        out = []
        for name in self._SHAPE:
            if name == "p":
                out.append((torch.tensor(math.log(10 * (rl / n)), dtype=f64), torch.tensor(math.log(rl / 5), dtype=f64)))
            else:
                out.append((torch.tensor(5 * rl / n, dtype=f64), torch.tensor(rl / 3, dtype=f64)))
        if global_param.p_scaled_base_kernel:
            jit = float(torch.as_tensor(global_param.p_cov_matrix_jitter))
            out.append((torch.tensor(jit * 100, dtype=f64), torch.tensor(math.inf, dtype=f64)))
        return out

    def get_hyper_parameter_names(self, kernel_id: int = -1) -> List[str]:
        rep = self.get_string_representation() + ("_%i" % kernel_id if kernel_id >= 0 else "")
        names = [rep + "_" + s for s in self._SHAPE]
        if global_param.p_scaled_base_kernel:
            names.append(rep + "_sg")
        return names

    def set_last_hyper_parameter(self, last_hyper_parameter: List):
        if not isinstance(last_hyper_parameter, list):
            raise Exception("Wrong type for last_hyper_parameter to be set!")
        assert len(last_hyper_parameter) == self.get_number_of_hyper_parameter(), "Invalid hyper_param size: %s" % str(self)
        hp = list(last_hyper_parameter)
        # length scale (and PER's period) are stored as absolute values (BaseKernels.py:429-432, :629-634)
        for i, name in enumerate(self._SHAPE):
            hp[i] = _abs_tensor(hp[i])
        self.last_hyper_parameter = hp

    def get_last_hyper_parameter(self, scaling_x_param=None):
        result = self.last_hyper_parameter
        if scaling_x_param is None or result is None:
            return result
        out = [result[i] * scaling_x_param[1] for i in range(len(self._SHAPE))]
        if global_param.p_scaled_base_kernel:
            out.append(result[len(self._SHAPE)])
        return out

    # -- misc ---------------------------------------------------------------------------------
    def get_string_representation(self) -> str:
        return self.manifestation.name

    def get_string_representation_weight(self) -> int:
        return self.manifestation.value - 100

    def get_json(self) -> dict:
        hp = self.get_last_hyper_parameter() or []
        return {"type": self.get_string_representation(),
                "hyper_param": [torch.as_tensor(h).tolist() for h in hp]}

    def deepcopy(self):
        c = type(self)(input_dimensionality=self.input_dimensionality, ard=self.ard, standard=self.standard)
        if self.last_hyper_parameter is not None:
            c.set_last_hyper_parameter(list(self.last_hyper_parameter))
        if self.noise is not None:
            c.set_noise(self.noise)
        return c

    def type_compare_to(self, other):
        return isinstance(other, type(self))

    def __repr__(self):
        return self.get_string_representation()


class SquaredExponentialKernel(BaseKernel):
    """exp(-0.5 * dist^2 / l^2) (BaseKernels.py:277-294)."""
    _OP = nat.OP_SE
    _SHAPE = ("l",)

    def __init__(self, input_dimensionality: int, ard: bool = False, standard=None):
        super().__init__(k.KernelManifestation.SE, input_dimensionality, ard, standard)


class PeriodicKernel(BaseKernel):
    """exp(-2 sin^2(pi d1 / p) / l^2) with the L1 distance d1 (BaseKernels.py:440-457)."""
    _OP = nat.OP_PER
    _SHAPE = ("l", "p")
    _ARD_CAPABLE = False

    def __init__(self, input_dimensionality: int, ard: bool = False, standard=None):
        super().__init__(k.KernelManifestation.PER, input_dimensionality, ard, standard)


class MaternKernel3_2(BaseKernel):
    """(1 + f) e^-f, f = sqrt(3) d1 / |l| (BaseKernels.py:702-720)."""
    _OP = nat.OP_MAT32
    _SHAPE = ("l",)

    def __init__(self, input_dimensionality: int, ard: bool = False, standard=None):
        super().__init__(k.KernelManifestation.MAT32, input_dimensionality, ard, standard)


class MaternKernel5_2(BaseKernel):
    """(1 + f + 5 d1^2 / (3 l^2)) e^-f, f = sqrt(5) d1 / |l| (BaseKernels.py:859-880)."""
    _OP = nat.OP_MAT52
    _SHAPE = ("l",)

    def __init__(self, input_dimensionality: int, ard: bool = False, standard=None):
        super().__init__(k.KernelManifestation.MAT52, input_dimensionality, ard, standard)
