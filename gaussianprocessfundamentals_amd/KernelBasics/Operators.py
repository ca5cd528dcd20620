"""ADD / MUL kernel operators (gpbasics/KernelBasics/Operators.py:15-367).

A whole operator tree is evaluated by ONE device launch: the tree is flattened into a postfix
program whose binary ADD/MUL nodes fold the children left to right, exactly the order of the
reference's ``result = op(result, child_i)`` loops (Operators.py:214-223, :314-324).
Hyperparameters are one flat list in child DFS order, sliced by each child's
``get_number_of_hyper_parameter`` (Operators.py:28-32).

ChangePointOperator (Operators.py:370-681) splits the (1-D) input axis at its change points; its
matrix is the sum of the child matrices masked by the segment indicators, and its hyperparameters
are the change points followed by the children's.  The segmented LML path does not build that
matrix at all: SegmentedCovarianceMatrix factors the segments as one ragged device batch.
"""
from __future__ import annotations

from typing import List

import torch

from .. import _native as nat
from .. import global_parameters as global_param
from . import BaseKernels as bk
from . import Kernel as k

global_param.ensure_init()


class Operator(k.Kernel):
    _BINARY_OP = 0
    operator_sign = "UNKNOWN"

    def __init__(self, manifestation: k.KernelManifestation, input_dimensionality: int, child_nodes: List[k.Kernel]):
        super().__init__(k.KernelType.OPERATOR, manifestation, input_dimensionality)
        self.child_nodes: List[k.Kernel] = list(child_nodes)
        self.sortable = True

    # -- device program -----------------------------------------------------------------------
    def _emit(self, nodes: list, offset: int, ard_slots: list, dim: int) -> int:
        if not self.child_nodes:
            raise ValueError("operator without child nodes")
        for i, cn in enumerate(self.child_nodes):
            offset = cn._emit(nodes, offset, ard_slots, dim)
            if i > 0:
                nodes.append((self._BINARY_OP, 0, -1, 0))
        return offset

    def _slices(self, hyper_parameter: List):
        idx = 0
        for cn in self.child_nodes:
            cnt = cn.get_number_of_hyper_parameter()
            yield cn, list(hyper_parameter[idx:idx + cnt])
            idx += cnt

    def _record_hyper_parameter(self, hyper_parameter: List):
        # children record their slices, as the reference's recursive evaluation does
        for cn, sl in self._slices(hyper_parameter):
            cn._record_hyper_parameter(sl)

    # -- plumbing -----------------------------------------------------------------------------
    def get_number_of_hyper_parameter(self) -> int:
        return sum(cn.get_number_of_hyper_parameter() for cn in self.child_nodes)

    def add_kernel(self, kernel):
        self.child_nodes = self.child_nodes + [kernel]

    def replace_child_node(self, index: int, new_child_node: k.Kernel):
        assert index < len(self.child_nodes), "cannot replace child node at index %d" % index
        self.child_nodes[index] = new_child_node

    def get_number_base_kernels(self) -> int:
        return sum(cn.get_number_base_kernels() for cn in self.child_nodes)

    def get_number_of_child_nodes(self) -> int:
        return len(self.child_nodes)

    def get_string_representation(self) -> str:
        if len(self.child_nodes) == 1:
            return self.child_nodes[0].get_string_representation()
        sep = " %s " % self.operator_sign
        return "(" + sep.join(cn.get_string_representation() for cn in self.child_nodes) + ")"

    def get_string_representation_weight(self) -> int:
        return sum(cn.get_string_representation_weight() for cn in self.child_nodes)

    def get_default_hyper_parameter(self, xrange, n, from_distribution: bool = False) -> List:
        out = []
        for cn in self.child_nodes:
            out += cn.get_default_hyper_parameter(xrange, n, from_distribution)
        return out

    def get_json(self) -> dict:
        return {"type": self.manifestation.name, "child_nodes": [cn.get_json() for cn in self.child_nodes]}

    def set_last_hyper_parameter(self, last_hyper_parameter: List):
        assert len(last_hyper_parameter) == self.get_number_of_hyper_parameter(), "Invalid hyper_param size: " + str(self)
        for cn, sl in self._slices(last_hyper_parameter):
            cn.set_last_hyper_parameter(sl)

    def get_last_hyper_parameter(self, scaling_x_param=None):
        out = []
        for cn in self.child_nodes:
            hp = cn.get_last_hyper_parameter(scaling_x_param)
            if hp is None:
                return None
            out.extend(hp)
        return out

    def get_hyper_parameter_bounds(self, xrange, n) -> List[tuple]:
        return [b for cn in self.child_nodes for b in cn.get_hyper_parameter_bounds(xrange, n)]

    def get_hyper_parameter_dimensionalities(self) -> List[list]:
        return [d for cn in self.child_nodes for d in cn.get_hyper_parameter_dimensionalities()]

    def get_hyper_parameter_distribution_definition(self, xrange, n) -> List[dict]:
        return [d for cn in self.child_nodes for d in cn.get_hyper_parameter_distribution_definition(xrange, n)]

    def get_hyper_parameter_names(self, kernel_id: int = -1) -> List[str]:
        names = []
        for cn in self.child_nodes:
            names += cn.get_hyper_parameter_names(kernel_id)
            if isinstance(cn, bk.BaseKernel) and kernel_id >= 0:
                kernel_id += 1
        return names

    def set_noise(self, noise):
        super().set_noise(noise)
        for cn in self.child_nodes:
            cn.set_noise(noise)

    def set_dimensionality(self, input_dimensionality: int):
        super().set_dimensionality(input_dimensionality)
        for cn in self.child_nodes:
            cn.set_dimensionality(input_dimensionality)

    def sort_child_nodes(self):
        if self.sortable:
            self.child_nodes = sorted(self.child_nodes, key=lambda c: c.get_string_representation_weight())
        for cn in self.child_nodes:
            if isinstance(cn, Operator):
                cn.sort_child_nodes()

    def type_compare_to(self, other):
        while isinstance(other, Operator) and len(other.child_nodes) == 1:
            other = other.child_nodes[0]
        if len(self.child_nodes) == 1:
            return self.child_nodes[0].type_compare_to(other)
        if not isinstance(other, Operator) or len(other.child_nodes) != len(self.child_nodes):
            return False
        self.sort_child_nodes()
        other.sort_child_nodes()
        return all(a.type_compare_to(b) for a, b in zip(self.child_nodes, other.child_nodes))

    def get_hash_tuple(self):
        return super().get_hash_tuple() + (sum(hash(cn) for cn in self.child_nodes),)

    def deepcopy(self):
        c = type(self)(self.input_dimensionality, [cn.deepcopy() for cn in self.child_nodes])
        if self.noise is not None:
            c.set_noise(self.noise)
        return c

    def __repr__(self):
        return self.get_string_representation()


class MultiplicationOperator(Operator):
    _BINARY_OP = nat.OP_MUL
    operator_sign = "x"

    def __init__(self, input_dimensionality: int, child_nodes: List[k.Kernel]):
        super().__init__(k.KernelManifestation.MUL, input_dimensionality, child_nodes)

    def get_simplified_version(self):
        """Flatten nested products and distribute over the first sum (Operators.py:271-297)."""
        flat, add_at = [], None
        for cn in (c.get_simplified_version() for c in self.child_nodes):
            if isinstance(cn, MultiplicationOperator):
                flat.extend(cn.child_nodes)
            else:
                if isinstance(cn, AdditionOperator) and add_at is None:
                    add_at = len(flat)
                flat.append(cn)
        if add_at is None:
            return MultiplicationOperator(self.input_dimensionality, flat)
        others = [c for i, c in enumerate(flat) if i != add_at]
        terms = [MultiplicationOperator(self.input_dimensionality, others + [t]) for t in flat[add_at].child_nodes]
        return AdditionOperator(self.input_dimensionality, terms).get_simplified_version()


class AdditionOperator(Operator):
    _BINARY_OP = nat.OP_ADD
    operator_sign = "+"

    def __init__(self, input_dimensionality: int, child_nodes: List[k.Kernel]):
        super().__init__(k.KernelManifestation.ADD, input_dimensionality, child_nodes)

    def get_simplified_version(self):
        """Flatten nested sums (Operators.py:356-367)."""
        flat = []
        for cn in (c.get_simplified_version() for c in self.child_nodes):
            flat.extend(cn.child_nodes if isinstance(cn, AdditionOperator) else [cn])
        return AdditionOperator(self.input_dimensionality, flat)


class ChangePointOperator(Operator):
    """Change-point operator (Operators.py:370-681).

    K = sum_i K_i * (a_i a_i'^T), a_i(x) = (1 - ind_{i-1}(x)) ind_i(x) with ind_i the indicator of
    x < cp_i (ind_{-1} = 0, ind_last = 1) -- the product of the mask outer products that
    get_cp_encapsulated_kernel applies child by child (:410-440).  The indicator follows
    ``global_parameters.p_cp_operator_type``: INDICATOR (default, :397-400), SIGMOID (:387-394) or
    APPROX_INDICATOR (:379-385).  Every child matrix comes from the device kernel-matrix build; the
    masks are applied on the device.
    """
    operator_sign = "]["

    def __init__(self, input_dimensionality: int, child_nodes: List[k.Kernel], change_point_positions: List):
        super().__init__(k.KernelManifestation.CP, input_dimensionality, child_nodes)
        assert (len(child_nodes) - 1) == len(change_point_positions), \
            "Error. Change Point positions and/or their positions wrongly initialized."
        self.change_point_positions = list(change_point_positions)
        self.sortable = False

    def _emit(self, nodes: list, offset: int, ard_slots: list, dim: int) -> int:
        if len(self.child_nodes) == 1:
            return self.child_nodes[0]._emit(nodes, offset, ard_slots, dim)
        raise NotImplementedError("a ChangePointOperator is evaluated segment by segment (masked child "
                                  "matrices / SegmentedCovarianceMatrix), not as one device program")

    @staticmethod
    def _mask(x: torch.Tensor, cp) -> torch.Tensor:
        xv = x.reshape(-1)
        c = torch.as_tensor(cp, dtype=torch.float64, device=xv.device).reshape(())
        t = global_param.p_cp_operator_type
        if t == global_param.ChangePointOperatorType.SIGMOID:
            return 0.5 * (1 + torch.tanh((c - xv) / 0.0025))
        if t == global_param.ChangePointOperatorType.APPROX_INDICATOR:
            return 1.0 / (1.0 + torch.exp(-100.0 * (xv - c)))
        return (xv < c).to(torch.float64)

    # the reference's mask functions on [N, 1] inputs (Operators.py:379-408), device tensors in and out
    @staticmethod
    def approx_indicator(x, cp) -> torch.Tensor:
        """1 / (1 + exp(-100 (x - cp))) (:379-385)."""
        return 1.0 / (1.0 + torch.exp(-100.0 * (x - cp)))

    @staticmethod
    def sigmoid(x, cp) -> torch.Tensor:
        """0.5 (1 + tanh((cp - x) / 0.0025)) (:387-394)."""
        return 0.5 * (1 + torch.tanh((cp - x) / 0.0025))

    @staticmethod
    def indicator_function_tf_less(x, cp) -> torch.Tensor:
        """[x < cp] as fp64, shape [N, 1] (:396-400)."""
        c = torch.as_tensor(cp, dtype=torch.float64, device=x.device).reshape(())
        return (x.reshape(-1) < c).to(torch.float64).reshape(-1, 1)

    @staticmethod
    def indicator_function_relu_sign(x, cp) -> torch.Tensor:
        """relu(sign(x - cp)) (:402-404; unused by the reference's operator)."""
        return torch.relu(torch.sign(x - cp))

    def indicator_function(self, x, cp) -> torch.Tensor:
        return self.indicator_function_tf_less(x, cp)

    def get_cp_encapsulated_kernel(self, kernel, x_vector, x_vector_, hyper_param, previous_sigmoid, cp):
        """(K * previous_sigmoid * ind ind'^T, (1 - ind)(1 - ind')^T) for one child (:410-440): its
        matrix from the device kernel build, masked by this change point's outer indicator; the second
        value is the complement mask the next child starts from (0 when cp is None, as in the reference)."""
        from .. import engine
        x, x_ = engine.as_device_f64(x_vector), engine.as_device_f64(x_vector_)
        K = kernel.get_tf_tensor(hyper_param, x, x_) * previous_sigmoid
        if cp is None:
            return K, torch.zeros((), dtype=torch.float64, device=K.device)
        cp = torch.as_tensor(cp, dtype=torch.float64, device=K.device)
        t = global_param.p_cp_operator_type
        if t == global_param.ChangePointOperatorType.SIGMOID:
            ind, ind_ = self.sigmoid(x, cp), self.sigmoid(x_, cp)
        elif t == global_param.ChangePointOperatorType.APPROX_INDICATOR:
            ind, ind_ = self.approx_indicator(x, cp), self.approx_indicator(x_, cp)
        else:
            ind, ind_ = self.indicator_function(x, cp), self.indicator_function(x_, cp)
        return K * (ind @ ind_.transpose(-1, -2)), (1.0 - ind) @ (1.0 - ind_).transpose(-1, -2)

    def get_tf_tensor(self, hyper_parameter: List, x_vector, x_vector_) -> torch.Tensor:
        assert x_vector is not None and x_vector_ is not None, "Input vectors x and x_ uninitialized: " + str(self)
        assert len(hyper_parameter) == self.get_number_of_hyper_parameter(), "Invalid hyper_param size: %s" % str(self)
        if len(self.child_nodes) == 1:
            return self.child_nodes[0].get_tf_tensor(hyper_parameter, x_vector, x_vector_)
        from .. import engine
        x = engine.as_device_f64(x_vector)
        x_ = engine.as_device_f64(x_vector_)
        ncp = len(self.change_point_positions)
        cps = list(hyper_parameter[:ncp])
        idx = ncp
        prev, prev_ = torch.ones(x.shape[0], dtype=torch.float64, device=x.device), \
            torch.ones(x_.shape[0], dtype=torch.float64, device=x.device)
        result = None
        for i, cn in enumerate(self.child_nodes):
            nh = cn.get_number_of_hyper_parameter()
            Ki = cn.get_tf_tensor(list(hyper_parameter[idx:idx + nh]), x, x_)
            idx += nh
            if i < ncp:
                ind, ind_ = self._mask(x, cps[i]), self._mask(x_, cps[i])
                a, a_ = prev * ind, prev_ * ind_
                prev, prev_ = 1.0 - ind, 1.0 - ind_
            else:
                a, a_ = prev, prev_
            term = Ki * (a[:, None] * a_[None, :])
            result = term if result is None else result + term
        self.last_hyper_parameter = cps
        return result

    get_tensor = get_tf_tensor

    def _slices(self, hyper_parameter: List):
        idx = len(self.change_point_positions)
        for cn in self.child_nodes:
            cnt = cn.get_number_of_hyper_parameter()
            yield cn, list(hyper_parameter[idx:idx + cnt])
            idx += cnt

    def _record_hyper_parameter(self, hyper_parameter: List):
        if len(self.child_nodes) == 1:
            self.child_nodes[0]._record_hyper_parameter(hyper_parameter)
            return
        for cn, sl in self._slices(hyper_parameter):
            cn._record_hyper_parameter(sl)

    def get_number_of_hyper_parameter(self) -> int:
        return sum(cn.get_number_of_hyper_parameter() for cn in self.child_nodes) + len(self.change_point_positions)

    def get_hyper_parameter_dimensionalities(self) -> List[list]:
        return [[len(self.change_point_positions), ]] + super().get_hyper_parameter_dimensionalities()

    def set_last_hyper_parameter(self, last_hyper_parameter: List):
        assert len(last_hyper_parameter) == self.get_number_of_hyper_parameter(), \
            "Invalid hyper_param size: %s" % str(last_hyper_parameter)
        if len(self.child_nodes) == 1:
            self.child_nodes[0].set_last_hyper_parameter(last_hyper_parameter)
            return
        self.change_point_positions = list(last_hyper_parameter[0:len(self.change_point_positions)])
        self.last_hyper_parameter = self.change_point_positions
        for cn, sl in self._slices(last_hyper_parameter):
            cn.set_last_hyper_parameter(sl)

    def get_last_hyper_parameter(self, scaling_x_param=None):
        out = []
        for cn in self.child_nodes:
            out.extend(cn.get_last_hyper_parameter(scaling_x_param))
        return list(self.change_point_positions) + out

    def add_kernel(self, kernel: k.Kernel, new_cp_position=None):
        assert kernel is not None, "Adding None as kernel to ChangePoint is not allowed."
        assert new_cp_position is not None
        if self.change_point_positions:
            assert float(torch.as_tensor(new_cp_position).min()) > \
                float(torch.as_tensor(self.change_point_positions[-1]).max()), \
                "New Changepoints _must_ be larger in value than the former largest change point."
        self.child_nodes.append(kernel)
        self.change_point_positions.append(new_cp_position)

    def add_preceding_kernel(self, kernel, new_cp_position):
        assert kernel is not None, "Adding None as kernel to ChangePoint is not allowed."
        assert new_cp_position is not None
        if self.change_point_positions:
            assert float(torch.as_tensor(self.change_point_positions[-1]).min()) > \
                float(torch.as_tensor(new_cp_position).max()), \
                "New Changepoints _must_ be larger in value than the former largest change point."
        self.child_nodes = [kernel] + self.child_nodes
        self.change_point_positions = [new_cp_position] + self.change_point_positions

    def get_default_hyper_parameter(self, xrange, n, from_distribution: bool = False) -> List:
        return list(self.change_point_positions) + super().get_default_hyper_parameter(xrange, n, from_distribution)

    def get_hyper_parameter_bounds(self, xrange, n) -> List[tuple]:
        span = xrange[0][1] - xrange[0][0]
        lo, hi = xrange[0][0] - 1.5 * span, xrange[0][1] + 1.5 * span
        return [(lo, hi)] * len(self.change_point_positions) + super().get_hyper_parameter_bounds(xrange, n)

    def get_simplified_kernel(self, data_range: List[float]):
        """Drop change points outside the data range or overtaken by their successor, with the
        children they separate (Operators.py:533-582); returns (kernel, changed)."""
        cps = [float(torch.as_tensor(c)) for c in self.change_point_positions]
        blur = 4 if global_param.p_cp_operator_type == global_param.ChangePointOperatorType.SIGMOID else 0
        del_cp, del_cn = [], []
        for i, c in enumerate(cps):
            if c >= data_range[1] + blur:
                del_cp.append(i)
                del_cn.append(i + 1)
            if c <= data_range[0] - blur:
                del_cp.append(i)
                del_cn.append(i)
            if len(cps) - 1 > i and c >= cps[i + 1]:
                del_cp.append(i)
                del_cn.append(i + 1)
        if not del_cp:
            return self, False
        new_cps = [self.change_point_positions[i] for i in range(len(cps)) if i not in del_cp]
        new_cn = [cn for i, cn in enumerate(self.child_nodes) if i not in del_cn]
        assert len(new_cps) + 1 == len(new_cn), \
            "Error in get_simplified_kernel, new_change_points: %s, new_child_nodes: %s" % (new_cps, new_cn)
        return ChangePointOperator(self.input_dimensionality, new_cn, new_cps), True

    def get_json(self) -> dict:
        if len(self.child_nodes) == 1:
            return {"type": self.manifestation.name, "child_nodes": [self.child_nodes[0].get_json()]}
        nodes = []
        cps = [float(torch.as_tensor(c)) for c in self.change_point_positions]
        for i, cn in enumerate(self.child_nodes):
            j = cn.get_json()
            j["start_index"] = 0 if i == 0 else cps[i - 1]
            j["stop_index"] = 1.0 if i == len(cps) else cps[i]
            nodes.append(j)
        return {"type": self.manifestation.name, "child_nodes": nodes}

    def get_simplified_version(self):
        return ChangePointOperator(self.input_dimensionality, [cn.get_simplified_version() for cn in self.child_nodes],
                                   self.change_point_positions)

    def deepcopy(self):
        c = ChangePointOperator(self.input_dimensionality, [cn.deepcopy() for cn in self.child_nodes],
                                [torch.as_tensor(cp).clone() if isinstance(cp, torch.Tensor) else cp
                                 for cp in self.change_point_positions])
        if self.noise is not None:
            c.set_noise(self.noise)
        return c

    def get_hash_tuple(self):
        return super().get_hash_tuple() + tuple(hash(cn) for cn in self.child_nodes)
