"""ADD / MUL kernel operators (gpbasics/KernelBasics/Operators.py:15-367).

A whole operator tree is evaluated by ONE device launch: the tree is flattened into a postfix
program whose binary ADD/MUL nodes fold the children left to right, exactly the order of the
reference's ``result = op(result, child_i)`` loops (Operators.py:214-223, :314-324).
Hyperparameters are one flat list in child DFS order, sliced by each child's
``get_number_of_hyper_parameter`` (Operators.py:28-32).

Out of scope: ChangePointOperator (Operators.py:370-681), PartitionOperator.
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
