"""Partition operator (gpbasics/KernelBasics/PartitionOperator.py:15-123).

Child kernel i covers the records its partition criterion assigns to it; records of different
partitions are independent.  ``get_tf_tensor(hyp, x, x_)`` returns the block matrix the reference
builds (PartitionOperator.py:24-82): the child blocks k_i(x[P_i], x_[P_i']) laid out block-diagonally
**in partition order** (the rows are regrouped partition by partition, not kept in the order of
x), each child block computed by the device kernel-matrix build.  Hyperparameters are the
children's in order (no extra parameters of the operator itself).
"""
from __future__ import annotations

from typing import List

import torch

from .. import global_parameters as global_param
from . import Kernel as k
from . import Operators as op
from . import PartitioningModel as pm

global_param.ensure_init()


def block_matrix_from_blocks(shapes: List[tuple], blocks: List, device, dtype=torch.float64) -> torch.Tensor:
    """Block-diagonal placement of possibly non-square blocks at cumulative offsets
    (Auxiliary/NonSquareBlockMatrices.py:8-65).  ``blocks[i]`` is a tensor or None for an empty
    partition of shape shapes[i] (one side zero).  Quirk kept: when the leading partitions are
    empty on the column side only, the reference pads ROWS instead of columns
    (NonSquareBlockMatrices.py:35-36) and its shape assertion fails; this raises the same
    AssertionError."""
    lead_rows = lead_cols = 0
    for (r, c), bm in zip(shapes, blocks):
        if bm is not None:
            break
        lead_rows += r
        lead_cols += c
    if lead_cols > 0 and lead_rows == 0 and any(b is not None for b in blocks):
        raise AssertionError("x_vector.shape / result_shape mismatch (empty leading partitions on the column side)")
    R, C = sum(s[0] for s in shapes), sum(s[1] for s in shapes)
    out = torch.zeros((R, C), dtype=dtype, device=device)
    r0 = c0 = 0
    for (r, c), bm in zip(shapes, blocks):
        if bm is not None:
            out[r0:r0 + r, c0:c0 + c] = bm
        r0 += r
        c0 += c
    return out


class PartitionOperator(op.Operator):
    operator_sign = "|"

    def __init__(self, input_dimensionality: int, child_nodes: List[k.Kernel],
                 partitioning_model: pm.PartitioningModel):
        assert len(child_nodes) == partitioning_model.get_number_of_partitions(), \
            "One partitioning criterion for each kernel has to be supplied"
        super().__init__(k.KernelManifestation.PART, input_dimensionality, child_nodes)
        self.partitioning_model = partitioning_model
        self.sortable = False

    def _emit(self, nodes: list, offset: int, ard_slots: list, dim: int) -> int:
        raise NotImplementedError("a PartitionOperator is evaluated block by block (SegmentedCovarianceMatrix / "
                                  "get_tf_tensor), not as one device program")

    def get_list_of_block_matrices(self, hyper_parameter, x_vector, x_vector_):
        """(blocks, square, indices, indices_) as PartitionOperator.py:46-80: blocks[i] is the child
        matrix, or the [len, len_] shape of a partition that is empty on one side."""
        indices = self.partitioning_model.get_data_record_indices_per_partition(x_vector)
        indices_ = indices if x_vector is x_vector_ else \
            self.partitioning_model.get_data_record_indices_per_partition(x_vector_)
        assert len(indices) == len(indices_) and len(indices) == len(self.child_nodes)
        square = True
        blocks = []
        idx = 0
        for i, cn in enumerate(self.child_nodes):
            nh = cn.get_number_of_hyper_parameter()
            if len(indices[i]) == 0 or len(indices_[i]) == 0:
                if len(indices[i]) != len(indices_[i]):
                    blocks.append([len(indices[i]), len(indices_[i])])
            else:
                a = torch.as_tensor(indices[i], dtype=torch.long, device=x_vector.device)
                b = torch.as_tensor(indices_[i], dtype=torch.long, device=x_vector_.device)
                blocks.append(cn.get_tf_tensor(list(hyper_parameter[idx:idx + nh]), x_vector[a], x_vector_[b]))
            if len(indices[i]) != len(indices_[i]):
                square = False
            idx += nh
        return blocks, square, indices, indices_

    def get_tf_tensor(self, hyper_parameter: List, x_vector, x_vector_) -> torch.Tensor:
        assert x_vector is not None and x_vector_ is not None, "Input vectors x and x_ uninitialized: " + str(self)
        from .. import engine
        x = engine.as_device_f64(x_vector)
        x_ = x if x_vector_ is x_vector else engine.as_device_f64(x_vector_)
        blocks, _, _, _ = self.get_list_of_block_matrices(hyper_parameter, x, x_)
        shapes = [tuple(b.shape) if isinstance(b, torch.Tensor) else tuple(b) for b in blocks]
        mats = [b if isinstance(b, torch.Tensor) else None for b in blocks]
        result = block_matrix_from_blocks(shapes, mats, x.device)
        assert result.shape[0] == x.shape[0] and result.shape[1] == x_.shape[0], \
            "x_vector.shape=%s, result_shape=%s" % (str(tuple(x.shape)), str(tuple(result.shape)))
        return result

    get_tensor = get_tf_tensor

    def add_kernel(self, kernel: k.Kernel, criterion: pm.PartitionCriterion):
        assert kernel is not None, "Adding None as kernel to ChangePoint is not allowed."
        self.child_nodes.append(kernel)
        self.partitioning_model.add_partitioning_criterion(criterion)

    def deepcopy(self):
        c = PartitionOperator(self.input_dimensionality, [cn.deepcopy() for cn in self.child_nodes],
                              self.partitioning_model.deepcopy())
        if self.noise is not None:
            c.set_noise(self.noise)
        return c

    def get_json(self) -> dict:
        if len(self.child_nodes) == 1:
            return {"type": self.manifestation.name, "child_nodes": [self.child_nodes[0].get_json()]}
        nodes = []
        for i, cn in enumerate(self.child_nodes):
            j = cn.get_json()
            j["partitioning_criterion"] = self.partitioning_model.partitioning[i].get_json()
            nodes.append(j)
        return {"type": self.manifestation.name, "child_nodes": nodes}

    def get_simplified_version(self):
        return PartitionOperator(self.input_dimensionality, [cn.get_simplified_version() for cn in self.child_nodes],
                                 self.partitioning_model)

    def get_hash_tuple(self):
        return super().get_hash_tuple() + tuple(hash(cn) for cn in self.child_nodes) + \
            (hash(self.partitioning_model),)
