"""Partitioning of the input space (gpbasics/KernelBasics/PartitioningModel.py).

Host-side index bookkeeping (which data record belongs to which partition); the covariance work
of the partitions runs on the device (SegmentedCovarianceMatrix / PartitionOperator).

* ``PartitionCriterion.get_score(x)`` scores every record for one partition
  (PartitioningModel.py:21-32); concrete criteria are supplied by the caller, as in the reference.
* ``PartitioningModel.get_data_record_indices_per_partition`` (:109-131): SELF_SUFFICIENT
  criteria score 1 for the records of their partition; SMALLEST_DISTANCE assigns each record to
  the criterion with the smallest score, ties broken by N(0, 1e-10) noise from numpy's global
  generator (as the reference does, so a seeded numpy reproduces its assignment).
* ``partition_data_input`` (:62-107) builds the PartitionedDataInput of the partitions.
"""
from __future__ import annotations

import logging
from enum import Enum
from typing import List

import numpy as np
import torch

from .. import global_parameters as global_param

global_param.ensure_init()


class PartitioningClass(Enum):
    SELF_SUFFICIENT = 0,
    SMALLEST_DISTANCE = 1


class PartitionCriterion:
    def __init__(self, partitioning_type: PartitioningClass):
        self.partitioning_type = partitioning_type

    def get_score(self, x_vector: np.ndarray) -> np.ndarray:
        pass

    def deepcopy(self):
        pass

    def get_json(self) -> dict:
        pass


def _host(x) -> np.ndarray:
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


class PartitioningModel:
    def __init__(self, partition_class: PartitioningClass, ignored_dimensions: List[int]):
        self.partitioning: List[PartitionCriterion] = []
        self.partition_class = partition_class
        self.ignored_dimensions = list(ignored_dimensions)

    def automatic_init_criteria(self, data_input, optimize_metric, model_selection_metric,
                                number_of_partitions: int = None, predecessor_criterion: PartitionCriterion = None):
        pass

    def init_partitioning(self, partitioning: List[PartitionCriterion]):
        if len(self.partitioning) > 0:
            logging.warning("%s: Overwriting old partitioning." % str(self))
        self.partitioning = partitioning

    def get_number_of_partitions(self) -> int:
        return len(self.partitioning)

    def add_partitioning_criterion(self, criterion: PartitionCriterion):
        assert criterion.partitioning_type == self.partition_class, \
            "Partitioning Criterion does not match Partitioning Model"
        assert criterion is not None, "Criterion cannot be None"
        self.partitioning.append(criterion)

    def partition_data_input(self, data_input):
        """PartitionedDataInput of the partitions, records regrouped partition by partition
        (PartitioningModel.py:62-107)."""
        from ..DataHandling import DataInput as di
        if len(self.partitioning) <= 1:
            logging.warning("Dataset cannot be partitioned as only one / none partition criterion is available.")
            return di.PartitionedDataInput(data_input.data_x_train, data_input.data_y_train, data_input.data_x_test,
                                           data_input.data_y_test, [data_input])
        xtr, xte = _host(data_input.data_x_train), _host(data_input.data_x_test)
        separate = not np.array_equal(xtr, xte)
        train_idx = self.get_data_record_indices_per_partition(xtr)
        test_idx = self.get_data_record_indices_per_partition(xte) if separate else train_idx
        assert len(train_idx) == len(test_idx)
        blocks = []
        parts = {"xtr": [], "ytr": [], "xte": [], "yte": []}
        for tr, te in zip(train_idx, test_idx):
            trt = torch.as_tensor(tr, dtype=torch.long, device=data_input.data_x_train.device)
            tet = torch.as_tensor(te, dtype=torch.long, device=data_input.data_x_test.device)
            bx, by = data_input.data_x_train[trt], data_input.data_y_train[trt]
            bxt = data_input.data_x_test[tet]
            byt = data_input.data_y_test[tet] if data_input.data_y_test is not None else None
            blocks.append(di.DataInput(data_x_train=bx, data_y_train=by, data_x_test=bxt, data_y_test=byt))
            parts["xtr"].append(bx)
            parts["ytr"].append(by)
            parts["xte"].append(bxt)
            parts["yte"].append(byt)
        yte = None if any(v is None for v in parts["yte"]) else torch.cat(parts["yte"], dim=0)
        return di.PartitionedDataInput(torch.cat(parts["xtr"], dim=0), torch.cat(parts["ytr"], dim=0),
                                       torch.cat(parts["xte"], dim=0), yte, blocks)

    def get_data_record_indices_per_partition(self, x_vector) -> List[np.ndarray]:
        """Indices of the records of each partition (PartitioningModel.py:109-131)."""
        x = _host(x_vector)
        cols = [np.asarray(c.get_score(self.filter_data_by_ignored_dimensions(x))).reshape(-1)
                for c in self.partitioning]
        if not cols:
            return [np.linspace(0, len(x) - 1, len(x), dtype=int)]
        score = np.transpose(np.array(cols))
        if self.partition_class == PartitioningClass.SMALLEST_DISTANCE:
            score = score + np.random.normal(0, 1e-10, score.shape)
            col_min = np.amin(score, axis=1)
            score = score == col_min.reshape(-1, 1)
        return [np.where(score[:, i] == 1)[0] for i in range(self.get_number_of_partitions())]

    def filter_data_by_ignored_dimensions(self, vector):
        if len(self.ignored_dimensions) == 0:
            return vector
        assert vector.shape[1] > max(self.ignored_dimensions)
        keep = [i not in self.ignored_dimensions for i in range(vector.shape[1])]
        return vector[:, keep]

    def deepcopy(self):
        pm = PartitioningModel(self.partition_class, list(self.ignored_dimensions))
        pm.partitioning = [pc.deepcopy() for pc in self.partitioning]
        return pm

    def get_hash_tuple(self):
        return tuple(self.ignored_dimensions) + (sum(hash(c) for c in self.partitioning),)

    def __hash__(self):
        return hash(self.get_hash_tuple())
