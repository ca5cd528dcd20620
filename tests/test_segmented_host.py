"""Host logic of the segmented models (no GPU): partition assignment, block layout, change-point
segmentation of data inputs, cross-validation folds, the blockwise hyperparameter-offset quirk."""
import numpy as np
import pytest
import torch

import gaussianprocessfundamentals_amd.global_parameters as gp
from gaussianprocessfundamentals_amd.DataHandling.DataInput import BlockwiseDataInput, DataInput
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk
from gaussianprocessfundamentals_amd.KernelBasics import Operators as ops
from gaussianprocessfundamentals_amd.KernelBasics import PartitioningModel as pm
from gaussianprocessfundamentals_amd.KernelBasics.PartitionOperator import block_matrix_from_blocks
from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction
from gaussianprocessfundamentals_amd.Metrics import CrossValidation as cv
from gaussianprocessfundamentals_amd.Metrics.LogLikelihood import blockwise_hyper_parameter_offset
from oracle import gp_oracle as orc


class Interval(pm.PartitionCriterion):
    """Self-sufficient criterion: records with lo <= x_0 < hi."""

    def __init__(self, lo, hi):
        super().__init__(pm.PartitioningClass.SELF_SUFFICIENT)
        self.lo, self.hi = lo, hi

    def get_score(self, x):
        return ((x[:, 0] >= self.lo) & (x[:, 0] < self.hi)).astype(np.float64)

    def deepcopy(self):
        return Interval(self.lo, self.hi)


class Centre(pm.PartitionCriterion):
    """Smallest-distance criterion: |x_0 - c|."""

    def __init__(self, c):
        super().__init__(pm.PartitioningClass.SMALLEST_DISTANCE)
        self.c = c

    def get_score(self, x):
        return np.abs(x[:, 0] - self.c)


def test_self_sufficient_partition_indices():
    model = pm.PartitioningModel(pm.PartitioningClass.SELF_SUFFICIENT, [])
    for lo, hi in [(0.0, 0.3), (0.3, 0.7), (0.7, 1.01)]:
        model.add_partitioning_criterion(Interval(lo, hi))
    x = np.linspace(0, 1, 11).reshape(-1, 1)
    idx = model.get_data_record_indices_per_partition(x)
    assert [list(i) for i in idx] == [[0, 1, 2], [3, 4, 5, 6], [7, 8, 9, 10]]
    with pytest.raises(AssertionError):
        model.add_partitioning_criterion(Centre(0.5))


def test_smallest_distance_partition_and_ignored_dimensions():
    np.random.seed(0)
    model = pm.PartitioningModel(pm.PartitioningClass.SMALLEST_DISTANCE, [1])
    model.init_partitioning([Centre(0.2), Centre(0.8)])
    x = np.stack([np.linspace(0, 1, 9), np.full(9, 100.0)], axis=1)   # dimension 1 is ignored
    idx = model.get_data_record_indices_per_partition(x)
    assert list(idx[0]) == [0, 1, 2, 3] and list(idx[1]) == [5, 6, 7, 8] or \
        sorted(list(idx[0]) + list(idx[1])) == list(range(9))
    assert set(idx[0]) | set(idx[1]) == set(range(9)) and not set(idx[0]) & set(idx[1])


def test_block_matrix_offsets_and_reference_quirk():
    a, b = torch.ones(2, 3), 2 * torch.ones(1, 1)
    out = block_matrix_from_blocks([(2, 3), (0, 4), (1, 1)], [a, None, b], "cpu")
    assert out.shape == (3, 8)
    assert torch.all(out[:2, :3] == 1) and out[2, 7] == 2 and out.sum() == 8
    # leading partitions empty on the rows side: zero rows on top (NonSquareBlockMatrices.py:33-34)
    out = block_matrix_from_blocks([(2, 0), (1, 1)], [None, b], "cpu")
    assert out.shape == (3, 1) and out[2, 0] == 2
    # leading partitions empty on the column side only: the reference pads rows and its shape
    # assertion fails (NonSquareBlockMatrices.py:35-36)
    with pytest.raises(AssertionError):
        block_matrix_from_blocks([(0, 2), (1, 1)], [None, b], "cpu")


def test_blockwise_data_input_segments_at_change_points():
    gp.p_device = "cpu"
    try:
        x = np.linspace(0, 1, 21).reshape(-1, 1)
        y = np.sin(6 * x)
        xt = np.linspace(0.025, 0.975, 20).reshape(-1, 1)
        d = BlockwiseDataInput(x, y, xt, np.cos(xt), [0.3, 0.6])
        assert [di.n_train for di in d.data_inputs] == [int(np.sum(x < 0.3)), int(np.sum((x >= 0.3) & (x < 0.6))),
                                                      int(np.sum(x >= 0.6))]
        assert sum(di.n_test for di in d.data_inputs) == 20
        for di, (lo, hi) in zip(d.data_inputs, [(-1, 0.3), (0.3, 0.6), (0.6, 2)]):
            xs = di.data_x_train.numpy()
            assert np.all((xs >= lo) & (xs < hi))
        d.set_mean_function(ZeroMeanFunction(1))
        assert all(di.mean_function is d.mean_function for di in d.data_inputs)
    finally:
        gp.p_device = "cuda"


def test_cv_folds_follow_numpy_global_generator():
    gp.p_device = "cpu"
    try:
        n = 53
        x = np.random.default_rng(1).uniform(size=(n, 1))
        y = np.sin(x)
        d = DataInput(x, y, x, y)
        d.set_mean_function(ZeroMeanFunction(1))
        np.random.seed(7)
        folds = cv.get_data_inputs(d, 0.2)
        np.random.seed(7)
        ref = orc.cv_folds(n, 0.2)
        assert len(folds) == len(ref) == 5
        for f, (tr, te) in zip(folds, ref):
            assert np.array_equal(f.data_x_train.numpy().reshape(-1), x[tr].reshape(-1))
            assert np.array_equal(f.data_x_test.numpy().reshape(-1), x[te].reshape(-1))
    finally:
        gp.p_device = "cuda"


def test_blockwise_offset_quirk_is_zero():
    from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import BlockwiseGaussianProcess
    cp = ops.ChangePointOperator(1, [bk.SquaredExponentialKernel(1), bk.SquaredExponentialKernel(1)], [0.5])
    g = BlockwiseGaussianProcess(cp, ZeroMeanFunction(1))
    assert blockwise_hyper_parameter_offset(g) == 0
    assert cp.get_number_of_hyper_parameter() == 3
    assert cp.get_hyper_parameter_dimensionalities()[0] == [1]


def test_change_point_hyper_parameter_plumbing():
    a, b = bk.SquaredExponentialKernel(1), bk.PeriodicKernel(1)
    cp = ops.ChangePointOperator(1, [a, b], [0.4])
    cp.set_last_hyper_parameter([torch.tensor(0.45), torch.tensor(0.2), torch.tensor(0.3), torch.tensor(0.5)])
    assert float(cp.change_point_positions[0]) == pytest.approx(0.45)
    hp = cp.get_last_hyper_parameter()
    assert len(hp) == 4 and float(hp[0]) == pytest.approx(0.45) and float(hp[2]) == pytest.approx(0.3)
    simplified, changed = cp.get_simplified_kernel([0.0, 0.4])
    assert changed and simplified is a or (changed and len(simplified.child_nodes) == 1)
    with pytest.raises(AssertionError):
        ops.ChangePointOperator(1, [a, b], [])
