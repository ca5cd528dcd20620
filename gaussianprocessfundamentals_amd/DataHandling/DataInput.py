"""Data inputs (gpbasics/DataHandling/AbstractDataInput.py, DataInput.py, BatchDataInput.py).

Inputs are cast to fp64 (DataInput.py:198-206) and kept resident on the engine's device.
Shapes: X [N, D], y [N, 1] (AbstractDataInput.py:17-27) or, for :class:`BatchDataInput`,
X [B, N, D], y [B, N, 1].  Without an explicit test set, ``test_ratio`` of the points (default
0.2) is held out by a seeded random permutation (AbstractDataInput.py:41-60); the permutation
comes from torch's generator, not TensorFlow's, so the held-out indices differ from the
reference's for the same seed.
"""
from __future__ import annotations

import logging
from typing import List

import torch

from .. import global_parameters as global_param
from ..MeanFunctionBasics import BaseMeanFunctions as bmf

global_param.ensure_init()


def _dev():
    from ..engine import device
    try:
        return device()
    except Exception:  # noqa: BLE001 - no GPU: host-side data handling still works
        return torch.device("cpu")


def _f64(x) -> torch.Tensor:
    t = x.detach() if isinstance(x, torch.Tensor) else torch.as_tensor(x)
    return t.to(device=_dev(), dtype=torch.float64)


def is_equidistant(input_vector) -> bool:
    """Consecutive differences within 1 / (100 len) of their mean (DataInput.py:17-23), over every
    element of the [N, D] array (numpy's flat mean / max / min)."""
    v = _f64(input_vector)
    diff = v[:len(v) - 1] - v[1:]
    mean = torch.mean(diff)
    allowed_error = 1 / (100 * len(v))
    return bool(torch.abs(torch.max(diff) - mean) < allowed_error) and \
        bool(torch.abs(torch.min(diff) - mean) < allowed_error)


def is_equidistant_batch(input_data) -> torch.Tensor:
    """BatchDataInput.py:14-21 as written: the mean over the BATCH axis [N-1, D] against the per-member
    max / min over the points [B, D] (the two broadcast only when B or N - 1 is 1 or they are equal,
    as in TensorFlow); returns the boolean tensor."""
    x = _f64(input_data)
    length = x.shape[1]
    diff = x[:, :length - 1, :] - x[:, 1:, :]
    mean = torch.mean(diff, dim=0)
    diff_max = torch.abs(torch.max(diff, dim=1).values - mean)
    diff_min = torch.abs(torch.min(diff, dim=1).values - mean)
    allowed_error = 1 / (100 * length)
    return torch.logical_and(diff_max < allowed_error, diff_min < allowed_error)


class AbstractDataInput:
    def __init__(self, data_x_train, data_y_train, data_x_test=None, data_y_test=None,
                 test_ratio: float = -1, seed: int = 3061941):
        assert (data_x_test is None or (len(data_x_train.shape) == len(data_x_test.shape)
                                        and len(data_y_train.shape) == len(data_y_test.shape)
                                        and len(data_x_train.shape) == len(data_y_train.shape))) and \
            len(data_x_train.shape) in (2, 3), \
            "Shape of input and target data (test as well as train data) needs to be either " \
            "[instance#, length, dimensionality] or [length, dimensionality]."
        assert data_y_train.shape[-1] == 1, \
            "Target training data (data_y_train) has to be unidimensional, shape=[n_train, 1] / [instance#, n_train, 1]"
        assert data_y_test is None or data_y_test.shape[-1] == 1, \
            "Target test data (data_y_test) has to be unidimensional, shape=[n_test, 1] / [instance#, n_test, 1]"
        assert data_x_test is None or data_x_train.shape[-1] == data_x_test.shape[-1], \
            "Dimensionality of training and test input data (data_x_train and data_x_test) need to match"
        assert test_ratio <= 1, "test_ratio has to be in the range [0; 1]"
        self.seed = seed
        if test_ratio > 0 and data_x_test is not None:
            logging.warning("test_ratio is ignored if test_data is explicitly given.")
        if data_x_test is None and test_ratio != 0:
            if test_ratio < 0:
                logging.warning("test_ratio is not given although explicit test data was not provided. "
                                "default value '0.2' is assumed for test_ratio.")
                test_ratio = 0.2
            length = data_x_train.shape[0]
            test_size = min(length - 1, int(length * test_ratio))
            gen = torch.Generator().manual_seed(int(seed))
            perm = torch.randperm(length, generator=gen)
            idx_train = torch.sort(perm[:length - test_size]).values
            idx_test = torch.sort(perm[length - test_size:]).values
            self.data_x_train = data_x_train[idx_train.to(data_x_train.device)]
            self.data_y_train = data_y_train[idx_train.to(data_y_train.device)]
            self.data_x_test = data_x_train[idx_test.to(data_x_train.device)]
            self.data_y_test = data_y_train[idx_test.to(data_y_train.device)]
        elif data_x_test is None:
            self.data_x_train = self.data_x_test = data_x_train
            self.data_y_train = self.data_y_test = data_y_train
        else:
            self.data_x_train, self.data_y_train = data_x_train, data_y_train
            self.data_x_test, self.data_y_test = data_x_test, data_y_test
        self.detrended_y_test = None
        self.detrended_y_train = None
        self.mean_function = None
        self.n_train = int(self.data_x_train.shape[-2])
        self.n_test = int(self.data_x_test.shape[-2])
        self.n_inducting_train = max(20, int(self.n_train * global_param.p_nystroem_ratio))
        self.n_inducting_test = max(20, int(self.n_test * global_param.p_nystroem_ratio))

    def get_input_dimensionality(self) -> int:
        return int(self.data_x_train.shape[-1])

    def set_seed(self, seed: int):
        self.seed = seed

    def set_mean_function(self, mean_function):
        """Reset the detrended targets (AbstractDataInput.py:104-115)."""
        self.detrended_y_train = None
        self.detrended_y_test = None
        self.mean_function = mean_function
        if self.mean_function.get_last_hyper_parameter() is None:
            self.mean_function.last_hyper_parameter = self.mean_function.get_default_hyper_parameter()

    def is_batch(self) -> bool:
        return self.data_x_train.dim() == 3

    def _detrend(self, x, y):
        if isinstance(self.mean_function, bmf.ZeroMeanFunction):
            return y
        mf = self.mean_function
        if self.is_batch():
            means = torch.stack([mf.get_tf_tensor(mf.get_last_hyper_parameter(), xb).reshape(-1, 1) for xb in x])
        else:
            means = mf.get_tf_tensor(mf.get_last_hyper_parameter(), x).reshape(-1, 1)
        return y - means

    def get_detrended_y_train(self):
        """y - m(X) (DataInput.py:244-264); the zero mean returns y itself."""
        if self.mean_function is None:
            logging.error("Mean Function is None.")
            return None
        if self.detrended_y_train is None:
            self.detrended_y_train = self._detrend(self.data_x_train, self.data_y_train)
        return self.detrended_y_train

    def get_detrended_y_test(self):
        if self.mean_function is None:
            logging.error("Mean Function is None.")
            return None
        if self.detrended_y_test is None:
            self.detrended_y_test = self._detrend(self.data_x_test, self.data_y_test)
        return self.detrended_y_test

    def get_detrended_y_test_individual(self, data_x_test, data_y_test) -> torch.Tensor:
        """Detrended targets of a caller-given test set (DataInput.py:108-124): y itself (fp64) for the
        zero mean, else y - m(X) with the mean function's last hyperparameters; not memoised."""
        y = _f64(data_y_test)
        if isinstance(self.mean_function, bmf.ZeroMeanFunction):
            return y
        mf = self.mean_function
        return y - mf.get_tf_tensor(mf.get_last_hyper_parameter(), _f64(data_x_test)).reshape(-1, 1)

    def get_independent_smoothed_grid_subset(self, subset_size: int, smoothing_kernel=None):
        """Declared without a body in the reference (AbstractDataInput.py:138-139): None."""
        return None

    def get_x_range(self) -> List[List[float]]:
        """[min, max] per input dimension over train and test (DataInput.py:229-242)."""
        d = self.get_input_dimensionality()
        xa = torch.cat([self.data_x_train.reshape(-1, d), self.data_x_test.reshape(-1, d)], dim=0)
        lo = torch.min(xa, dim=0).values.tolist()
        hi = torch.max(xa, dim=0).values.tolist()
        return [[float(a), float(b)] for a, b in zip(lo, hi)]

    @staticmethod
    def get_k_fold_data_inputs(x_train, y_train, k: int, seed: int = 3061941):
        """k train/test folds from one seeded permutation (AbstractDataInput.py:147-168)."""
        length = x_train.shape[0]
        gen = torch.Generator().manual_seed(int(seed))
        perm = torch.randperm(length, generator=gen)
        sizes = [length // k] * (k - 1) + [length - (length // k) * (k - 1)]
        parts = list(torch.split(perm, sizes))
        out = []
        for i in range(k):
            te = torch.sort(parts[i]).values
            tr = torch.sort(torch.cat([parts[j] for j in range(k) if j != i])).values
            out.append(AbstractDataInput(x_train[tr], y_train[tr], x_train[te], y_train[te], seed=seed))
        return out


class DataInput(AbstractDataInput):
    """Single data set: X [N, D], y [N, 1] (DataInput.py:193-206)."""

    def __init__(self, data_x_train, data_y_train, data_x_test=None, data_y_test=None,
                 test_ratio: float = -1, seed: int = 3061941):
        if data_x_test is not None and data_y_test is not None:
            data_x_test, data_y_test = _f64(data_x_test), _f64(data_y_test)
        super().__init__(_f64(data_x_train), _f64(data_y_train), data_x_test, data_y_test, test_ratio, seed)


    def get_inducting_x_train(self, indices) -> torch.Tensor:
        """Rows of the training inputs at ``indices`` (DataInput.py:41-50)."""
        self.inducting_x_train = self.data_x_train[torch.as_tensor(indices, device=self.data_x_train.device)]
        return self.inducting_x_train

    def get_inducting_x_test(self, indices) -> torch.Tensor:
        self.inducting_x_test = self.data_x_test[torch.as_tensor(indices, device=self.data_x_test.device)]
        return self.inducting_x_test

    def _subset(self, idx):
        separate = not (self.data_x_train.shape == self.data_x_test.shape and
                        bool(torch.equal(self.data_x_train, self.data_x_test)))
        idx = idx.to(self.data_x_train.device)
        xs, ys = (self.data_x_test, self.data_y_test) if separate else (self.data_x_train, self.data_y_train)
        d = DataInput(self.data_x_train[idx], self.data_y_train[idx], xs, ys)
        d.set_mean_function(self.mean_function)
        return d

    def get_random_subset(self, subset_size: int):
        """subset_size training records drawn uniformly WITH replacement and sorted
        (DataInput.py:126-145).  The draw uses torch's generator seeded with self.seed, not
        TensorFlow's stateless Philox stream, so the indices differ from the reference's."""
        gen = torch.Generator().manual_seed(int(self.seed))
        idx = torch.sort(torch.randint(0, self.n_train, (int(subset_size),), generator=gen)).values
        return self._subset(idx)

    def get_grid_subset(self, subset_size: int):
        """Every (n / subset_size)-th training record: linspace(0, n, subset_size, endpoint=False)
        cast to int (DataInput.py:147-167) -- the reference's exact indices."""
        import numpy as np
        idx = torch.as_tensor(np.linspace(start=0, stop=self.n_train, num=int(subset_size), endpoint=False, dtype=int))
        return self._subset(idx)

    def is_equidistant_input_x(self) -> bool:
        """DataInput.py:169-170."""
        return is_equidistant(self.data_x_train)

    def get_subset(self, subset_size: int, subset_of_data_approach):
        from ..Metrics import MatrixHandlingTypes as mht
        if subset_of_data_approach is mht.SubsetOfDataApproaches.SOD_GRID:
            return self.get_grid_subset(subset_size)
        if subset_of_data_approach is mht.SubsetOfDataApproaches.SOD_RANDOM:
            return self.get_random_subset(subset_size)
        raise Exception("Invalid subset-of-data approach: %s" % str(subset_of_data_approach))


class BatchDataInput(AbstractDataInput):
    """B data sets evaluated together: X [B, N, D], y [B, N, 1] (BatchDataInput.py:24-28)."""

    def __init__(self, data_x_train, data_y_train, data_x_test=None, data_y_test=None,
                 test_ratio: float = -1, seed: int = 3061941):
        if data_x_test is not None and data_y_test is not None:
            data_x_test, data_y_test = _f64(data_x_test), _f64(data_y_test)
        super().__init__(_f64(data_x_train), _f64(data_y_train), data_x_test, data_y_test, test_ratio, seed)

    def is_equidistant_input_x(self):
        """BatchDataInput.py:97-98."""
        return is_equidistant_batch(self.data_x_train)

    # not implemented for batches in the reference either (BatchDataInput.py:30-34, :94-95, :100-101)
    def get_inducting_x_train(self, *args):
        raise Exception("get_inducting_x_train -- Not implemented for BatchDataInput.")

    def get_inducting_x_test(self, *args):
        raise Exception("get_inducting_x_test -- Not implemented for BatchDataInput.")

    def get_independent_smoothed_grid_subset(self, subset_size: int, smoothing_kernel=None):
        raise Exception("get_independent_smoothed_grid_subset -- Not implemented for BatchDataInput.")

    def get_subset(self, subset_size: int, subset_of_data_approach):
        raise Exception("get_subset -- Not implemented for BatchDataInput.")


class PartitionedDataInput(DataInput):
    """A data set together with the DataInput of each of its partitions (DataInput.py:191-207).
    The partitions are what SegmentedCovarianceMatrix factors as one ragged device batch."""

    def __init__(self, data_x_train, data_y_train, data_x_test, data_y_test, data_inputs: List[DataInput]):
        super().__init__(data_x_train, data_y_train, data_x_test, data_y_test)
        self.data_inputs: List[DataInput] = list(data_inputs)

    def set_mean_function(self, mean_function):
        """Also sets the mean function of every partition (DataInput.py:197-207)."""
        super().set_mean_function(mean_function)
        for d in self.data_inputs:
            d.set_mean_function(mean_function)


class BlockwiseDataInput(PartitionedDataInput):
    """Segments of a 1-D data set split at change points (DataInput.py:210-253): segment i holds
    the records with cp_{i-1} <= x < cp_i (open-ended at both ends)."""

    def __init__(self, data_x_train, data_y_train, data_x_test, data_y_test, change_points: List):
        xtr, ytr = _f64(data_x_train), _f64(data_y_train)
        xte, yte = _f64(data_x_test), _f64(data_y_test)
        cps = [float(torch.as_tensor(c, dtype=torch.float64).reshape(())) for c in change_points]
        blocks = []
        for i in range(len(cps) + 1):
            lo = cps[i - 1] if i > 0 else None
            hi = cps[i] if i < len(cps) else None

            def sel(x):
                m = torch.ones(x.shape[0], dtype=torch.bool, device=x.device)
                if hi is not None:
                    m &= (x < hi).any(dim=1)
                if lo is not None:
                    m &= (x >= lo).any(dim=1)
                return torch.nonzero(m).flatten()
            tr, te = sel(xtr), sel(xte)
            blocks.append(DataInput(xtr[tr], ytr[tr], xte[te], yte[te]))
        super().__init__(xtr, ytr, xte, yte, blocks)
