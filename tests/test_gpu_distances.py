"""Auxiliary/Distances.py on the device (gpk_distance_matrix) against the oracle's restatement
(A/Distances.py:4-12).  Bars: manhattan and the direct euclidean rel <= 1e-14 (elementwise fp64,
same operation order up to the summation over d); the expanded-norm euclidean max-abs <= 1e-7 where
both are finite (sqrt of a cancellation-prone argument: the error is sqrt(eps |a|^2)), and NaN
exactly where the oracle's argument is negative by more than rounding can flip."""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as o

from gaussianprocessfundamentals_amd.Auxiliary import Distances as dist

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,m,d", [(1, 1, 1), (300, 257, 1), (130, 70, 4), (64, 64, 8)])
def test_manhattan_and_direct_euclidean(n, m, d):
    rng = np.random.default_rng(n + m + d)
    a, b = rng.uniform(0, 1, (n, d)), rng.uniform(0, 1, (m, d))
    got = dist.manhattan_distance(a, b).cpu().numpy()
    ref = o.manhattan_distance(a, b)
    assert got.shape == (n, m) and np.allclose(got, ref, rtol=1e-14, atol=1e-15)
    got2 = dist.euclidean_distance_direct(a, b).cpu().numpy()
    assert np.allclose(got2, np.sqrt(o.squared_l2_direct(a, b)), rtol=1e-14, atol=1e-15)


@pytest.mark.parametrize("d", [1, 4, 8])
def test_expanded_euclidean_quirk(d):
    rng = np.random.default_rng(d)
    a = rng.uniform(0, 1, (200, d))
    got = dist.euclidian_distance(a, a).cpu().numpy()
    ref = o.euclidian_distance(a, a)
    both = np.isfinite(got) & np.isfinite(ref)
    assert np.max(np.abs(got[both] - ref[both])) <= 1e-7
    if d == 1:
        assert np.all(np.isfinite(got))  # exact for D = 1
    else:
        # the reference's unclamped sqrt reaches NaN on the diagonal (the norms and the matmul round
        # differently); where exactly depends on the summation order, so only its presence is pinned
        assert np.isnan(np.diag(got)).any() and np.isnan(np.diag(ref)).any()


def test_batched_and_broadcast():
    rng = np.random.default_rng(7)
    a, b = rng.uniform(0, 1, (3, 50, 2)), rng.uniform(0, 1, (1, 40, 2))
    got = dist.manhattan_distance(a, b).cpu().numpy()
    assert got.shape == (3, 50, 40)
    for i in range(3):
        assert np.allclose(got[i], o.manhattan_distance(a[i], b[0]), rtol=1e-14, atol=1e-15)
    with pytest.raises(ValueError):
        dist.manhattan_distance(a, rng.uniform(0, 1, (2, 40, 2)))


def test_more_rows_than_one_grid_dimension():
    """n > 65535 rows (the kernel's gridDim.y bound): split into launches over row ranges."""
    rng = np.random.default_rng(11)
    a, b = rng.uniform(0, 1, (70000, 2)), rng.uniform(0, 1, (5, 2))
    got = dist.manhattan_distance(a, b).cpu().numpy()
    assert got.shape == (70000, 5) and np.allclose(got, o.manhattan_distance(a, b), rtol=1e-14, atol=1e-15)
