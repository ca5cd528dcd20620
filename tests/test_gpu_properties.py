"""Hypothesis property tests of the device path (test layer 4): symmetry and unit diagonal of
K, invariance of the -LML under a joint permutation of the training points, the batch aggregation
quirk (Q7: data fit averaged, log-determinants summed) against single-problem evaluations, and
interpolation of the posterior mean at the training inputs.  Inputs, sizes and hyperparameters are
drawn by hypothesis (bounded so that K + noise I stays well conditioned: noise >= 1e-3).

Tolerances: K symmetric to 1e-15 (both triangles come from the same distances), k(x, x) = 1 to 1e-15
(unscaled kernels); -LML permutation rel <= 1e-10, against the oracle rel <= 1e-9; batch quirk
rel <= 1e-10; posterior mean at the training points within 1e-3 of y at noise 1e-6 (interpolation)."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, example, given, settings
from hypothesis import strategies as st

from oracle import gp_oracle as o
from tests.helpers import hyp_list, make_kernel

from gaussianprocessfundamentals_amd.DataHandling.DataInput import BatchDataInput, DataInput
from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction
from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type
from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType
from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import GaussianProcess

pytestmark = pytest.mark.gpu

BASES = [("SE", {"ard": False}), ("MAT32", {}), ("MAT52", {}), ("PER", {})]
SETTINGS = settings(max_examples=15, deadline=None, suppress_health_check=[HealthCheck.too_slow])


def hyp_for(tree, ls, per):
    return [ls, per] if tree[0] == "PER" else [ls]


def gp_for(tree, x, y):
    di = DataInput(x, y.reshape(-1, 1), x[:4], y[:4].reshape(-1, 1))
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(make_kernel(tree, 1), ZeroMeanFunction(1))
    g.set_data_input(di)
    return g


@SETTINGS
@given(b=st.integers(0, 3), n=st.integers(1, 300), seed=st.integers(0, 2 ** 31 - 1),
       ls=st.floats(0.02, 2.0), per=st.floats(0.2, 2.0))
# the case hypothesis found in round 4 (gpurun_out/r04fin3_tests.log): the contracted form of the periodic
# entry's sa cb - ca sb left |K - K^T| = 1.1e-15; fixed in gpk_kernels.h by rounding both products
@example(b=3, n=31, seed=0, ls=0.0625, per=1.0)
def test_kernel_matrix_symmetric_unit_diagonal(b, n, seed, ls, per):
    tree = BASES[b]
    x = np.random.default_rng(seed).uniform(-2, 2, (n, 1))
    K = make_kernel(tree, 1).get_tf_tensor(hyp_list(hyp_for(tree, ls, per)), x, x).cpu().numpy()
    assert np.max(np.abs(K - K.T)) <= 1e-15
    assert np.max(np.abs(np.diag(K) - 1.0)) <= 1e-15


@pytest.mark.parametrize("standard", [False, True])
@pytest.mark.parametrize("n,seed,ls,per", [(31, 0, 0.0625, 1.0), (300, 1, 0.02, 0.2), (257, 7, 0.5, 1.7),
                                           (64, 3, 2.0, 0.37)])
def test_periodic_kernel_matrix_bitwise_symmetric(n, seed, ls, per, standard):
    """Deterministic pin of the round-4 regression (the hypothesis example above): K(x, x) of the periodic kernel
    is bitwise symmetric, for the reference form and the per-dimension standard form, at D = 1 and D = 3."""
    for d in (1, 3):
        x = np.random.default_rng(seed).uniform(-2, 2, (n, d))
        K = make_kernel(("PER", {"standard": standard}), d).get_tf_tensor(hyp_list([ls, per]), x, x).cpu().numpy()
        assert np.array_equal(K.view(np.uint64), K.T.view(np.uint64)), (d, float(np.max(np.abs(K - K.T))))


@SETTINGS
@given(b=st.integers(0, 2), n=st.integers(2, 400), seed=st.integers(0, 2 ** 31 - 1),
       ls=st.floats(0.05, 1.0), noise=st.floats(1e-3, 1.0))
def test_nlml_invariant_under_permutation(b, n, seed, ls, noise):
    tree = BASES[b]
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, 1, (n, 1))
    y = np.sin(5 * x[:, 0]) + 0.1 * rng.standard_normal(n)
    perm = rng.permutation(n)
    nz = torch.tensor(noise, dtype=torch.float64)
    a = float(get_metric_by_type(MetricType.LL, gp_for(tree, x, y)).get_metric(hyp_list([ls]), nz))
    c = float(get_metric_by_type(MetricType.LL, gp_for(tree, x[perm], y[perm])).get_metric(hyp_list([ls]), nz))
    assert abs(a - c) <= 1e-10 * max(1.0, abs(a))
    assert abs(a - o.nlml(tree, [ls], noise, x, y)) <= 1e-9 * max(1.0, abs(a))


@SETTINGS
@given(batch=st.integers(1, 4), n=st.integers(2, 200), seed=st.integers(0, 2 ** 31 - 1),
       ls=st.floats(0.05, 1.0), noise=st.floats(1e-3, 1.0))
def test_batch_quirk_against_single_problems(batch, n, seed, ls, noise):
    """BatchDataInput -LML = -(mean_b(-fit_b / 2) - sum_b(logdet_b) / 2 - n log(2 pi) / 2)
    (LogLikelihood.py:39-63 with the axis-free reduce_sum of Metrics.py:152-154)."""
    tree = BASES[0]
    rng = np.random.default_rng(seed)
    x = np.sort(rng.uniform(0, 1, (batch, n, 1)), axis=1)
    y = np.sin(4 * x[..., 0]) + 0.1 * rng.standard_normal((batch, n))
    di = BatchDataInput(x, y[..., None], x[:, :3], y[:, :3, None], test_ratio=0)
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(make_kernel(tree, 1), ZeroMeanFunction(1))
    g.set_data_input(di)
    nz = torch.tensor(noise, dtype=torch.float64)
    got = float(get_metric_by_type(MetricType.LL, g).get_metric(hyp_list([ls]), nz))
    fits, dets = [], []
    for b in range(batch):
        K = o.k_noised(tree, [ls], noise, x[b])
        L = np.linalg.cholesky(K)
        z = np.linalg.solve(L, y[b])
        fits.append(float(z @ z))
        dets.append(2.0 * np.sum(np.log(np.diag(L))))
    ref = -((-0.5 * np.mean(fits)) + (-0.5 * np.sum(dets)) + (-0.5 * n * np.log(2 * np.pi)))
    assert abs(got - ref) <= 1e-10 * max(1.0, abs(ref))


@SETTINGS
@given(n=st.integers(2, 60), seed=st.integers(0, 2 ** 31 - 1))
def test_posterior_mean_interpolates_training_points(n, seed):
    tree = BASES[0]
    rng = np.random.default_rng(seed)
    x = np.linspace(0, 1, n).reshape(-1, 1) + 0.2 * rng.uniform(-1, 1) / n
    y = np.sin(3 * x[:, 0])
    di = DataInput(x, y.reshape(-1, 1), x, y.reshape(-1, 1))
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(make_kernel(tree, 1), ZeroMeanFunction(1))
    g.set_data_input(di)
    _, _, mu = g.predict(hyp_list([0.5 / n]), noise=torch.tensor(1e-6, dtype=torch.float64))
    assert np.max(np.abs(mu.cpu().numpy().reshape(-1) - y)) <= 1e-3
