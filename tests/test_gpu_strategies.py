"""Numerical handlings other than CHOLESKY_BASED and subset-of-data metrics on the device vs the
oracle (needs the MI355X).

Tolerances: STRICT / PSEUDO inverse NLL rel <= 1e-9 (noise 1e-2, cond(K) ~ 1e4); the linear-CG
NLL is approximate by construction (stopping rule |max r| <= 1e-2): compared with the oracle's
own CG restatement at rel <= 1e-3 and with the exact NLL at rel <= 1e-2; GEMV max-abs <= 1e-12
relative to the row norms."""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as o
from tests.helpers import hyp_list, make_kernel

from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd.DataHandling.DataInput import DataInput
from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction
from gaussianprocessfundamentals_amd.Metrics import MatrixHandlingTypes as mht
from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type
from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType
from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import GaussianProcess

pytestmark = pytest.mark.gpu

SE = ("SE", {"ard": False})
NOISE = 1e-2
H = mht.NumericalMatrixHandlingType


def T(v):
    return torch.tensor(v, dtype=torch.float64)


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


def setup(n=700, n_test=90, seed=3):
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, 1, (n, 1))
    y = np.sin(6 * x[:, 0]) + 0.1 * rng.standard_normal(n)
    xt = rng.uniform(0, 1, (n_test, 1))
    yt = np.sin(6 * xt[:, 0])
    di = DataInput(x, y.reshape(-1, 1), xt, yt.reshape(-1, 1))
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(make_kernel(SE, 1), ZeroMeanFunction(1))
    g.set_data_input(di)
    return g, x, y, xt, yt


@pytest.mark.parametrize("n,m", [(1, 1), (5, 3), (130, 257), (1000, 1000), (333, 4097)])
def test_gemv_matches_numpy(n, m):
    rng = np.random.default_rng(n + m)
    A = rng.standard_normal((n, m + 3))
    x = rng.standard_normal(m)
    At = torch.tensor(A, device="cuda")[:, :m]          # lda = m + 3 (odd strides, unaligned rows)
    got = engine.gemv(At, torch.tensor(x, device="cuda")).cpu().numpy()
    ref = A[:, :m] @ x
    assert np.max(np.abs(got - ref) / (np.abs(A[:, :m]) @ np.abs(x) + 1e-300)) < 1e-13
    y0 = rng.standard_normal(n)
    yt = torch.tensor(y0, device="cuda")
    engine.gemv(At, torch.tensor(x, device="cuda"), yt, alpha=2.0, beta=-0.5)
    np.testing.assert_allclose(yt.cpu().numpy(), 2.0 * ref - 0.5 * y0, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("handling", [H.STRICT_INVERSE, H.PSEUDO_INVERSE])
def test_inverse_handlings_match_exact_nlml(handling):
    g, x, y, xt, yt = setup()
    m = get_metric_by_type(MetricType.LL, g, numerical_matrix_handling=handling)
    got = float(m.get_metric(hyp_list([0.12]), T(NOISE)))
    assert rel(got, o.nlml(SE, [0.12], NOISE, x, y)) < 1e-9
    mse = get_metric_by_type(MetricType.MSE, g, numerical_matrix_handling=handling)
    assert rel(float(mse.get_metric(hyp_list([0.12]), T(NOISE))), o.mse(SE, [0.12], NOISE, x, y, xt, yt)) < 1e-8


def test_linear_cg_handling_matches_oracle_cg():
    g, x, y, _, _ = setup(n=500)
    m = get_metric_by_type(MetricType.LL, g, numerical_matrix_handling=H.LINEAR_CONJUGATE_GRADIENT)
    got = float(m.get_metric(hyp_list([0.12]), T(NOISE)))
    A = o.k_noised(SE, [0.12], NOISE, x)
    a_cg = o.linear_cg(A, y, np.zeros(len(y)))
    logdet = float(np.linalg.slogdet(A)[1])
    ref_cg = o.nlml_with_alpha(a_cg, y, logdet, len(y))
    assert rel(got, ref_cg) < 1e-3, (got, ref_cg)
    assert rel(got, o.nlml(SE, [0.12], NOISE, x, y)) < 1e-2


def test_subset_of_data_grid_is_exact_on_the_grid_subset():
    g, x, y, _, _ = setup(n=800)
    m = get_metric_by_type(MetricType.LL, g, local_approx=mht.SubsetOfDataApproaches.SOD_GRID, subset_size=200)
    got = float(m.get_metric(hyp_list([0.12]), T(NOISE)))
    idx = np.linspace(0, 800, 200, endpoint=False, dtype=int)
    assert rel(got, o.nlml(SE, [0.12], NOISE, x[idx], y[idx])) < 1e-9
    # SOD_RANDOM: an exact evaluation on the drawn subset (torch's generator, see DataInput)
    r = get_metric_by_type(MetricType.LL, g, local_approx=mht.SubsetOfDataApproaches.SOD_RANDOM, subset_size=150)
    sub = r.data_input
    got_r = float(r.get_metric(hyp_list([0.12]), T(NOISE)))
    assert rel(got_r, o.nlml(SE, [0.12], NOISE, sub.data_x_train.cpu().numpy(),
                              sub.data_y_train.cpu().numpy().reshape(-1))) < 1e-9
