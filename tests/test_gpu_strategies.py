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


@pytest.mark.parametrize("handling", [H.STRICT_INVERSE, H.PSEUDO_INVERSE])
def test_handlings_of_an_indefinite_covariance(handling):
    """K + noise I with a negative noise is indefinite: the Cholesky reports it, and STRICT_INVERSE /
    PSEUDO_INVERSE + slogdet fall back to the eigendecomposition (gpk_syevd), as the reference's LU-based
    tf.linalg.inv / SVD-based pinv / slogdet handle it.  NLL rel <= 1e-8 (cond(K) ~ 1e3 here)."""
    g, x, y, _, _ = setup(n=300)
    noise = -0.3
    K = o.k_noised(SE, [0.1], noise, x)
    assert np.min(np.linalg.eigvalsh(K)) < 0
    met = get_metric_by_type(MetricType.LL, g, numerical_matrix_handling=handling)
    got = float(met.get_metric(hyp_list([0.1]), T(noise)).reshape(-1)[0])
    alpha = (np.linalg.inv(K) if handling is H.STRICT_INVERSE else o.tf_pinv(K)) @ y
    ref = o.nlml_with_alpha(alpha, y, np.linalg.slogdet(K)[1], 300)
    assert rel(got, ref) <= 1e-8, (got, ref)


@pytest.mark.parametrize("handling,n", [(H.STRICT_INVERSE, 4096), (H.PSEUDO_INVERSE, 4096), (H.PSEUDO_INVERSE, 6144)])
def test_handlings_of_an_indefinite_covariance_large(handling, n):
    """The same at n = 4096 and 6144 (the eigendecomposition fallback, gpk_syevd, whose top merges sort in HBM
    above 4096): K - 0.3 I of n SE inputs.  Reference alpha / log|det| from numpy's eigh (no eigenvalue near
    tf.linalg.pinv's cutoff here, so pinv = inv); NLL rel <= 1e-8."""
    g, x, y, _, _ = setup(n=n)
    noise = -0.3
    K = o.k_noised(SE, [0.1], noise, x)
    lam, V = np.linalg.eigh(K)
    assert lam[0] < 0 and np.min(np.abs(lam)) > 1e-3
    met = get_metric_by_type(MetricType.LL, g, numerical_matrix_handling=handling)
    got = float(met.get_metric(hyp_list([0.1]), T(noise)).reshape(-1)[0])
    alpha = V @ ((V.T @ y) / lam)
    ref = o.nlml_with_alpha(alpha, y, float(np.sum(np.log(np.abs(lam)))), n)
    assert rel(got, ref) <= 1e-8, (got, ref)


@pytest.mark.parametrize("handling", [H.STRICT_INVERSE, H.PSEUDO_INVERSE])
def test_handlings_of_an_indefinite_covariance_beyond_16384(handling):
    """the eigendecomposition fallback above its old n <= 16384 cap (Metrics.py raised there; the
    reference's tf.linalg.inv / pinv take any n, M/Metrics.py:132-136).  n = 16400 SE inputs in 8 clusters 10 apart,
    shuffled: K - 0.3 I is a permuted block-diagonal indefinite matrix, so the reference alpha and log|det| come
    from numpy's eigh block by block (no eigenvalue near pinv's cutoff: pinv = inv).  NLL rel <= 1e-8."""
    n, nc, noise = 16400, 8, -0.3
    rng = np.random.default_rng(100)
    per = n // nc
    x = np.concatenate([10.0 * c + rng.uniform(0, 1, per) for c in range(nc)])
    perm = rng.permutation(n)
    xs = x[perm]
    y = np.sin(6 * xs) + 0.1 * np.random.default_rng(7).standard_normal(n)
    fit, logdet = 0.0, 0.0
    for c in range(nc):
        idx = np.nonzero((xs >= 10.0 * c) & (xs < 10.0 * c + 1.0))[0]
        lam, V = np.linalg.eigh(o.k_noised(SE, [0.1], noise, xs[idx].reshape(-1, 1)))
        assert np.min(np.abs(lam)) > 1e-3
        fit += float(y[idx] @ (V @ ((V.T @ y[idx]) / lam)))
        logdet += float(np.sum(np.log(np.abs(lam))))
    ref = 0.5 * fit + 0.5 * logdet + 0.5 * n * np.log(2.0 * np.pi)
    di = DataInput(xs.reshape(-1, 1), y.reshape(-1, 1), xs[:8].reshape(-1, 1), y[:8].reshape(-1, 1))
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(make_kernel(SE, 1), ZeroMeanFunction(1))
    g.set_data_input(di)
    met = get_metric_by_type(MetricType.LL, g, numerical_matrix_handling=handling)
    got = float(met.get_metric(hyp_list([0.1]), T(noise)).reshape(-1)[0])
    print("n = %d %s: -LML %.12g vs numpy blockwise %.12g (rel %.2e)" % (n, handling.name, got, ref, rel(got, ref)))
    assert rel(got, ref) <= 1e-8, (got, ref)


def test_pseudo_inverse_of_a_singular_covariance():
    """Duplicated inputs and zero noise: K is singular (rank 150 of 300), pinv truncates below
    10 n eps max|lam| exactly like tf.linalg.pinv.  alpha compared through K alpha (= the projection
    of y on K's range, O(1)), max-abs <= 1e-6: the kept eigenvalues reach down to the cutoff, where
    pinv amplifies the eigensolvers' rounding differences (alpha itself is O(1e3))."""
    rng = np.random.default_rng(3)
    xh = np.sort(rng.uniform(0, 1, (150, 1)), axis=0)
    x = np.concatenate([xh, xh])
    y = np.sin(6 * x[:, 0])
    di = DataInput(x, y.reshape(-1, 1), x[:5], y[:5].reshape(-1, 1))
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(make_kernel(SE, 1), ZeroMeanFunction(1))
    g.set_data_input(di)
    met = get_metric_by_type(MetricType.LL, g, numerical_matrix_handling=H.PSEUDO_INVERSE)
    alpha = met.get_alpha(hyp_list([0.5]), T(0.0), None).cpu().numpy().reshape(-1)
    K = o.k_noised(SE, [0.5], 0.0, x)
    ref = o.tf_pinv(K) @ y
    assert np.max(np.abs(K @ alpha - K @ ref)) <= 1e-6
