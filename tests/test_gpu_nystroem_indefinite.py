"""Nystroem with an INDEFINITE K_mm (needs the MI355X): the reference's default L1 Matern-5/2 at D = 4
(K/BaseKernels.py, Auxiliary/Distances.py:10-12) is not positive semidefinite beyond D = 1, and
tf.linalg.pinv + slogdet still give the reference a value (Statistics/Nystroem_K.py:49-55, :73-108).  The device
takes the signed symmetric forms (Statistics/Nystroem_K.py docstring): log|det(noise S + G^T G)| on gpk_syevd, the
Woodbury inverse with (noise S + G^T G)^-1, and the signed reverse mode (Metrics/_approx_grad.py).

Oracle: oracle/gp_oracle.py (nystroem_det, nystroem_k_approx_inv -- the reference's Woodbury with pinv, op for op --
nystroem_nlml) and oracle/gp_autodiff.py (torch's tape of the same ops, slogdet of the nonsymmetric matrix).
Tolerances: determinant and -LML rel 1e-9 (eigenvalue-accurate log|det| of an m = 30 matrix), inverse 1e-8
normwise, gradients 1e-6 max-relative (the indefinite C is inverted through its eigendecomposition)."""
import numpy as np
import pytest
import torch

from oracle import gp_autodiff as ad
from oracle import gp_oracle as o
from tests.helpers import make_kernel

from gaussianprocessfundamentals_amd.DataHandling.DataInput import DataInput
from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction
from gaussianprocessfundamentals_amd.Metrics import MatrixHandlingTypes as mht
from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type
from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType
from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import GaussianProcess

pytestmark = pytest.mark.gpu

F64 = torch.float64
TREE = ("MAT52", {"ard": True})        # the reference form: L1 distance of the scaled inputs
HYP = [[1.0, 1.0, 1.0, 1.0]]
N, M, D = 120, 30, 4


def _inputs(seed=21):
    rng = np.random.default_rng(seed)
    x, z = rng.uniform(0, 1, (N, D)), rng.uniform(0, 1, (M, D))
    y = np.sin(3 * x.sum(1)) + 0.1 * rng.standard_normal(N)
    return x, y, z


def _gp(x, y):
    di = DataInput(x, y.reshape(-1, 1), x[:5], y[:5].reshape(-1, 1))
    di.set_mean_function(ZeroMeanFunction(D))
    g = GaussianProcess(make_kernel(TREE, D), ZeroMeanFunction(D))
    g.set_data_input(di)
    return g


def _metric(g, handling):
    return get_metric_by_type(MetricType.LL, g, mht.MatrixApproximations.BASIC_NYSTROEM, handling, subset_size=M)


def test_kmm_is_indefinite_above_the_cutoff():
    _, _, z = _inputs()
    lam = np.linalg.eigvalsh(o.kernel_matrix(TREE, HYP, z, z))
    assert (lam < -10 * M * np.finfo(np.float64).eps * np.abs(lam).max()).sum() >= 2


@pytest.mark.parametrize("noise", [0.5, 1e-2])
def test_determinant_and_inverse_match_the_oracle(noise):
    x, y, z = _inputs()
    met = _metric(_gp(x, y), mht.NumericalMatrixHandlingType.STRICT_INVERSE)
    nys = met.nystroem_matrix
    h = [torch.tensor(v, dtype=F64) for v in HYP]
    zt = torch.tensor(z, dtype=F64)
    det = float(nys.get_K_approx_det(h, torch.tensor(noise, dtype=F64), zt))
    exp = o.nystroem_det(TREE, HYP, noise, x, z)
    print("indefinite K_mm, noise %g: det %.12g vs oracle %.12g (rel %.2e)" % (noise, det, exp, abs(det - exp) / abs(exp)))
    assert abs(det - exp) <= 1e-9 * abs(exp)
    inv = nys.get_K_approx_inv(h, torch.tensor(noise, dtype=F64), zt).cpu().numpy()
    inv_exp = o.nystroem_k_approx_inv(TREE, HYP, noise, x, z)
    assert np.max(np.abs(inv - inv_exp)) <= 1e-8 * np.max(np.abs(inv_exp))


@pytest.mark.parametrize("handling", ["STRICT_INVERSE", "PSEUDO_INVERSE"])
@pytest.mark.parametrize("noise", [0.5, 1e-2])
def test_metric_matches_the_oracle(handling, noise):
    x, y, z = _inputs()
    met = _metric(_gp(x, y), mht.NumericalMatrixHandlingType[handling])
    got = float(met.get_metric([torch.tensor(v, dtype=F64) for v in HYP], torch.tensor(noise, dtype=F64),
                               torch.tensor(z, dtype=F64)))
    exp = o.nystroem_nlml(TREE, HYP, noise, x, y, z, handling=handling)
    assert abs(got - exp) <= 1e-9 * abs(exp), (got, exp)


@pytest.mark.parametrize("noise", [0.5, 1e-2])
def test_gradient_matches_the_oracle(noise):
    x, y, z = _inputs()
    met = _metric(_gp(x, y), mht.NumericalMatrixHandlingType.STRICT_INVERSE)
    h = [torch.tensor(v, dtype=F64, requires_grad=True) for v in HYP]
    nz = torch.tensor(noise, dtype=F64, requires_grad=True)
    zt = torch.tensor(z, dtype=F64, requires_grad=True)
    out = met.get_metric(h, nz, zt)
    out.sum().backward()
    nl, gh, gn, gz = ad.nystroem_nlml_and_grad(TREE, HYP, noise, x, y, z, "STRICT_INVERSE")
    assert abs(float(out.detach()) - nl) <= 1e-9 * abs(nl)
    got = np.concatenate([h[0].grad.numpy().reshape(-1), [float(nz.grad)]])
    exp = np.concatenate([np.asarray(gh[0]).reshape(-1), [gn]])
    assert np.max(np.abs(got - exp)) <= 1e-6 * np.max(np.abs(exp)), (got, exp)
    assert np.max(np.abs(zt.grad.numpy() - gz)) <= 1e-6 * np.max(np.abs(gz))


def _inputs_with_a_duplicate(seed=21):
    """The same inputs with the last inducing input replaced by a copy of the first: K_mm keeps its negative
    eigenvalues and gains an exact zero one, below tf.linalg.pinv's cutoff (dropped)."""
    x, y, z = _inputs(seed)
    z = z.copy()
    z[-1] = z[0]
    return x, y, z


def test_kmm_with_a_duplicate_is_indefinite_with_a_dropped_eigenvalue():
    _, _, z = _inputs_with_a_duplicate()
    lam = np.linalg.eigvalsh(o.kernel_matrix(TREE, HYP, z, z))
    cut = 10 * M * np.finfo(np.float64).eps * np.abs(lam).max()
    assert (lam < -cut).sum() >= 2 and (np.abs(lam) <= cut).sum() == 1


@pytest.mark.parametrize("handling", ["STRICT_INVERSE", "PSEUDO_INVERSE"])
def test_indefinite_kmm_with_dropped_eigenvalues_metric_and_gradient(handling):
    """the signed reverse mode where an indefinite K_mm also has eigenvalues below the cutoff (the
    kept x dropped block of pinv's reverse mode, Metrics/_approx_grad.py nystroem_logdet) -- value rel 1e-9,
    gradients 1e-6 max-relative against the autodiff oracle (torch's tape through pinv's SVD with TF's cutoff)."""
    x, y, z = _inputs_with_a_duplicate()
    noise = 0.5
    met = _metric(_gp(x, y), mht.NumericalMatrixHandlingType[handling])
    h = [torch.tensor(v, dtype=F64, requires_grad=True) for v in HYP]
    nz = torch.tensor(noise, dtype=F64, requires_grad=True)
    zt = torch.tensor(z, dtype=F64, requires_grad=False)
    out = met.get_metric(h, nz, zt)
    exp_v = o.nystroem_nlml(TREE, HYP, noise, x, y, z, handling=handling)
    print("duplicate inducing input, %s: -LML %.12g vs oracle %.12g" % (handling, float(out.detach()), exp_v))
    assert abs(float(out.detach()) - exp_v) <= 1e-9 * abs(exp_v)
    out.sum().backward()
    nl, gh, gn, _ = ad.nystroem_nlml_and_grad(TREE, HYP, noise, x, y, z, handling)
    assert abs(nl - exp_v) <= 1e-9 * abs(exp_v)
    got = np.concatenate([h[0].grad.numpy().reshape(-1), [float(nz.grad)]])
    exp = np.concatenate([np.asarray(gh[0]).reshape(-1), [gn]])
    print("gradient", got, "oracle", exp)
    assert np.max(np.abs(got - exp)) <= 1e-6 * np.max(np.abs(exp)), (got, exp)
