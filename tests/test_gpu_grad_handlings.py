"""-LML gradients beyond the DataInput + CHOLESKY_BASED case on the device: the BatchDataInput
aggregate (quirk Q7, M/LogLikelihood.py:62-63 -- the reference's fitter differentiates it through
tf.GradientTape, O/Fitter.py:124-132), STRICT / PSEUDO inverse of an indefinite K + noise I (the
eigendecomposition route; M/Metrics.py:132-136, :146-147) and AbstractMetric.get_gradients (M/Metrics.py:31,
called by O/ConjugateGradient.py:28-31).  Oracle: oracle/gp_autodiff.py (torch reverse mode).
Tolerances: -LML rel <= 1e-9, gradients |g - g_ref| <= 1e-7 max|g_ref| (1e-6 for the indefinite K, whose
inverse the Jacobi eigensolver supplies)."""
import numpy as np
import pytest
import torch

import gaussianprocessfundamentals_amd.global_parameters as gpar
from oracle import gp_autodiff as ad
from tests.helpers import hyp_list, make_kernel, set_flags
from tests.test_gpu_parity import build_gp

from gaussianprocessfundamentals_amd.Metrics import MatrixHandlingTypes as mht
from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type
from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType

pytestmark = pytest.mark.gpu
H = mht.NumericalMatrixHandlingType
F64 = torch.float64


def _close(got, exp, tol):
    got, exp = np.asarray(got, dtype=np.float64).ravel(), np.asarray(exp, dtype=np.float64).ravel()
    assert float(np.max(np.abs(got - exp))) <= tol * max(1e-300, float(np.max(np.abs(exp)))), (got, exp)


def _batch(B=3, n=150, d=1, seed=0):
    rng = np.random.default_rng(seed)
    xb = rng.uniform(0, 1, (B, n, d))
    yb = np.sin(5 * xb.sum(-1)) + 0.1 * rng.standard_normal((B, n))
    return xb, yb


@pytest.mark.parametrize("handling", [H.CHOLESKY_BASED, H.STRICT_INVERSE, H.PSEUDO_INVERSE])
@pytest.mark.parametrize("agg", ["mean", "sum"])
@pytest.mark.parametrize("tree,hyp,scaled", [(("SE", {}), [0.2], False),
                                             (("ADD", [("SE", {}), ("PER", {})]), [0.2, 0.8, 0.6], False),
                                             (("MAT52", {}), [0.3, 1.4], True)])
def test_batch_gradient_matches_oracle(handling, agg, tree, hyp, scaled):
    set_flags(scaled=scaled)
    gpar.p_batch_metric_aggregator = torch.mean if agg == "mean" else torch.sum
    try:
        xb, yb = _batch()
        met = get_metric_by_type(MetricType.LL, build_gp(tree, xb, yb), numerical_matrix_handling=handling)
        h = [torch.tensor(v, dtype=F64, requires_grad=True) for v in hyp]
        nz = torch.tensor(0.05, dtype=F64, requires_grad=True)
        out = met.get_metric(h, nz)
        out.sum().backward()
        nl, gh, gn = ad.batch_nlml_and_grad(tree, hyp, 0.05, xb, yb, handling.name, agg, scaled)
        assert abs(float(out.detach().reshape(-1)[0]) - nl) <= 1e-9 * abs(nl)
        _close([float(t.grad) for t in h] + [float(nz.grad)], [float(v) for v in gh] + [gn], 1e-7)
    finally:
        gpar.p_batch_metric_aggregator = torch.mean


@pytest.mark.parametrize("handling", [H.STRICT_INVERSE, H.PSEUDO_INVERSE])
def test_indefinite_covariance_gradient_matches_oracle(handling):
    """noise -0.3: K + noise I indefinite (the reference's LU inv / SVD pinv and slogdet handle it; the
    Cholesky-based gradient would be NaN)."""
    rng = np.random.default_rng(3)
    x = rng.uniform(0, 1, (300, 1))
    y = np.sin(6 * x[:, 0]) + 0.1 * rng.standard_normal(300)
    met = get_metric_by_type(MetricType.LL, build_gp(("SE", {}), x, y), numerical_matrix_handling=handling)
    h = [torch.tensor(0.1, dtype=F64, requires_grad=True)]
    nz = torch.tensor(-0.3, dtype=F64, requires_grad=True)
    out = met.get_metric(h, nz)
    out.sum().backward()
    nl, gh, gn = ad.inverse_nlml_and_grad(("SE", {}), [0.1], -0.3, x, y, handling.name)
    assert abs(float(out.detach()) - nl) <= 1e-8 * abs(nl)
    _close([float(h[0].grad), float(nz.grad)], [float(gh[0]), gn], 1e-6)


def test_get_gradients_is_the_device_gradient():
    rng = np.random.default_rng(9)
    x = rng.uniform(0, 1, (200, 2))
    y = np.sin(4 * x.sum(1))
    tree, hyp = ("ADD", [("SE", {}), ("MAT32", {"standard": True})]), [0.3, 0.5]
    met = get_metric_by_type(MetricType.LL, build_gp(tree, x, y))
    g = met.get_gradients(hyp_list(hyp), torch.tensor(0.02, dtype=F64))
    _, gref, _ = ad.nlml_and_grad(tree, hyp, 0.02, x, y)
    assert tuple(g.shape) == (2,)
    _close(g.cpu().numpy(), np.concatenate([np.ravel(v) for v in gref]), 1e-7)


@pytest.mark.parametrize("noise", [0.3, 1.0])
def test_lcg_gradient_matches_oracle(noise):
    """LINEAR_CONJUGATE_GRADIENT: the gradient tf.GradientTape takes through the executed CG iterations
    (Auxiliary/LinearConjugateGradients.py:9-41) plus slogdet's (M/Metrics.py:141-147), on the device
    (Auxiliary.LinearConjugateGradients.linear_cg_backward + gpk_kernel_vjp) vs the oracle's torch tape of the
    same loop (oracle.gp_autodiff.lcg_nlml_and_grad, pinned by finite differences in test_grad_oracle.py).
    The device GEMV and the host matmul round differently, which the CG recurrences carry: value rel <= 1e-9,
    gradient 1e-6 relative to its largest entry; the iteration counts agree."""
    from gaussianprocessfundamentals_amd.Auxiliary.LinearConjugateGradients import linear_cg
    rng = np.random.default_rng(8)
    x = rng.uniform(0, 1, (300, 1))
    y = np.sin(6 * x[:, 0]) + 0.1 * rng.standard_normal(300)
    met = get_metric_by_type(MetricType.LL, build_gp(("SE", {}), x, y),
                             numerical_matrix_handling=H.LINEAR_CONJUGATE_GRADIENT)
    h = [torch.tensor(0.1, dtype=F64, requires_grad=True)]
    nz = torch.tensor(noise, dtype=F64, requires_grad=True)
    out = met.get_metric(h, nz)
    out.sum().backward()
    nl, gh, gn, its = ad.lcg_nlml_and_grad(("SE", {}), [0.1], noise, x, y)
    tape = []
    K = met.get_covariance_matrix(hyp_list([0.1]), torch.tensor(noise, dtype=F64), None).contiguous()
    yd = met._y(None)
    linear_cg(K, yd, torch.zeros_like(yd), tape=tape)
    assert len(tape) == its
    assert abs(float(out.detach()) - nl) <= 1e-9 * abs(nl)
    _close([float(h[0].grad), float(nz.grad)], [float(gh[0]), gn], 1e-6)
    v, g2, gn2 = met.get_metric_and_gradient(hyp_list([0.1]), torch.tensor(noise, dtype=F64))
    _close([float(g2[0]), float(gn2)], [float(gh[0]), gn], 1e-6)


@pytest.mark.parametrize("handling", [H.CHOLESKY_BASED, H.STRICT_INVERSE])
def test_batch_gradient_with_an_indefinite_member_raises(handling):
    """BatchDataInput whose second member is not positive definite at noise -0.05 (dense SE inputs) while the
    first is (points 10 apart, K ~ I): the batched gradient raises CholeskyError -- as the reference's
    tf.linalg.cholesky does -- instead of returning NaN gradients beside an +inf value."""
    from gaussianprocessfundamentals_amd.engine import CholeskyError
    n = 120
    xb = np.stack([np.arange(n, dtype=np.float64).reshape(-1, 1) * 10.0,
                   np.sort(np.random.default_rng(2).uniform(0, 1, (n, 1)), axis=0)])
    yb = np.sin(3 * xb[..., 0])
    met = get_metric_by_type(MetricType.LL, build_gp(("SE", {}), xb, yb), numerical_matrix_handling=handling)
    with pytest.raises(CholeskyError):
        met.get_metric_and_gradient(hyp_list([0.2]), torch.tensor(-0.05, dtype=F64))
