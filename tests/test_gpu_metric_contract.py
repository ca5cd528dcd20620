"""Contract of LogLikelihood.get_metric's return values (needs the MI355X).

* independence: every returned -LML is a tensor of its own -- later evaluations (which reuse the
  covariance object's factorisation buffers) must not change it, as the reference's fresh TF tensors
  never change (gpbasics/Metrics/LogLikelihood.py:30-65);
* a BatchDataInput with one member that is not positive definite gives +inf for the aggregate (no
  NaN leaking through the summed log-determinant, Q7) and get_metric_checked raises CholeskyError
  (the reference's tf.linalg.cholesky raises, Statistics/CovarianceMatrix.py:250);
* the value under autograd equals the value without it for every numerical handling that supports
  gradients; LINEAR_CONJUGATE_GRADIENT refuses gradients instead of pairing its CG value with the
  exact gradient.
"""
import math

import numpy as np
import pytest
import torch

from oracle import gp_oracle as o
from tests.helpers import hyp_list
from tests.test_gpu_parity import build_gp

from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd.Metrics import MatrixHandlingTypes as mht
from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type
from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType

pytestmark = pytest.mark.gpu

SE = ("SE", {})
H = mht.NumericalMatrixHandlingType


def _nz(v):
    return torch.tensor(v, dtype=torch.float64)


def test_returned_metrics_are_independent_of_later_calls():
    x, y = o.make_inputs("C1", n=300, seed=3)
    m = get_metric_by_type(MetricType.LL, build_gp(SE, x, y))
    cands = [0.05, 0.1, 0.3]
    outs = [m.get_metric(hyp_list([c]), _nz(1e-2)) for c in cands]
    vals = [float(t) for t in outs]
    assert len(set(vals)) == 3
    for c, v in zip(cands, vals):
        assert abs(v - o.nlml(SE, [c], 1e-2, x, y)) <= 1e-9 * abs(v)
    first = outs[0].clone()
    m.get_metric(hyp_list([0.7]), _nz(0.5))
    assert torch.equal(outs[0], first)
    nl, grads, gn = m.get_metric_and_gradient(hyp_list([0.2]), _nz(1e-2))
    keep = (nl.clone(), grads[0].clone(), gn.clone())
    m.get_metric_and_gradient(hyp_list([0.4]), _nz(3e-2))
    assert torch.equal(nl, keep[0]) and torch.equal(grads[0], keep[1]) and torch.equal(gn, keep[2])


def test_batch_with_one_indefinite_member_is_inf_not_nan():
    n = 120
    far = (np.arange(n, dtype=np.float64) * 10.0).reshape(n, 1)  # K ~ I: K - 0.5 I stays PD
    near = np.linspace(0.0, 1.0, n).reshape(n, 1)                # K - 0.5 I indefinite
    x = np.stack([far, near])
    y = np.sin(x[..., 0])
    g = build_gp(SE, x, y, x[:, :3], y[:, :3, None])
    m = get_metric_by_type(MetricType.LL, g)
    got = float(m.get_metric(hyp_list([0.1]), _nz(-0.5)))
    assert math.isinf(got) and got > 0
    with pytest.raises(engine.CholeskyError):
        m.get_metric_checked(hyp_list([0.1]), _nz(-0.5))
    # both members PD: finite, as before
    assert math.isfinite(float(m.get_metric(hyp_list([0.1]), _nz(1e-2))))


@pytest.mark.parametrize("handling", [H.CHOLESKY_BASED, H.STRICT_INVERSE, H.PSEUDO_INVERSE])
def test_value_is_the_same_with_and_without_autograd(handling):
    x, y = o.make_inputs("C1", n=200, seed=9)
    m = get_metric_by_type(MetricType.LL, build_gp(SE, x, y), numerical_matrix_handling=handling)
    plain = float(m.get_metric(hyp_list([0.15]), _nz(2e-2)))
    h = torch.tensor(0.15, dtype=torch.float64, requires_grad=True)
    out = m.get_metric([h], _nz(2e-2))
    assert out.requires_grad
    assert abs(float(out) - plain) <= 1e-12 * abs(plain)
    out.sum().backward()
    assert h.grad is not None and math.isfinite(float(h.grad))


def test_linear_cg_differentiates():
    # round 3: LINEAR_CONJUGATE_GRADIENT carries a CG tape instead of refusing requires_grad
    x, y = o.make_inputs("C1", n=100, seed=2)
    m = get_metric_by_type(MetricType.LL, build_gp(SE, x, y), numerical_matrix_handling=H.LINEAR_CONJUGATE_GRADIENT)
    assert math.isfinite(float(m.get_metric(hyp_list([0.15]), _nz(2e-2))))
    h = torch.tensor(0.15, dtype=torch.float64, requires_grad=True)
    v = m.get_metric([h], _nz(2e-2))
    (g,) = torch.autograd.grad(v, [h])
    assert math.isfinite(float(g)) and float(g) != 0.0
