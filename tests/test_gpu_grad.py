"""-LML gradient and explicit inverses on the HIP path vs the autodiff oracle (needs the MI355X).

Oracle: oracle/gp_autodiff.py (torch reverse mode of the restated reference op sequence, the
gradient tf.GradientTape takes in gpbasics/Optimizer/Fitter.py:104-158), itself pinned by finite
differences in tests/test_grad_oracle.py.
The oracle tests run through both single-evaluation paths (the launch path and the persistent launch, fixture
factor_path); the schedule tests below are launch-path only (tests/conftest.py).
Tolerances (fp64): -LML rel <= 1e-9; gradient |g - g_ref| <= 1e-7 * max(1, |g_ref|_max) per
hyperparameter set; K^-1 / L^-1 normwise relative error <= 1e-8 (noise >= 1e-2).
"""
import math

import numpy as np
import pytest
import torch

from oracle import gp_autodiff as ad
from oracle import gp_oracle as o
from tests.helpers import hyp_list, make_kernel, set_flags
from tests.test_gpu_parity import build_gp
from tests.test_grad_oracle import GRAD_CASES, _inputs

from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type
from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType

pytestmark = pytest.mark.gpu

SE = ("SE", {})


def _metric(tree, x, y):
    return get_metric_by_type(MetricType.LL, build_gp(tree, x, y))


def _check_grad(got, exp, tol=1e-7):
    scale = max(1.0, max(float(np.max(np.abs(e))) for e in exp))
    for g, e in zip(got, exp):
        np.testing.assert_allclose(np.asarray(g), np.asarray(e).reshape(np.shape(g)), rtol=0, atol=tol * scale)


@pytest.mark.parametrize("case", range(len(GRAD_CASES)))
@pytest.mark.parametrize("n", [70, 333])
def test_gradient_matches_autodiff_oracle(case, n, factor_path):
    """Through both factorisation paths of a single evaluation (fixture factor_path): the launch path and the
    persistent launch of the identity-augmented factorisation (gpk_tune chain_eye)."""
    tree, hyp, d, scaled, expanded = GRAD_CASES[case]
    set_flags(scaled=scaled, expanded=expanded)
    x, y = _inputs(n, d, 100 + case)
    noise = 0.05
    nl_ref, g_ref, gn_ref = ad.nlml_and_grad(tree, hyp, noise, x, y, scaled, expanded)
    m = _metric(tree, x, y)
    nl, grads, gn = m.get_metric_and_gradient(hyp_list(hyp), torch.tensor(noise, dtype=torch.float64))
    assert abs(float(nl) - nl_ref) <= 1e-9 * abs(nl_ref)
    _check_grad([g.cpu().numpy() for g in grads] + [float(gn)], list(g_ref) + [gn_ref])


def test_autograd_backward_uses_device_gradient(factor_path):
    tree, hyp = ("ADD", [("SE", {}), ("PER", {})]), [0.3, 0.9, 0.5]
    x, y = _inputs(257, 1, 7)
    h = [torch.tensor(v, dtype=torch.float64, requires_grad=True) for v in hyp]
    nz = torch.tensor(0.02, dtype=torch.float64, requires_grad=True)
    m = _metric(tree, x, y)
    out = m.get_metric(h, nz)
    assert out.shape == (1, 1) and out.requires_grad
    (2.0 * out.sum()).backward()
    nl_ref, g_ref, gn_ref = ad.nlml_and_grad(tree, hyp, 0.02, x, y)
    assert abs(float(out) - nl_ref) <= 1e-9 * abs(nl_ref)
    _check_grad([float(t.grad) for t in h] + [float(nz.grad)],
                [2.0 * g for g in g_ref] + [2.0 * gn_ref])
    # no grad requested: the plain (cheaper) factorisation path, no graph
    with torch.no_grad():
        assert not m.get_metric(h, nz).requires_grad


def test_gradient_at_multi_group_sizes_and_inverse():
    """n spans several panel groups (group_eye 1 / 3 / 4 / 8) with a ragged end (the zero-tile skipping of
    the identity rows is exercised on every schedule variant); K^-1 and L^-1 against numpy."""
    x, y = o.make_inputs("C1", n=1100, seed=11)
    for group in (1, 3, 4, 8):
        old = engine.nat.tune("group_eye", group)
        try:
            f = build_gp(SE, x, y).covariance_matrix.inverse_factorization(hyp_list([0.1]), torch.tensor(1e-2, dtype=torch.float64))
            Kn = o.k_noised(SE, [0.1], 1e-2, x)
            Ki = np.linalg.inv(Kn)
            got = f.k_inv(0).cpu().numpy()
            assert np.linalg.norm(got - Ki) / np.linalg.norm(Ki) < 1e-8
            Li = np.linalg.inv(np.linalg.cholesky(Kn))
            assert np.linalg.norm(f.l_inv(0).cpu().numpy() - Li) / np.linalg.norm(Li) < 1e-8
            a = np.linalg.solve(Kn, y)
            np.testing.assert_allclose(f.alpha(0).cpu().numpy(), a, rtol=1e-7, atol=1e-7 * np.abs(a).max())
            nl_ref, g_ref, gn_ref = ad.nlml_and_grad(SE, [0.1], 1e-2, x, y)
            g = f.gradient()[0].cpu().numpy()
            _check_grad([g[:1], g[1]], [g_ref[0], gn_ref])
        finally:
            engine.nat.tune("group_eye", old)


def test_batched_gradient_members_are_independent():
    x, y = _inputs(300, 1, 3)
    k = make_kernel(SE, 1)
    kd = engine.kernel_descriptor(k, 1)
    cands = [0.08, 0.2, 0.5]
    f = engine.InverseFactorization(300, 1, len(cands), torch.float64)
    dev = engine.device()
    H = torch.tensor([[c] for c in cands], dtype=torch.float64, device=dev)
    X = torch.as_tensor(x, device=dev)
    Y = torch.as_tensor(y, device=dev).reshape(1, -1).contiguous()
    f.run(kd, H, 1, torch.tensor([0.03], dtype=torch.float64, device=dev), 0, X, 0, Y, 0)
    G = f.gradient().cpu().numpy()
    for b, c in enumerate(cands):
        nl_ref, g_ref, gn_ref = ad.nlml_and_grad(SE, [c], 0.03, x, y)
        assert abs(float(f.nlml()[b]) - nl_ref) <= 1e-9 * abs(nl_ref)
        _check_grad([G[b, :1], G[b, 1]], [g_ref[0], gn_ref])


def test_gradient_not_positive_definite_is_nan():
    x = np.linspace(0, 1, 200).reshape(-1, 1)
    y = np.sin(x[:, 0])
    m = _metric(SE, x, y)
    nl, grads, gn = m.get_metric_and_gradient(hyp_list([0.5]), torch.tensor(-1.0, dtype=torch.float64))
    assert math.isinf(float(nl)) and math.isnan(float(gn)) and math.isnan(float(grads[0]))


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_gradient_under_every_in_group_schedule(mode):
    """The identity-augmented factorisation (K^-1 rows, structurally zero tiles skipped) under the
    left-looking, right-looking and two-level in-group schedules, over several panel groups."""
    old = engine.nat.tune("ingroup", mode)
    try:
        x, y = o.make_inputs("C1", n=1100, seed=12)
        f = build_gp(SE, x, y).covariance_matrix.inverse_factorization(hyp_list([0.1]), torch.tensor(1e-2, dtype=torch.float64))
        Kn = o.k_noised(SE, [0.1], 1e-2, x)
        Ki = np.linalg.inv(Kn)
        assert np.linalg.norm(f.k_inv(0).cpu().numpy() - Ki) / np.linalg.norm(Ki) < 1e-8
        nl_ref, g_ref, gn_ref = ad.nlml_and_grad(SE, [0.1], 1e-2, x, y)
        g = f.gradient()[0].cpu().numpy()
        _check_grad([g[:1], g[1]], [g_ref[0], gn_ref])
        assert abs(float(f.nlml()[0]) - nl_ref) <= 1e-9 * abs(nl_ref)
    finally:
        engine.nat.tune("ingroup", old)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [2, 3])
def test_zero_band_skip_is_bitwise_neutral(mode):
    """Leaving the zero band's tiles out of the grid (band_skip, the default) changes which workgroups
    exist, not what any tile computes: K^-1, the gradient and the -LML match the full grid bit for bit,
    for a batch (two-level in-group schedule) and a single member (right-looking)."""
    x, y = o.make_inputs("C1", n=1300, seed=13)
    g = build_gp(SE, x, y)
    batch = 3 if mode == 3 else 1
    hyp = [0.08] if batch == 1 else None
    res = {}
    old_mode = engine.nat.tune("ingroup", mode)
    try:
        for skip in (0, 1):
            old = engine.nat.tune("band_skip", skip)
            try:
                if batch == 1:
                    f = g.covariance_matrix.inverse_factorization(hyp_list(hyp), torch.tensor(1e-2, dtype=torch.float64))
                    res[skip] = (f.k_inv(0).cpu().numpy().copy(), f.gradient().cpu().numpy().copy(),
                                 f.nlml().cpu().numpy().copy())
                else:
                    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
                    dev = engine.device()
                    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
                    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
                    H = torch.tensor([[0.06], [0.1], [0.14]], dtype=torch.float64, device=dev)
                    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
                    f = engine.InverseFactorization(len(x), 1, batch).run(kd, H, 1, NZ, 0, X, 0, Y, 0)
                    res[skip] = (f.k_inv(2).cpu().numpy().copy(), f.gradient().cpu().numpy().copy(),
                                 f.nlml().cpu().numpy().copy())
            finally:
                engine.nat.tune("band_skip", old)
    finally:
        engine.nat.tune("ingroup", old_mode)
    for a, b in zip(res[0], res[1]):
        assert np.array_equal(a, b)
