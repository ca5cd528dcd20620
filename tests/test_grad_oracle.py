"""The gradient oracle (torch reverse mode of the restated reference op sequence) pinned by
(a) its forward value == the numpy oracle's -LML and (b) central finite differences of it."""
import numpy as np
import pytest

from oracle import gp_autodiff as ad
from oracle import gp_oracle as o

# (tree, hyp, d, scaled, se_expanded): every base kernel, both operators, ARD, standard forms
GRAD_CASES = [
    (("SE", {}), [0.3], 1, False, False),
    (("SE", {}), [0.3, 1.7], 1, True, False),
    (("SE", {}), [0.45], 1, False, True),
    (("PER", {}), [0.8, 0.6], 1, False, False),
    (("PER", {"standard": True}), [0.9, 0.7, 1.3], 2, True, False),
    (("MAT32", {}), [-0.35], 1, False, False),
    (("MAT52", {}), [0.4, 0.8], 1, True, False),
    (("MAT52", {"ard": True, "standard": True}), [[0.5, 0.9, 1.4]], 3, False, False),
    (("MAT32", {"ard": True}), [[0.6]], 1, False, False),
    (("MAT32", {"ard": True, "standard": True}), [[0.6, 1.1]], 2, False, False),
    (("SE", {"ard": True}), [[0.4, 0.7], 1.5], 2, True, False),
    (("ADD", [("SE", {}), ("PER", {})]), [0.3, 0.9, 0.5], 1, False, False),
    (("MUL", [("SE", {}), ("MAT52", {})]), [0.5, 0.6], 1, False, False),
    (("MUL", [("ADD", [("SE", {}), ("MAT32", {})]), ("PER", {})]), [0.4, 0.7, 1.0, 0.8], 1, False, False),
]


def _inputs(n, d, seed):
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, 1, (n, d))
    y = np.sin(4 * x.sum(1)) + 0.1 * rng.standard_normal(n)
    return x, y


@pytest.mark.parametrize("case", range(len(GRAD_CASES)))
def test_autodiff_oracle_matches_value_and_finite_differences(case):
    tree, hyp, d, scaled, expanded = GRAD_CASES[case]
    x, y = _inputs(40, d, case)
    noise = 0.05
    nl, grads, gnoise = ad.nlml_and_grad(tree, hyp, noise, x, y, scaled, expanded)
    assert abs(nl - o.nlml(tree, hyp, noise, x, y, scaled, expanded)) < 1e-10 * max(1.0, abs(nl))
    f = lambda h, nz: o.nlml(tree, h, nz, x, y, scaled, expanded)
    fd, fdn = ad.finite_difference(f, hyp, noise)
    for g, e in zip(grads, fd):
        np.testing.assert_allclose(g, e, rtol=1e-5, atol=1e-6)
    assert abs(gnoise - fdn) < 1e-5 * max(1.0, abs(fdn))


# Nystroem / SKC / SKI gradient oracle (SURVEY §8f.1 x §8f.4): value == gp_oracle's, gradients == central
# differences on well-conditioned K_mm (short length scales: FD through a near-singular pinv is noise)
NYS_CASES = [
    ("CHOLESKY_BASED", False, ("SE", {}), [0.03], False),
    ("CHOLESKY_BASED", True, ("SE", {}), [0.03, 1.3], True),
    ("STRICT_INVERSE", False, ("MAT52", {}), [0.05], False),
    ("PSEUDO_INVERSE", True, ("ADD", [("SE", {}), ("PER", {})]), [0.03, 0.5, 1.7], False),
]


@pytest.mark.parametrize("case", range(len(NYS_CASES)))
def test_nystroem_gradient_oracle_matches_finite_differences(case):
    handling, lower, tree, hyp, scaled = NYS_CASES[case]
    x, y = o.make_inputs("C1", n=120, seed=3)
    z = np.sort(np.random.default_rng(case).uniform(0, 1, (12, 1)), axis=0)
    noise, jitter = 0.05, 1e-3
    f = lambda h, nz, zz=z: o.nystroem_nlml(tree, h, nz, x, y, zz, handling, lower, jitter, scaled)
    nl, g, gn, gz = ad.nystroem_nlml_and_grad(tree, hyp, noise, x, y, z, handling, lower, jitter, scaled)
    assert abs(nl - f(hyp, noise)) < 1e-9 * abs(nl)
    fd, fdn = ad.finite_difference(f, hyp, noise, h=1e-6)
    for a, e in zip(g, fd):
        np.testing.assert_allclose(a, e, rtol=2e-5, atol=1e-5)
    assert abs(gn - fdn) < 2e-5 * max(1.0, abs(fdn))
    for j in (0, 5, 11):
        zp, zm = z.copy(), z.copy()
        zp[j, 0] += 1e-6
        zm[j, 0] -= 1e-6
        e = (f(hyp, noise, zp) - f(hyp, noise, zm)) / 2e-6
        assert abs(gz[j, 0] - e) < 2e-4 * max(1.0, abs(e)), (j, gz[j, 0], e)


def test_ski_gradient_oracle_matches_finite_differences():
    x, y = o.make_inputs("C1", n=100, seed=4)
    tree, hyp, noise = ("SE", {}), [0.08], 0.05
    f = lambda h, nz: o.ski_nlml(tree, h, nz, x, y, 20, "STRICT_INVERSE")
    nl, g, gn = ad.ski_nlml_and_grad(tree, hyp, noise, x, y, 20, "STRICT_INVERSE")
    assert abs(nl - f(hyp, noise)) < 1e-9 * abs(nl)
    fd, fdn = ad.finite_difference(f, hyp, noise, h=1e-6)
    np.testing.assert_allclose(g[0], fd[0], rtol=2e-5)
    assert abs(gn - fdn) < 2e-5 * max(1.0, abs(fdn))


@pytest.mark.parametrize("handling,agg", [("CHOLESKY_BASED", "mean"), ("CHOLESKY_BASED", "sum"),
                                          ("STRICT_INVERSE", "mean"), ("PSEUDO_INVERSE", "sum")])
def test_batch_gradient_oracle_matches_value_and_finite_differences(handling, agg):
    rng = np.random.default_rng(1)
    xb = rng.uniform(0, 1, (3, 40, 1))
    yb = np.sin(5 * xb.sum(-1)) + 0.1 * rng.standard_normal((3, 40))
    tree, hyp = ("ADD", [("SE", {}), ("PER", {})]), [0.2, 0.8, 0.6]
    nl, g, gn = ad.batch_nlml_and_grad(tree, hyp, 0.05, xb, yb, handling, agg)
    if handling == "CHOLESKY_BASED" and agg == "mean":
        assert abs(nl - o.batch_nlml(tree, hyp, 0.05, xb, yb)) < 1e-10 * abs(nl)
    f = lambda h, nz: ad.batch_nlml_and_grad(tree, h, nz, xb, yb, handling, agg)[0]
    fd, fdn = ad.finite_difference(f, hyp, 0.05, h=1e-6)
    for a, e in zip(g, fd):
        np.testing.assert_allclose(a, e, rtol=1e-5, atol=1e-5)
    assert abs(gn - fdn) < 1e-5 * max(1.0, abs(fdn))


@pytest.mark.parametrize("handling", ["STRICT_INVERSE", "PSEUDO_INVERSE"])
def test_indefinite_gradient_oracle_matches_finite_differences(handling):
    x, y = _inputs(60, 1, 5)
    nl, g, gn = ad.inverse_nlml_and_grad(("SE", {}), [0.1], -0.3, x, y, handling)
    K = o.k_noised(("SE", {}), [0.1], -0.3, x)
    assert np.min(np.linalg.eigvalsh(K)) < 0
    ref = o.nlml_with_alpha(np.linalg.inv(K) @ y, y, np.linalg.slogdet(K)[1], 60)
    assert abs(nl - ref) < 1e-9 * abs(ref)
    f = lambda h, nz: ad.inverse_nlml_and_grad(("SE", {}), h, nz, x, y, handling)[0]
    fd, fdn = ad.finite_difference(f, [0.1], -0.3, h=1e-6)
    np.testing.assert_allclose(g[0], fd[0], rtol=1e-5)
    assert abs(gn - fdn) < 1e-5 * max(1.0, abs(fdn))


@pytest.mark.parametrize("n,ls,noise", [(40, 0.1, 0.3), (40, 0.05, 0.5), (60, 0.1, 1.0)])
def test_lcg_gradient_oracle_matches_finite_differences(n, ls, noise):
    """LINEAR_CONJUGATE_GRADIENT: the restated CG loop's value and its tape gradient.  The iterate depends
    smoothly on the hyperparameters while the number of executed iterations stays fixed, so the
    finite-difference steps are checked to run the same iteration count.  (With small noise the CG iterate
    is so sensitive to rounding that central differences of it are noise below h ~ 1e-4 -- the tape's
    gradient is still exact for the executed operations -- so the checks use noise >= 0.3.)"""
    x, y = _inputs(n, 1, 8)
    nl, g, gn, its = ad.lcg_nlml_and_grad(("SE", {}), [ls], noise, x, y)
    assert its >= 3
    h = 1e-6
    for dh in (h, -h):
        assert ad.lcg_nlml_and_grad(("SE", {}), [ls + dh], noise, x, y)[3] == its
        assert ad.lcg_nlml_and_grad(("SE", {}), [ls], noise + dh, x, y)[3] == its
    f = lambda hh, nz: ad.lcg_nlml_and_grad(("SE", {}), hh, nz, x, y)[0]
    fd, fdn = ad.finite_difference(f, [ls], noise, h=h)
    np.testing.assert_allclose(g[0], fd[0], rtol=1e-6)
    assert abs(gn - fdn) < 1e-6 * max(1.0, abs(fdn))


@pytest.mark.parametrize("approx", ["NYSTROEM", "SKC_LOWER", "SKI"])
def test_approximation_lcg_gradient_oracle_matches_finite_differences(approx):
    """LINEAR_CONJUGATE_GRADIENT under BASIC_NYSTROEM / SKC_LOWER_BOUND / SKI (M/Metrics.py:141-147 on the
    approximate matrix): the value equals gp_oracle's, the tape gradient through the executed CG iterations
    equals central differences (same iteration count at the perturbed points)."""
    x, y = o.make_inputs("C1", n=80, seed=6)
    tree, hyp, noise = ("SE", {}), [0.05], 0.4
    if approx == "SKI":
        f = lambda h, nz: o.ski_nlml(tree, h, nz, x, y, 20, "LINEAR_CONJUGATE_GRADIENT")
        nl, g, gn = ad.ski_nlml_and_grad(tree, hyp, noise, x, y, 20, "LINEAR_CONJUGATE_GRADIENT")
        gz = None
    else:
        lower = approx == "SKC_LOWER"
        z = np.sort(np.random.default_rng(2).uniform(0, 1, (10, 1)), axis=0)
        f = lambda h, nz: o.nystroem_nlml(tree, h, nz, x, y, z, "LINEAR_CONJUGATE_GRADIENT", lower, 1e-3)
        nl, g, gn, gz = ad.nystroem_nlml_and_grad(tree, hyp, noise, x, y, z, "LINEAR_CONJUGATE_GRADIENT", lower, 1e-3)
        assert gz is not None
    assert abs(nl - f(hyp, noise)) < 1e-9 * abs(nl)
    fd, fdn = ad.finite_difference(f, hyp, noise, h=1e-6)
    np.testing.assert_allclose(g[0], fd[0], rtol=1e-5, atol=1e-6)
    assert abs(gn - fdn) < 1e-5 * max(1.0, abs(fdn))


@pytest.mark.parametrize("k_fresh,det_fresh", [(True, True), (True, False), (False, True)])
def test_skc_upper_bound_gradient_oracle(k_fresh, det_fresh):
    """The SKC upper bound's tape gradient: alpha (one VariationalSGD step, a variable assignment) is a
    constant, so the gradient is the partial derivative of 1/2 a^T K a - a^T y - 1/2 det at the stepped a --
    checked by central differences of that expression with a held fixed; cached K / determinant contribute
    nothing."""
    x, y = o.make_inputs("C1", n=90, seed=5)
    z = np.sort(np.random.default_rng(3).uniform(0, 1, (12, 1)), axis=0)
    tree, hyp, noise = ("SE", {}), [0.04], 0.05
    val, g, gn, gz = ad.skc_upper_nlml_and_grad(tree, hyp, noise, x, y, z, k_fresh, det_fresh)
    assert abs(val - o.skc_upper_bound(tree, hyp, noise, x, y, z)) < 1e-9 * abs(val)
    yv = y.reshape(-1, 1)
    n = len(y)
    K0 = o.k_noised(tree, hyp, noise, x)
    a = o.vsgd_step(np.ones((n, 1)), (K0 @ np.ones((n, 1)) - yv) + K0 @ np.ones((n, 1)))
    det0 = o.nystroem_det(tree, hyp, noise, x, z)

    def f(h, nz):
        K = o.k_noised(tree, h, nz, x) if k_fresh else K0
        det = o.nystroem_det(tree, h, nz, x, z) if det_fresh else det0
        return 0.5 * float((a.T @ K @ a)[0, 0]) - float((a.T @ yv)[0, 0]) - 0.5 * det
    fd, fdn = ad.finite_difference(f, hyp, noise, h=1e-6)
    np.testing.assert_allclose(g[0], fd[0], rtol=1e-5, atol=1e-6)
    assert abs(gn - fdn) < 1e-5 * max(1.0, abs(fdn))
    if not det_fresh:
        assert gz is None or np.all(gz == 0)
