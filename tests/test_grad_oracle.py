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
