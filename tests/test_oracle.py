"""The CPU oracle against closed-form answers and its own committed golden vectors."""
import numpy as np
import pytest

from oracle import gp_oracle as o
from tests.helpers import golden

SE = ("SE", {"ard": False})


@pytest.mark.parametrize("name,got,exp", o.known_answers())
def test_known_answer(name, got, exp):
    assert abs(got - exp) <= 1e-12 * max(1.0, abs(exp)), name


def test_expanded_norm_exact_on_1d_diagonal_and_nan_in_8d():
    x = np.random.default_rng(0).uniform(0, 1, (500, 1))
    d = o.euclidian_distance(x, x)
    assert np.all(np.diag(d) == 0.0)
    x8 = np.random.default_rng(1).uniform(0, 1, (500, 8))
    assert np.isnan(np.diag(o.euclidian_distance(x8, x8))).any()


def test_batch_quirk_logdet_summed_fit_averaged():
    rng = np.random.default_rng(2)
    xb = rng.uniform(0, 1, (3, 20, 1))
    yb = rng.standard_normal((3, 20))
    comps = [o.nlml_components(SE, [0.3], 0.1, xb[b], yb[b]) for b in range(3)]
    ld = sum(c["logdet"] for c in comps)
    exp = -np.mean([-0.5 * c["fit"] - 0.5 * ld - 10 * o.LOG_2PI for c in comps])
    assert abs(o.batch_nlml(SE, [0.3], 0.1, xb, yb) - exp) < 1e-10


def test_l1_forms_are_indefinite_beyond_1d():
    x, y = o.make_inputs("C3", n=600)
    K = o.kernel_matrix(("MAT52", {"ard": True}), [[0.25, 0.5, 0.75, 1.0]], x, x)
    assert np.linalg.eigvalsh(K)[0] < -0.1
    Ks = o.kernel_matrix(("MAT52", {"ard": True, "standard": True}), [[0.25, 0.5, 0.75, 1.0]], x, x)
    assert np.linalg.eigvalsh(Ks)[0] > -1e-10
    x1 = x[:, :1]
    for op in ("MAT52", "MAT32", "PER"):
        hyp = [0.3, 0.4] if op == "PER" else [0.3]
        a = o.kernel_matrix((op, {}), hyp, x1, x1)
        b = o.kernel_matrix((op, {"standard": True}), hyp, x1, x1)
        np.testing.assert_allclose(a, b, rtol=1e-14, atol=1e-15)


def test_golden_c1_recomputes():
    g = golden("c1_se_n256")
    c = o.nlml_components(SE, [0.1], 1e-8, g["x"], g["y"])
    assert abs(c["nlml"] - float(g["nlml"])) <= 1e-9 * abs(float(g["nlml"]))
    np.testing.assert_allclose(c["L"], g["L"], rtol=0, atol=1e-12)


def test_golden_small_trees_recompute():
    g = golden("small_trees")
    tree = ("MUL", [("ADD", [SE, ("MAT32", {})]), ("PER", {})])
    got = o.nlml(tree, list(g["hyp"]), 1e-3, g["x"], g["y"], scaled=True)
    assert abs(got - float(g["nlml_scaled_tree"])) <= 1e-10 * abs(got)
    assert abs(o.batch_nlml(SE, [0.2], 1e-2, g["xb"], g["yb"]) - float(g["nlml_batch"])) < 1e-9


def test_golden_inputs_are_reproducible():
    """The large configs regenerate their inputs from a seed: pin the generator."""
    from tests.golden.make_golden import digest
    for name, cfg in (("c3_mat52ard_n8192", "C3"), ("c5_seard_per_n16384", "C5")):
        g = golden(name)
        x, y = o.make_inputs(cfg)
        assert digest(x) == str(g["x_sha256"]) and digest(y) == str(g["y_sha256"])
    g = golden("c2_se_n4096")
    x, y = o.make_inputs("C2")
    np.testing.assert_array_equal(x, g["x"])


# ------------------------------------------------------------------ approximations (§8f.4)
def test_nystroem_with_all_points_is_exact():
    """Inducing points = training points: K_hat = K, so the Nystroem determinant is logdet(K + s I)
    and SKC's correction is n s / (2 jitter)."""
    rng = np.random.default_rng(2)
    x = np.linspace(0, 1, 12).reshape(-1, 1)
    y = rng.standard_normal(12)
    tree = ("SE", {"ard": False})
    K = o.k_noised(tree, [0.1], 1e-2, x)
    assert abs(o.nystroem_det(tree, [0.1], 1e-2, x, x) - np.linalg.slogdet(K)[1]) < 1e-9
    exact = o.nlml(tree, [0.1], 1e-2, x, y)
    for h in ("CHOLESKY_BASED", "STRICT_INVERSE", "PSEUDO_INVERSE"):
        assert abs(o.nystroem_nlml(tree, [0.1], 1e-2, x, y, x, handling=h) - exact) < 1e-8 * abs(exact)
    lb = o.nystroem_nlml(tree, [0.1], 1e-2, x, y, x, lower_bound=True, jitter=1e-8)
    assert abs(lb - (exact + 12 * 1e-2 / (2 * 1e-8))) < 1e-6 * abs(lb)


def test_nystroem_indefinite_kmm_known_answers():
    """The reference's default L1 Matern-5/2 at D = 4 gives an indefinite K_mm (negative eigenvalues above
    tf.linalg.pinv's cutoff).  The restated Woodbury inverse (Nystroem_K.py:73-90) is then still the inverse of
    K_hat + noise I, and the restated determinant (:92-108) its log|det| (Sylvester: det(noise I_n + K_nm P K_mn)
    = noise^(n - m) det(noise I_m + K_mn K_nm P)) -- the identities the device's symmetric forms rely on."""
    rng = np.random.default_rng(21)
    x, z = rng.uniform(0, 1, (120, 4)), rng.uniform(0, 1, (30, 4))
    tree, hyp = ("MAT52", {"ard": True}), [[1.0, 1.0, 1.0, 1.0]]
    kmm = o.kernel_matrix(tree, hyp, z, z)
    lam = np.linalg.eigvalsh(kmm)
    assert lam[0] < -10 * 30 * np.finfo(np.float64).eps * np.abs(lam).max()
    for noise in (0.5, 1e-2):
        khat, _, _ = o.nystroem_k_approx(tree, hyp, x, z)
        A = khat + noise * np.eye(120)
        inv = o.nystroem_k_approx_inv(tree, hyp, noise, x, z)
        np.testing.assert_allclose(inv @ A, np.eye(120), atol=1e-8 * np.abs(inv).max() * np.abs(A).max())
        assert abs(o.nystroem_det(tree, hyp, noise, x, z) - np.linalg.slogdet(A)[1]) < 1e-9 * 120


def test_ski_weights_on_inducing_points_and_midpoints():
    z = np.array([[0.0], [1.0], [2.0]])
    w = o.ski_weight_matrix(z, z)
    assert np.array_equal(w, np.eye(3))
    x = np.array([[0.25], [1.5]])
    w = o.ski_weight_matrix(x, z)
    # x = 1.5 is equidistant from 1 and 2: BOTH are "nearest" (weight 1 - 0.5 / (0.5 + 1.5) each, with
    # the masking offset = the global max distance 1.5) and 0 becomes the second nearest -- the
    # reference's tie behaviour, rows need not sum to 1
    assert np.allclose(w, [[0.75, 0.25, 0.0], [0.25, 0.75, 0.75]])
    # all points inducing: K_ski = K + s I, so every handling gives the exact -LML
    xs = np.linspace(0, 1, 10).reshape(-1, 1)
    y = np.cos(3 * xs[:, 0])
    tree = ("SE", {"ard": False})
    exact = o.nlml(tree, [0.2], 1e-2, xs, y)
    assert abs(o.ski_nlml(tree, [0.2], 1e-2, xs, y, 10, handling="STRICT_INVERSE") - exact) < 1e-8 * abs(exact)
    assert list(o.ski_inducing_indices(10, 4)) == [0, 2, 5, 7]


def test_vsgd_step_burnin_cap():
    g = np.array([[1.0], [-2.0], [0.0]])
    a = o.vsgd_step(np.ones_like(g), g)
    assert np.allclose(a, 1 - 1e-6 * g)
    big = np.array([[1e6]])            # 2 / (0.05 * 0.9025 g^2) < 1e-6: the adaptive rate wins
    lr = 2.0 / (0.05 * (0.95e6) ** 2)
    assert np.allclose(o.vsgd_step(np.ones((1, 1)), big), 1 - lr * 1e6)


def test_function_draw_restatements():
    # prior draw with z = I and standardised targets is L itself: L L^T = K_ss + noise I
    xt = np.linspace(0.0, 1.0, 9).reshape(9, 1)
    y = np.array([-1.0, 1.0])  # mean 0, population std 1
    L = o.n_prior_functions(SE, [0.2], 1e-2, xt, y, np.eye(9))
    assert np.allclose(L @ L.T, o.k_noised(SE, [0.2], 1e-2, xt), atol=1e-14)
    # posterior draw with z = 0 is the posterior mean
    x, yy = o.make_inputs("C1", n=64)
    mu, _ = o.posterior(SE, [0.1], 1e-2, x, yy, xt)
    f = o.n_posterior_functions(SE, [0.1], 1e-2, x, yy, xt, np.zeros((9, 2)), 1e-8)
    assert np.array_equal(f, np.repeat(mu.reshape(-1, 1), 2, axis=1))


def test_bench_inputs_match_the_oracle_generator():
    """bench.py restates the SURVEY §8(d) generator (the measured path imports nothing from oracle/):
    it must produce the golden vectors' inputs bit for bit."""
    import bench
    for cfg, n in (("C2", 4096), ("C4", 512), ("metric", 8192), ("C3", 777), ("C5", 300)):
        a, b = bench.synthetic_inputs(cfg, n), o.make_inputs(cfg, n=n)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), cfg
