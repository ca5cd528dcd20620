"""The tridiagonal eigensolver gpk_syevd (Householder tridiagonalisation, compact-WY Q, implicit QL) against numpy's eigh, and the pseudo-inverse built on it against
tf.linalg.pinv's restatement (oracle.tf_pinv) -- the spectral half of Statistics/Nystroem_K.py:53 and of the
non-positive-definite handlings (Metrics/Metrics.py:132-147).  Tolerances: eigenvalues |lam - lam_ref| <=
1e-13 m max|lam| (as sets: QL leaves them unsorted, as the Jacobi solver did); residual ||A V - V diag(lam)|| and ||V^T V - I|| (max-abs) <= 1e-12 m max(1, max|lam|)."""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as o
from gaussianprocessfundamentals_amd import engine

pytestmark = pytest.mark.gpu


def _check(A, lam, V):
    m = A.shape[0]
    lam, V = lam.cpu().numpy(), V.cpu().numpy()
    ref = np.linalg.eigvalsh(A)
    sc = max(1.0, float(np.max(np.abs(ref))))
    assert np.max(np.abs(np.sort(lam) - ref)) <= 1e-13 * m * sc, np.max(np.abs(np.sort(lam) - ref))
    assert np.max(np.abs(A @ V - V * lam)) <= 1e-12 * m * sc
    assert np.max(np.abs(V.T @ V - np.eye(m))) <= 1e-12 * m


@pytest.mark.parametrize("m", [1, 2, 3, 17, 64, 130, 409, 1000])
def test_syevd_random_symmetric(m):
    rng = np.random.default_rng(m)
    A = rng.standard_normal((m, m))
    A = 0.5 * (A + A.T)
    lam, V = engine.syevd(torch.tensor(A, device="cuda"))
    _check(A, lam, V)


def test_syevd_clusters_and_zero_tail():
    """Repeated eigenvalues, a tight cluster and a tail below the pinv cutoff (QL's rotations keep the vectors of a
    cluster orthonormal)."""
    rng = np.random.default_rng(3)
    m = 300
    Q, _ = np.linalg.qr(rng.standard_normal((m, m)))
    lam = np.concatenate([np.full(40, 2.0), 1.0 + 1e-13 * rng.standard_normal(30), np.geomspace(0.5, 1e-6, 130),
                          1e-17 * rng.uniform(-1, 1, 100)])
    A = (Q * lam) @ Q.T
    A = 0.5 * (A + A.T)
    ev, V = engine.syevd(torch.tensor(A, device="cuda"))
    _check(A, ev, V)


def test_syevd_kernel_matrix_pinv_matches_tf_pinv():
    """K_mm of 409 inducing points (SE, l = 0.1 on [0, 1]: numerical rank 29 of 409), the Nystroem case.
    pinv compared through K pinv K = K (both sides' cutoffs drop the same numerically-zero directions).  The bar
    is the reference's own accuracy: an SVD / LAPACK pseudo-inverse of this K leaves |K pinv K - K| = 5.2e-7
    (the kept eigenvalues reach down to the 10 m eps max|lam| cutoff, 1/lam ~ 1e10 amplifies eigenvector
    rounding), so the device's residual must be within 4x of tf_pinv's and agree with it to that level."""
    z = np.linspace(0.0, 1.0, 409).reshape(-1, 1)
    K = o.kernel_matrix(("SE", {}), [0.1], z, z)
    P = engine.pinv_sym(torch.tensor(K, device="cuda")).cpu().numpy()
    ref = o.tf_pinv(K)
    r_ref = float(np.max(np.abs(K @ ref @ K - K)))
    assert np.max(np.abs(K @ P @ K - K)) <= 4 * r_ref
    assert np.max(np.abs(K @ (P - ref) @ K)) <= 4 * r_ref


def test_syevd_indefinite_matrix_n1024():
    """An indefinite K + noise I (noise -0.3), as the PSEUDO / STRICT handlings' fallback sees it, beyond the
    old n <= 2048 cap's scale in miniature."""
    rng = np.random.default_rng(5)
    x = rng.uniform(0, 1, (1024, 1))
    A = o.k_noised(("SE", {}), [0.1], -0.3, x)
    lam, V = engine.syevd(torch.tensor(A, device="cuda"))
    _check(A, lam, V)


@pytest.mark.parametrize("split", [False, True])
def test_syevd_tridiagonalisation_paths_agree(split):
    """The blocked tridiagonalisation in one workgroup per panel (m <= trd_split_m) and with A22 v spread over the
    chip (three launches per column, the large-m path) -- both against numpy at m = 300 (10 panels, a short last
    one)."""
    import gaussianprocessfundamentals_amd._native as nat
    rng = np.random.default_rng(11)
    A = rng.standard_normal((300, 300))
    A = 0.5 * (A + A.T)
    old = nat.tune("trd_split_m", 64 if split else 1024)
    try:
        lam, V = engine.syevd(torch.tensor(A, device="cuda"))
    finally:
        nat.tune("trd_split_m", old)
    _check(A, lam, V)


@pytest.mark.parametrize("m", [4096, 5000, 6144])
def test_syevd_large_indefinite(m):
    """n = 4096 (merged blocks sorted in LDS) and beyond (5000, 6144: the top merges sort in the workspace,
    dc_deflate_kernel's HBM path), the PSEUDO / STRICT fallback's sizes: K - 0.3 I."""
    rng = np.random.default_rng(6)
    x = rng.uniform(0, 1, (m, 1))
    A = o.k_noised(("SE", {}), [0.1], -0.3, x)
    lam, V = engine.syevd(torch.tensor(A, device="cuda"))
    lam, V = lam.cpu().numpy(), V.cpu().numpy()
    ref = np.linalg.eigvalsh(A)
    sc = float(np.max(np.abs(ref)))
    assert np.max(np.abs(np.sort(lam) - ref)) <= 1e-12 * sc
    assert np.max(np.abs(A @ V - V * lam)) <= 1e-11 * sc
    assert np.max(np.abs(V.T @ V - np.eye(m))) <= 1e-11


def _clustered_indefinite(n=16400, nc=8, seed=100):
    """K - 0.3 I of n SE inputs (l = 0.1) in nc clusters 10 apart, the points shuffled: a permuted block-diagonal
    matrix (cross-cluster entries exp(-4050) round to exactly 0) whose spectrum is the union of the blocks' -- so
    numpy checks it block by block.  Returns (x shuffled, A, reference eigenvalues sorted)."""
    rng = np.random.default_rng(seed)
    per = n // nc
    x = np.concatenate([10.0 * c + rng.uniform(0, 1, per) for c in range(nc)])
    ref = np.sort(np.concatenate([np.linalg.eigvalsh(o.k_noised(("SE", {}), [0.1], -0.3, x[c * per:(c + 1) * per]
                                                                   .reshape(-1, 1))) for c in range(nc)]))
    perm = rng.permutation(n)
    xs = x[perm].reshape(-1, 1)
    return xs, ref


def test_syevd_beyond_16384_rows():
    """gpk_syevd above the old 16384 cap: at m = 16400 the top merge's rows no longer fit in LDS and
    dc_gather_kernel stages them in the workspace.  A permuted block-diagonal indefinite K - 0.3 I (16288
    eigenvalues in a cluster at -0.3): eigenvalues vs numpy block by block <= 1e-12 max|lam|, residual
    |A V - V diag(lam)| and orthogonality |V^T V - I| <= 1e-11 (checked on the device by torch's fp64 matmul)."""
    xs, ref = _clustered_indefinite()
    m = xs.shape[0]
    A = torch.tensor(o.k_noised(("SE", {}), [0.1], -0.3, xs), device="cuda")
    lam, V = engine.syevd(A)
    sc = float(np.max(np.abs(ref)))
    err = float(np.max(np.abs(np.sort(lam.cpu().numpy()) - ref)))
    res = float((A @ V - V * lam[None, :]).abs().max())
    orth = float((V.T @ V - torch.eye(m, dtype=torch.float64, device="cuda")).abs().max())
    print("m = %d: eigenvalues max err %.2e (x max|lam| %.3g), residual %.2e, orthogonality %.2e" % (
        m, err / sc, sc, res / sc, orth))
    assert err <= 1e-12 * sc
    assert res <= 1e-11 * sc
    assert orth <= 1e-11
