"""Device building blocks of the approximation paths against numpy fp64: the MFMA
GEMM, the Jacobi eigensolver and pseudo-inverse, the SKI weights, the dense-matrix factorisation.

Tolerances: GEMM max-abs <= 1e-13 relative to |A||B|; eigenvalues <= 1e-13 max|lam| (Jacobi is
backward stable; the reference uses Eigen's SVD, same order of error); reconstruction and
orthogonality <= 1e-12; pinv <= 1e-9 relative on a rank-deficient PSD matrix with a clear gap at
the tf.linalg.pinv cutoff; SKI weights bit-exact for D = 1 (the reference's expanded-norm distance
is reproduced op for op); dense factorisation log-det / alpha / inverse <= 1e-10 relative."""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as o

from gaussianprocessfundamentals_amd import engine

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda")


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (5, 7, 3), (64, 64, 16), (130, 97, 257), (300, 200, 1000)])
def test_dgemm_matches_numpy(ta, tb, M, N, K):
    rng = np.random.default_rng(M * 7 + N * 3 + K + ta + 2 * tb)
    A = rng.standard_normal((K, M) if ta else (M, K))
    B = rng.standard_normal((N, K) if tb else (K, N))
    C0 = rng.standard_normal((M, N))
    opA = A.T if ta else A
    opB = B.T if tb else B
    got = engine.dgemm(dev(A), dev(B), bool(ta), bool(tb), 0.5, 2.0, dev(C0)).cpu().numpy()
    ref = 0.5 * opA @ opB + 2.0 * C0
    scale = 0.5 * np.abs(opA) @ np.abs(opB) + 2.0 * np.abs(C0)
    assert np.max(np.abs(got - ref) / scale) < 1e-13


def test_dgemm_batched_and_strided():
    rng = np.random.default_rng(1)
    A = rng.standard_normal((3, 40, 50))
    B = rng.standard_normal((50, 30))          # shared by every member (batch stride 0)
    got = engine.dgemm(dev(A), dev(B)).cpu().numpy()
    assert got.shape == (3, 40, 30)
    assert np.allclose(got, A @ B, rtol=0, atol=1e-12)
    big = dev(rng.standard_normal((70, 90)))[:, :50]   # lda = 90
    ref = big.cpu().numpy() @ B
    assert np.allclose(engine.dgemm(big, dev(B)).cpu().numpy(), ref, rtol=0, atol=1e-12)


@pytest.mark.parametrize("m", [1, 2, 3, 17, 64, 101, 256])
def test_syevj_symmetric(m):
    rng = np.random.default_rng(m)
    G = rng.standard_normal((m, m))
    A = (G + G.T) / 2
    lam, V, sweeps = engine.syevj(dev(A))
    lam, V = lam.cpu().numpy(), V.cpu().numpy()
    ref = np.linalg.eigvalsh(A)
    scale = np.max(np.abs(ref))
    assert np.max(np.abs(np.sort(lam) - ref)) <= 1e-13 * scale * max(1, m) ** 0.5
    assert np.max(np.abs(V @ np.diag(lam) @ V.T - A)) <= 1e-12 * scale
    assert np.max(np.abs(V.T @ V - np.eye(m))) <= 1e-12
    assert 1 <= sweeps <= 30


def test_syevj_kernel_matrix_and_pinv():
    """An SE Gram matrix of clustered points: numerically rank deficient (eigenvalues far below the
    cutoff 10 m eps max|lam| next to O(1) ones) -- the case tf.linalg.pinv exists for."""
    rng = np.random.default_rng(4)
    z = np.sort(rng.uniform(0, 1, (60, 1)), axis=0)
    K = o.kernel_matrix(("SE", {"ard": False}), [0.3], z, z)
    lam, V, _ = engine.syevj(dev(K))
    ref = np.linalg.eigvalsh(K)
    assert np.max(np.abs(np.sort(lam.cpu().numpy()) - ref)) <= 1e-13 * ref[-1]
    U, rank = engine.pinv_factor(lam, V, 0)
    kept = int(rank.cpu()[0])
    cut = 10 * 60 * np.finfo(np.float64).eps * ref[-1]
    assert abs(kept - int(np.sum(np.abs(ref) > cut))) <= 1


def test_pinv_rank_deficient_with_gap():
    """A = Q diag(lam) Q^T with 12 eigenvalues in [0.5, 3] and the rest 1e-20 (far below the cutoff
    10 m eps max|lam|): pinv keeps exactly the 12."""
    rng = np.random.default_rng(6)
    Q, _ = np.linalg.qr(rng.standard_normal((80, 80)))
    lam = np.full(80, 1e-20)
    lam[:12] = rng.uniform(0.5, 3.0, 12)
    A = (Q * lam) @ Q.T
    A = (A + A.T) / 2
    P = engine.pinv_sym(dev(A)).cpu().numpy()
    Pref = o.tf_pinv(A)
    assert np.max(np.abs(P - Pref)) <= 1e-12 * np.max(np.abs(Pref))
    lam_d, V_d, _ = engine.syevj(dev(A))
    _, rank = engine.pinv_factor(lam_d, V_d, 1)
    assert int(rank.cpu()[0]) == 12


def test_pinv_full_rank_equals_inverse():
    rng = np.random.default_rng(5)
    G = rng.standard_normal((50, 50))
    A = G @ G.T + 50 * np.eye(50)
    P = engine.pinv_sym(dev(A)).cpu().numpy()
    assert np.max(np.abs(P - np.linalg.inv(A))) <= 1e-13 * np.max(np.abs(np.linalg.inv(A))) * 50


@pytest.mark.parametrize("n,m", [(50, 5), (1000, 100), (777, 31)])
def test_ski_weights_bitexact_1d(n, m):
    rng = np.random.default_rng(n)
    x = np.sort(rng.uniform(0, 1, (n, 1)), axis=0)
    z = x[o.ski_inducing_indices(n, m)]
    got = engine.ski_weights(dev(x), dev(z)).cpu().numpy()
    ref = o.ski_weight_matrix(x, z)
    assert np.array_equal(got, ref)


def test_ski_weights_ties_and_multid():
    x = np.array([[0.0], [0.5], [1.0], [0.25], [2.0]])
    z = np.array([[0.0], [1.0], [0.5]])
    got = engine.ski_weights(dev(x), dev(z)).cpu().numpy()
    assert np.array_equal(got, o.ski_weight_matrix(x, z))
    rng = np.random.default_rng(8)
    x4 = rng.uniform(0, 1, (300, 4))
    z4 = x4[o.ski_inducing_indices(300, 30)]
    got4 = engine.ski_weights(dev(x4), dev(z4)).cpu().numpy()
    ref4 = o.ski_weight_matrix(x4, z4)
    # D > 1: the reference's matmul reduction order is not reproducible; weights agree to rounding
    # wherever the nearest / second-nearest choice agrees (NaN rows: sqrt of a negative expanded norm)
    ok = ~np.isnan(ref4).any(axis=1)
    assert np.allclose(got4[ok], ref4[ok], rtol=0, atol=1e-12)


@pytest.mark.parametrize("n", [1, 100, 300])
def test_dense_factorization(n):
    rng = np.random.default_rng(n)
    G = rng.standard_normal((n, n + 5))
    A = G @ G.T / n
    noise = 0.1
    y = rng.standard_normal(n)
    f = engine.DenseFactorization(n).run(dev(A), noise, dev(y))
    K = A + noise * np.eye(n)
    assert abs(float(f.logdet()[0]) - np.linalg.slogdet(K)[1]) <= 1e-10 * max(1, abs(np.linalg.slogdet(K)[1]))
    alpha = np.linalg.solve(K, y)
    assert np.allclose(f.alpha().cpu().numpy(), alpha, rtol=1e-10, atol=1e-10 * np.max(np.abs(alpha)))
    fi = engine.DenseFactorization(n, inverse=True).run(dev(A), noise, dev(y))
    assert np.allclose(fi.k_inv().cpu().numpy(), np.linalg.inv(K), rtol=0, atol=1e-10 * np.max(np.abs(np.linalg.inv(K))))


def test_add_diagonal():
    A = dev(np.zeros((5, 7)))
    engine.add_diagonal(A, 2.5)
    ref = np.zeros((5, 7))
    ref[np.arange(5), np.arange(5)] = 2.5
    assert np.array_equal(A.cpu().numpy(), ref)
