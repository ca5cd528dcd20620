"""The workspace-style entry points of SURVEY §8(b) (gpk_workspace_bytes, gpk_nlml_batched,
gpk_potrf_lower fp64 / fp32, gpk_trsv_lower, gpk_posterior) called through ctypes against numpy / the oracle.
Tolerances: NLL rel <= 1e-10; L max-abs <= 1e-12 relative to max|L| (fp32: 2e-5), log-det rel <= 1e-12 (fp32:
1e-5); the upper triangle untouched; triangular solves: normwise backward error <= 8 n eps; posterior mu / Sigma
max-abs <= 1e-10 against the oracle (noise 1e-2)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import gp_oracle as o

from gaussianprocessfundamentals_amd import _native as nat
from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk

pytestmark = pytest.mark.gpu

WS_NLML, WS_POTRF, WS_TRSV, WS_POSTERIOR = 0, 1, 2, 3


def P(t):
    return ctypes.c_void_p(t.data_ptr())


@pytest.mark.parametrize("n,batch", [(1, 1), (300, 3), (1000, 5)])
def test_nlml_batched_matches_oracle(n, batch):
    L = nat.lib()
    rng = np.random.default_rng(n)
    x = np.sort(rng.uniform(0, 1, (n, 1)), axis=0)
    y = np.sin(5 * x[:, 0]) + 0.1 * rng.standard_normal(n)
    ls = np.linspace(0.05, 0.3, batch)
    noise = np.linspace(1e-2, 5e-2, batch)
    kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
    X = torch.tensor(x, device="cuda")
    Y = torch.tensor(y, device="cuda")
    H = torch.tensor(ls.reshape(-1, 1), device="cuda")
    NZ = torch.tensor(noise, device="cuda")
    wb = int(L.gpk_workspace_bytes(WS_NLML, nat.GPK_F64, n, 0, batch))
    work = torch.empty(wb // 8 + 1, dtype=torch.float64, device="cuda")
    out = torch.empty(batch, dtype=torch.float64, device="cuda")
    info = torch.empty(batch, dtype=torch.int32, device="cuda")
    nat.check(L.gpk_nlml_batched(ctypes.byref(kd), batch, P(H), P(NZ), nat.GPK_F64, P(X), P(Y), n, 1, P(work), wb,
                                 P(out), P(info), nat.stream_handle()), "gpk_nlml_batched")
    got = out.cpu().numpy()
    assert (info.cpu().numpy() == 0).all()
    for b in range(batch):
        ref = o.nlml(("SE", {"ard": False}), [ls[b]], noise[b], x, y)
        assert abs(got[b] - ref) <= 1e-10 * abs(ref), (b, got[b], ref)
    assert nat.lib().gpk_nlml_batched(ctypes.byref(kd), batch, P(H), P(NZ), nat.GPK_F64, P(X), P(Y), n, 1, P(work),
                                      wb - 1, P(out), P(info), nat.stream_handle()) < 0


@pytest.mark.parametrize("n,pad", [(1, 0), (130, 3), (700, 0), (1100, 17)])
def test_potrf_lower_matches_numpy(n, pad):
    L = nat.lib()
    rng = np.random.default_rng(n + pad)
    G = rng.standard_normal((n, n + 4))
    A = G @ G.T / n + 0.5 * np.eye(n)
    lda = n + pad
    buf = np.full((n, lda), 7.0)
    buf[:, :n] = np.tril(A) + np.triu(np.full((n, n), 3.0), 1)   # upper triangle: marker values
    Ad = torch.tensor(buf, device="cuda")
    wb = int(L.gpk_workspace_bytes(WS_POTRF, nat.GPK_F64, n, 0, 1))
    work = torch.empty(wb // 8 + 1, dtype=torch.float64, device="cuda")
    info = torch.full((1,), -5, dtype=torch.int32, device="cuda")
    logdet = torch.empty(1, dtype=torch.float64, device="cuda")
    nat.check(L.gpk_potrf_lower(nat.GPK_F64, P(Ad), n, lda, P(work), wb, P(info), P(logdet), nat.stream_handle()),
              "gpk_potrf_lower")
    got = Ad.cpu().numpy()
    ref = np.linalg.cholesky(A)
    assert int(info.cpu()[0]) == 0
    assert np.max(np.abs(np.tril(got[:, :n]) - ref)) <= 1e-12 * np.max(np.abs(ref))
    assert np.array_equal(np.triu(got[:, :n], 1), np.triu(np.full((n, n), 3.0), 1))
    assert np.array_equal(got[:, n:], np.full((n, pad), 7.0))
    ld_ref = 2 * np.sum(np.log(np.diag(ref)))
    assert abs(float(logdet.cpu()[0]) - ld_ref) <= 1e-12 * max(1.0, abs(ld_ref))


def test_potrf_lower_reports_not_positive_definite():
    L = nat.lib()
    n = 200
    A = np.eye(n)
    A[150, 150] = -1.0
    Ad = torch.tensor(A, device="cuda")
    wb = int(L.gpk_workspace_bytes(WS_POTRF, nat.GPK_F64, n, 0, 1))
    work = torch.empty(wb // 8 + 1, dtype=torch.float64, device="cuda")
    info = torch.zeros(1, dtype=torch.int32, device="cuda")
    nat.check(L.gpk_potrf_lower(nat.GPK_F64, P(Ad), n, n, P(work), wb, P(info), None, nat.stream_handle()),
              "gpk_potrf_lower")
    assert int(info.cpu()[0]) == 151
    assert L.gpk_potrf_lower(7, P(Ad), n, n, P(work), wb, P(info), None, nat.stream_handle()) < 0


@pytest.mark.parametrize("n,pad", [(1, 0), (130, 3), (1100, 17)])
def test_potrf_lower_fp32_matches_numpy(n, pad):
    """dtype GPK_F32: the f32 MFMA factorisation of a float A (C3's precision), in place."""
    L = nat.lib()
    rng = np.random.default_rng(7 + n)
    G = rng.standard_normal((n, n + 4))
    A = G @ G.T / n + 0.5 * np.eye(n)
    lda = n + pad
    buf = np.full((n, lda), 7.0, dtype=np.float32)
    buf[:, :n] = np.tril(A) + np.triu(np.full((n, n), 3.0), 1)
    Ad = torch.tensor(buf, device="cuda")
    wb = int(L.gpk_workspace_bytes(WS_POTRF, nat.GPK_F32, n, 0, 1))
    assert 0 < wb < int(L.gpk_workspace_bytes(WS_POTRF, nat.GPK_F64, n, 0, 1)) or n == 1
    work = torch.empty(wb // 4 + 1, dtype=torch.float32, device="cuda")
    info = torch.full((1,), -5, dtype=torch.int32, device="cuda")
    logdet = torch.empty(1, dtype=torch.float64, device="cuda")
    nat.check(L.gpk_potrf_lower(nat.GPK_F32, P(Ad), n, lda, P(work), wb, P(info), P(logdet), nat.stream_handle()),
              "gpk_potrf_lower f32")
    got = Ad.cpu().numpy().astype(np.float64)
    ref = np.linalg.cholesky(A.astype(np.float32).astype(np.float64))
    assert int(info.cpu()[0]) == 0
    assert np.max(np.abs(np.tril(got[:, :n]) - ref)) <= 2e-5 * np.max(np.abs(ref))
    assert np.array_equal(np.triu(got[:, :n], 1), np.triu(np.full((n, n), 3.0), 1))
    assert np.array_equal(got[:, n:], np.full((n, pad), 7.0))
    ld_ref = 2 * np.sum(np.log(np.diag(ref)))
    assert abs(float(logdet.cpu()[0]) - ld_ref) <= 1e-5 * max(1.0, abs(ld_ref))


def _chol(n, seed):
    rng = np.random.default_rng(seed)
    G = rng.standard_normal((n, n + 4))
    return np.linalg.cholesky(G @ G.T / n + 0.5 * np.eye(n))


@pytest.mark.parametrize("n,pad", [(1, 0), (128, 0), (130, 5), (700, 0), (1100, 17)])
@pytest.mark.parametrize("trans", [0, 1])
def test_trsv_lower_on_a_caller_factor(n, pad, trans):
    """gpk_trsv_lower on an arbitrary lower-triangular L (ldl > n, junk in the upper triangle and the pad):
    the sketch's gpk_trsv_lower.  Normwise backward error |b - op(L) x| / (|op(L)| |x|) <= 8 n eps."""
    L = nat.lib()
    Lr = _chol(n, n + trans)
    buf = np.full((n, n + pad), np.nan)
    buf[:, :n] = Lr + np.triu(np.full((n, n), 1e30), 1)
    b = np.random.default_rng(3).standard_normal(n)
    Ld = torch.tensor(buf, device="cuda")
    x = torch.tensor(b, device="cuda")
    wb = int(L.gpk_workspace_bytes(WS_TRSV, nat.GPK_F64, n, 0, 1))
    work = torch.empty(wb // 8 + 1, dtype=torch.float64, device="cuda")
    nat.check(L.gpk_trsv_lower(nat.GPK_F64, trans, P(Ld), n, n + pad, P(x), P(work), wb, nat.stream_handle()),
              "gpk_trsv_lower")
    xs = x.cpu().numpy()
    op = Lr if trans == 0 else Lr.T
    err = np.max(np.abs(b - op @ xs)) / (np.max(np.abs(op).sum(axis=1)) * np.max(np.abs(xs)))
    assert err <= 8 * n * np.finfo(np.float64).eps, err
    assert L.gpk_trsv_lower(nat.GPK_F64, trans, P(Ld), n, n + pad, P(x), P(work), wb - 256, nat.stream_handle()) < 0


@pytest.mark.parametrize("n,m", [(130, 1), (700, 37), (1100, 300)])
def test_posterior_from_a_caller_factor(n, m):
    """gpk_posterior(L, alpha, X, Xs): mu = K_s^T alpha, diag Sigma (var_mode 0) and full Sigma (var_mode 1)
    against the oracle's posterior (S/Auxiliary.py:57-103) on the same inputs."""
    L = nat.lib()
    rng = np.random.default_rng(n + m)
    x = np.sort(rng.uniform(0, 1, (n, 1)), axis=0)
    y = np.sin(5 * x[:, 0]) + 0.1 * rng.standard_normal(n)
    xs = rng.uniform(-0.1, 1.1, (m, 1))
    ls, noise = 0.15, 1e-2
    Kn = o.k_noised(("SE", {}), [ls], noise, x)
    Lr = np.linalg.cholesky(Kn)
    alpha = np.linalg.solve(Kn, y)
    kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
    hyp = torch.tensor([ls], dtype=torch.float64, device="cuda")
    Ld = torch.tensor(Lr, device="cuda")
    ad = torch.tensor(alpha, device="cuda")
    X = torch.tensor(x, device="cuda")
    Xs = torch.tensor(xs, device="cuda")
    wb = int(L.gpk_workspace_bytes(WS_POSTERIOR, nat.GPK_F64, n, m, 1))
    work = torch.empty(wb // 8 + 1, dtype=torch.float64, device="cuda")
    mu = torch.empty(m, dtype=torch.float64, device="cuda")
    var = torch.empty(m, dtype=torch.float64, device="cuda")
    cov = torch.empty((m, m + 3), dtype=torch.float64, device="cuda")
    st = nat.stream_handle()
    nat.check(L.gpk_posterior(ctypes.byref(kd), P(hyp), nat.GPK_F64, P(Ld), n, P(ad), P(X), n, P(Xs), m, 1, 0,
                              P(mu), P(var), 0, P(work), wb, st), "gpk_posterior diag")
    nat.check(L.gpk_posterior(ctypes.byref(kd), P(hyp), nat.GPK_F64, P(Ld), n, P(ad), P(X), n, P(Xs), m, 1, 1,
                              None, P(cov), m + 3, P(work), wb, st), "gpk_posterior full")
    mu_ref, cov_ref = o.posterior(("SE", {}), [ls], noise, x, y, xs)
    np.testing.assert_allclose(mu.cpu().numpy(), mu_ref, rtol=0, atol=1e-10)
    np.testing.assert_allclose(var.cpu().numpy(), np.diag(cov_ref), rtol=0, atol=1e-10)
    np.testing.assert_allclose(cov.cpu().numpy()[:, :m], cov_ref, rtol=0, atol=1e-10)
