"""The workspace-style entry points of SURVEY §8(b) (gpk_workspace_bytes, gpk_nlml_batched,
gpk_potrf_lower) called through ctypes against the oracle.  Tolerances: NLL rel <= 1e-10;
L max-abs <= 1e-12 relative to max|L|, log-det rel <= 1e-12; the upper triangle untouched."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import gp_oracle as o

from gaussianprocessfundamentals_amd import _native as nat
from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk

pytestmark = pytest.mark.gpu

WS_NLML, WS_POTRF = 0, 1


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
    assert L.gpk_potrf_lower(nat.GPK_F32, P(Ad), n, n, P(work), wb, P(info), None, nat.stream_handle()) < 0
