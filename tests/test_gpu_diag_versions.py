"""The look-ahead diagonal-block kernel (diag_version 2, the default) against the phase-serial one
(diag_version 1): same tile algebra, same MFMA k-order, so the factor, the inverted diagonal blocks,
info and -LML must agree BIT FOR BIT, for fp64 and fp32, uniform and ragged ends, PD and not PD.
Both are checked against the oracle by the parity suite; this pins the schedule change alone."""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as o

from gaussianprocessfundamentals_amd import _native as nat
from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk

pytestmark = pytest.mark.gpu


def _factor(version, n, batch, dtype, noise, m=0):
    old = nat.tune("diag_version", version)
    try:
        dev = engine.device()
        x, y = o.make_inputs("C1", n=n, seed=4)
        f = engine.AugmentedFactorization(n, 1, m, batch, dtype)
        kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
        H = torch.linspace(0.05, 0.3, batch, dtype=torch.float64, device=dev).reshape(batch, 1).contiguous()
        X = torch.as_tensor(x, device=dev).contiguous()
        Y = torch.as_tensor(y, device=dev).reshape(1, -1).contiguous()
        NZ = torch.tensor([noise], dtype=torch.float64, device=dev)
        Xs = X[:m].contiguous() if m else None
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0, Xs=Xs, xs_bstride=0)
        torch.cuda.synchronize()
        e = f.layout.y_row + 1
        # the lower triangle of every member up to the y row (the rest is never written: torch.empty)
        Wl = torch.stack([torch.tril(f.w(i)[:e, :e]) for i in range(batch)])
        extra = (f.mu.clone(), f.var.clone()) if m else ()
        return (Wl, f.Winv.clone(), f.info.clone(), f.out.clone()) + extra
    finally:
        nat.tune("diag_version", old)


@pytest.mark.parametrize("n,batch,dtype,m", [(128, 1, torch.float64, 0), (1000, 3, torch.float64, 0),
                                             (1000, 2, torch.float64, 37), (700, 2, torch.float32, 0),
                                             (4096, 1, torch.float64, 0)])
def test_versions_bitwise_identical(n, batch, dtype, m):
    noise = 1e-2 if dtype == torch.float64 else 1e-1
    a = _factor(1, n, batch, dtype, noise, m)
    b = _factor(2, n, batch, dtype, noise, m)
    assert len(a) == len(b)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
    assert int(a[2].abs().sum()) == 0


def test_versions_agree_on_not_positive_definite():
    a = _factor(1, 500, 2, torch.float64, -0.5)
    b = _factor(2, 500, 2, torch.float64, -0.5)
    assert torch.equal(a[2], b[2]) and bool((a[2] > 0).all())
    assert np.all(np.isinf(b[3].view(2, 4)[:, 0].cpu().numpy()))


def _nlml_with(knob, value, n, batch, m=0):
    old = nat.tune(knob, value)
    try:
        return _factor(2, n, batch, torch.float64, 1e-2, m)
    finally:
        nat.tune(knob, old)


@pytest.mark.parametrize("n,batch,m", [(1100, 1, 0), (1100, 3, 21), (3000, 2, 0)])
def test_in_group_schedules_agree(n, batch, m):
    """Right-looking (latency), left-looking and two-level left-looking (throughput) in-group updates:
    the same factorisation up to summation order -- -LML rel <= 1e-12, the factor's lower triangle max-abs <= 1e-12 max|L|."""
    a = _nlml_with("ingroup", 1, n, batch, m)
    for mode in (2, 3):  # right-looking, two-level left-looking
        b = _nlml_with("ingroup", mode, n, batch, m)
        la, lb = a[0], b[0]
        assert float((la - lb).abs().max()) <= 1e-12 * float(la.abs().max())
        na, nb_ = a[3].view(batch, 4)[:, 0], b[3].view(batch, 4)[:, 0]
        assert float(((na - nb_).abs() / na.abs()).max()) <= 1e-12
        if m:
            assert float((a[4] - b[4]).abs().max()) <= 1e-10 and float((a[5] - b[5]).abs().max()) <= 1e-10
