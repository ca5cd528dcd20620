"""The persistent single-member factorisation (gpk_tune("chain"), chain_kernel in gpk_potrf.hip; on by default for single f64 evaluations since it measured faster,
DESIGN §4) against the launch-per-panel schedule and the oracle (needs the MI355X).

One f64 member without identity / ragged rows runs as ONE launch whose workgroups claim the tasks of
gpk_chain_plan (tests/test_chain_plan.py checks that list on the host).  Its trailing updates apply one
panel at a time where the launch path groups eight, so the two agree to summation order, not bit for
bit: L and the read-outs to ~1e-13 relative here.  Between runs of the chain itself the arithmetic order
is fixed (every tile's updates are serialised by its counter), so repeated runs are bitwise equal.
"""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as o
from tests.helpers import make_kernel

from gaussianprocessfundamentals_amd import engine

pytestmark = pytest.mark.gpu

SE = ("SE", {"ard": False})


def _run(n, m, chain, hyp=0.1, noise=1e-2, seed=3, sync=True):
    x, y = o.make_inputs("C1", n=n, seed=seed)
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    H = torch.tensor([[hyp]], dtype=torch.float64, device=dev)
    NZ = torch.tensor([noise], dtype=torch.float64, device=dev)
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    Xs = torch.linspace(-0.1, 1.1, max(m, 1), dtype=torch.float64, device=dev).reshape(-1, 1) if m else None
    old = engine.nat.tune("chain", chain)
    try:
        f = engine.AugmentedFactorization(n, 1, m, 1)
        f.W.zero_()
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0, Xs, 0)
        if sync:
            torch.cuda.synchronize()
    finally:
        engine.nat.tune("chain", old)
    return f, (x, y)


def _lower(f):
    lay = f.layout
    w = f.w(0).cpu().numpy()
    return np.tril(w[: lay.y_row + 1, : lay.y_row + 1])


@pytest.mark.parametrize("n,m", [(1, 0), (100, 0), (128, 0), (257, 0), (1000, 37), (2048, 0), (3000, 300),
                                 (4096, 0), (4096, 100), (6144, 0)])
def test_chain_matches_the_launch_path(n, m):
    fc, _ = _run(n, m, 1)
    fl, _ = _run(n, m, 0)
    assert int(fc.info.cpu()[0]) == 0 and int(fl.info.cpu()[0]) == 0
    a, b = _lower(fc), _lower(fl)
    scale = np.abs(b).max()
    assert np.abs(a - b).max() <= 1e-12 * scale
    oc, ol = fc.out.cpu().numpy(), fl.out.cpu().numpy()
    assert oc[0] == pytest.approx(ol[0], rel=1e-12)
    if m:
        np.testing.assert_allclose(fc.mu.cpu().numpy(), fl.mu.cpu().numpy(), rtol=0, atol=1e-10)
        np.testing.assert_allclose(fc.var.cpu().numpy(), fl.var.cpu().numpy(), rtol=0, atol=1e-10)


@pytest.mark.parametrize("n", [300, 4096])
def test_chain_nlml_matches_the_oracle(n):
    f, (x, y) = _run(n, 0, 1)
    ref = o.nlml(SE, [0.1], 1e-2, x, y)
    assert float(f.nlml().cpu()[0]) == pytest.approx(ref, rel=1e-9)


def test_chain_runs_as_one_launch():
    engine.nat.timing_reset()
    engine.nat.timing_enable(True)
    try:
        _run(2048, 0, 1)
        t = engine.nat.timing_read()
    finally:
        engine.nat.timing_enable(False)
    assert t["diag"]["launches"] == 0 and t["trsm"]["launches"] == 0
    assert t["update"]["launches"] == 1


def test_chain_is_deterministic():
    a, _ = _run(3000, 64, 1)
    b, _ = _run(3000, 64, 1)
    assert np.array_equal(_lower(a).view(np.uint64), _lower(b).view(np.uint64))


def test_chain_reports_the_first_non_positive_pivot():
    fc, _ = _run(700, 0, 1, hyp=0.3, noise=-0.5)
    fl, _ = _run(700, 0, 0, hyp=0.3, noise=-0.5)
    ic, il = int(fc.info.cpu()[0]), int(fl.info.cpu()[0])
    assert ic > 0 and ic == il
    with pytest.raises(engine.CholeskyError):
        fc.check_info()


def test_chain_on_concurrent_streams():
    ref = {n: _lower(_run(n, 0, 1, hyp=0.05 + 1e-4 * n)[0]) for n in (1500, 2600)}
    streams = [torch.cuda.Stream() for _ in range(2)]
    out = {}
    for s, n in zip(streams, (1500, 2600)):
        with torch.cuda.stream(s):
            out[n] = _run(n, 0, 1, hyp=0.05 + 1e-4 * n, sync=False)[0]
    torch.cuda.synchronize()
    for n in (1500, 2600):
        assert np.array_equal(_lower(out[n]).view(np.uint64), ref[n].view(np.uint64))
