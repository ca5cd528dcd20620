"""The persistent factorisation in f32 (gpk_tune("chain_f32"), chain_kernel<float> in gpk_potrf.hip) against the
f32 launch path and the fp64 oracle (needs the MI355X).

chain_kernel<float> runs the f32 tile tasks -- panel solves and slice updates on the f32 MFMA (slab_gemm32), the
deferred 128 x 128 tile updates (blk_tile<float>) -- and the diagonal blocks through the launch path's own body
(diag2_body<float>: f64 arithmetic in LDS, f32 in HBM).  Every element takes the launch path's MFMA k-steps in its
order, C first (gemm_kernel<float> accumulates onto C one k-step after another whatever the panel grouping), so the
persistent launch reproduces the f32 launch path bit for bit at every size and plan variant.  Against the fp64
oracle: rel <= 1e-3 on -LML (SURVEY §8d's fp32 bar), C3's MAT52-ARD included.
"""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as o
from tests.helpers import make_kernel

from gaussianprocessfundamentals_amd import engine

pytestmark = pytest.mark.gpu

SE = ("SE", {"ard": False})
MAT52 = ("MAT52", {"ard": True, "standard": True})


def _run(n, m, chain, cfg="C1", tree=SE, d=1, hyp=(0.1,), noise=1e-1, batch=1, seed=3, **knobs):
    x, y = o.make_inputs(cfg, n=n, seed=seed)
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(tree, d), d)
    rows = [[h * (1.0 + 0.05 * b) for h in hyp] for b in range(batch)]
    H = torch.tensor(rows, dtype=torch.float64, device=dev)
    NZ = torch.tensor([noise], dtype=torch.float64, device=dev)
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, d).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    Xs = torch.linspace(-0.1, 1.1, max(m, 1) * d, dtype=torch.float64, device=dev).reshape(-1, d) if m else None
    with engine.nat.thread_tune(chain=2 if chain else 0, chain_f32=1, chain_max_batch=8, **knobs):
        before = engine.nat.chain_stats()["launches"]
        f = engine.AugmentedFactorization(n, d, m, batch, torch.float32)
        f.W.zero_()
        f.run(kd, H, H.shape[1], NZ, 0, X, 0, Y, 0, Xs, 0)
        torch.cuda.synchronize()
        launched = engine.nat.chain_stats()["launches"] - before
    assert (launched > 0) == bool(chain), "persistent launches: %d" % launched
    return f, (x, y)


def _lower(f, b=0):
    lay = f.layout
    w = f.w(b).cpu().numpy()
    return np.tril(w[: lay.y_row + 1, : lay.y_row + 1])


def _bitwise(fc, fl, batch=1):
    for b in range(batch):
        a, c = _lower(fc, b), _lower(fl, b)
        diff = int(np.count_nonzero(a.view(np.uint32) != c.view(np.uint32)))
        assert diff == 0, "member %d: %d of %d lower-triangle words differ" % (b, diff, a.size)
    oc, ol = fc.out.cpu().numpy(), fl.out.cpu().numpy()
    assert np.array_equal(oc.view(np.uint64), ol.view(np.uint64)), (oc, ol)


@pytest.mark.parametrize("n,m", [(1, 0), (257, 0), (1000, 37), (3000, 300), (4096, 0), (8192, 0), (12288, 0)])
def test_f32_chain_bitwise_vs_f32_launch_path(n, m):
    fc, _ = _run(n, m, 1)
    fl, _ = _run(n, m, 0)
    assert int(fc.info.cpu()[0]) == 0
    _bitwise(fc, fl)


@pytest.mark.parametrize("group", [1, 4, 8, 16])
@pytest.mark.parametrize("n,m", [(2100, 40), (5000, 0)])
def test_f32_chain_plan_variants_bitwise(n, m, group):
    """Deferred-update depth chain_group (tile updates over 1 .. 16 panels in one task) and chain_uq (ignored in f32:
    one slice-update task per slice) -- the same bits as the launch path in every variant."""
    fc, _ = _run(n, m, 1, chain_group=group, chain_uq=1)
    fl, _ = _run(n, m, 0)
    _bitwise(fc, fl)


def test_f32_chain_two_lists_bitwise():
    fc, _ = _run(5000, 0, 1, chain_xcd=1)
    fl, _ = _run(5000, 0, 0)
    _bitwise(fc, fl)


@pytest.mark.parametrize("n,batch", [(1000, 2), (2048, 3)])
def test_f32_chain_batched_members_bitwise(n, batch):
    fc, _ = _run(n, 0, 1, batch=batch)
    fl, _ = _run(n, 0, 0, batch=batch)
    _bitwise(fc, fl, batch)


@pytest.mark.parametrize("n", [300, 4096])
def test_f32_chain_nlml_matches_the_fp64_oracle(n):
    f, (x, y) = _run(n, 0, 1)
    ref = o.nlml(SE, [0.1], 1e-1, x, y)
    got = float(f.nlml().cpu()[0])
    print("f32 chain N=%d: rel %.3e" % (n, abs(got - ref) / abs(ref)))
    assert got == pytest.approx(ref, rel=1e-3)


def test_f32_chain_c3_mat52_ard_bitwise_and_oracle():
    """C3's factorisation (MAT52-ARD, D = 4, N = 8192, noise 0.1) through the persistent f32 launch: bitwise the f32
    launch path, rel <= 1e-3 against the fp64 oracle."""
    ls = (0.25, 0.5, 0.75, 1.0)
    fc, (x, y) = _run(8192, 0, 1, cfg="C3", tree=MAT52, d=4, hyp=ls)
    fl, _ = _run(8192, 0, 0, cfg="C3", tree=MAT52, d=4, hyp=ls)
    _bitwise(fc, fl)
    ref = o.nlml(MAT52, [list(ls)], 0.1, x, y)
    got = float(fc.nlml().cpu()[0])
    print("C3 f32 chain: nlml %.6f oracle %.6f rel %.3e" % (got, ref, abs(got - ref) / abs(ref)))
    assert got == pytest.approx(ref, rel=1e-3)


def test_f32_chain_side_by_side_on_cu_shares():
    """Four f32 persistent launches on four streams, each with a quarter of the CUs (the bench's C3 schedule): every
    one bitwise the launch path's result."""
    dev = engine.device()
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    x, y = o.make_inputs("C1", n=4096, seed=3)
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    NZ = torch.tensor([1e-1], dtype=torch.float64, device=dev)
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    hs = [torch.tensor([[0.1 * (1 + 0.03 * i)]], dtype=torch.float64, device=dev) for i in range(4)]
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    facts = [engine.AugmentedFactorization(4096, 1, 0, 1, torch.float32) for _ in range(4)]
    with engine.nat.thread_tune(chain=2, chain_f32=1, chain_grid=max(1, ncu // 4)):
        for f, h, s in zip(facts, hs, streams):
            with torch.cuda.stream(s):
                f.run(kd, h, 1, NZ, 0, X, 0, Y, 0, None, 0)
    torch.cuda.synchronize()
    for f, h in zip(facts, hs):
        with engine.nat.thread_tune(chain=0):
            fl = engine.AugmentedFactorization(4096, 1, 0, 1, torch.float32)
            fl.run(kd, h, 1, NZ, 0, X, 0, Y, 0, None, 0)
            torch.cuda.synchronize()
        _bitwise(f, fl)


def test_f32_chain_timeout_falls_back_to_the_launch_path():
    """A timed-out wait of the f32 persistent launch (gpk_tune "chain_force_timeout") is recovered on the launch path
    at the first read of the results: the launch path's bits."""
    engine.nat.tune("chain_force_timeout", 1)
    try:
        fc, _ = _run(2048, 0, 1)
    finally:
        engine.nat.tune("chain_force_timeout", 0)
    fl, _ = _run(2048, 0, 0)
    assert float(fc.nlml().cpu()[0]) == float(fl.nlml().cpu()[0])
    _bitwise(fc, fl)


def test_f32_chain_off_keeps_the_launch_path():
    x, y = o.make_inputs("C1", n=1024, seed=3)
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    H = torch.tensor([[0.1]], dtype=torch.float64, device=dev)
    NZ = torch.tensor([1e-1], dtype=torch.float64, device=dev)
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    with engine.nat.thread_tune(chain=2, chain_f32=0):
        before = engine.nat.chain_stats()["launches"]
        f = engine.AugmentedFactorization(1024, 1, 0, 1, torch.float32)
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0, None, 0)
        torch.cuda.synchronize()
        assert engine.nat.chain_stats()["launches"] == before
