"""Panel solve fused into the diagonal-block launch (gpk_tune("fuse_trsm"), f64 small grids) vs the
separate gemm<TRSM> launch (needs the MI355X).

The fused kernel solves each 64-row tile against L^-1 in LDS with gemm<TRSM>'s MFMA k-order, so the
whole augmented matrix -- L, z, V^T, the Schur corner, K^-1 on the identity-augmented path -- and the
read-outs must agree BIT FOR BIT with the unfused schedule, on plain, test-row, ragged, identity-augmented
and batched layouts, and under every in-group schedule.  The oracle comparison itself is in
tests/test_gpu_parity.py, which now runs the fused path by default at these sizes."""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as o
from tests.helpers import hyp_list, make_kernel

from gaussianprocessfundamentals_amd import engine
from tests.test_gpu_segmented import ragged_members

pytestmark = pytest.mark.gpu

SE = ("SE", {"ard": False})
MAT52 = ("MAT52", {})


def _both(fn):
    """fn() under fuse_trsm 0 and 1 -> (unfused, fused) results as host numpy arrays."""
    out = {}
    for fuse in (0, 1):
        old = engine.nat.tune("fuse_trsm", fuse)
        try:
            res = fn()
            torch.cuda.synchronize()
            out[fuse] = [np.array(r.detach().cpu().numpy(), copy=True) for r in res]
        finally:
            engine.nat.tune("fuse_trsm", old)
    return out[0], out[1]


def _assert_bitwise(a, b):
    for u, v in zip(a, b):
        assert u.shape == v.shape
        assert np.array_equal(u.view(np.uint64) if u.dtype == np.float64 else u,
                              v.view(np.uint64) if v.dtype == np.float64 else v)


def _plain(n, m, batch, tree=SE, hyps=None, seed=3):
    x, y = o.make_inputs("C1", n=n, seed=seed)
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(tree, 1), 1)
    hyps = hyps or [[0.1]] * batch
    H = torch.tensor(hyps, dtype=torch.float64, device=dev)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    Xs = torch.linspace(-0.1, 1.1, max(m, 1), dtype=torch.float64, device=dev).reshape(-1, 1) if m else None

    def run():
        f = engine.AugmentedFactorization(n, 1, m, batch)
        f.W.zero_()  # upper tiles are never written: compare defined memory only
        f.run(kd, H, H.shape[1], NZ, 0, X, 0, Y, 0, Xs, 0)
        return [f.W, f.out] + ([f.mu, f.var] if m else [])
    return run


@pytest.mark.parametrize("n,m,batch", [(1300, 0, 1), (1300, 200, 1), (4096, 0, 1), (777, 64, 3), (257, 0, 1)])
def test_fused_panel_solve_is_bitwise_the_separate_launch(n, m, batch):
    hyps = [[0.05 + 0.03 * b] for b in range(batch)]
    a, b = _both(_plain(n, m, batch, hyps=hyps))
    _assert_bitwise(a, b)


@pytest.mark.parametrize("ingroup", [1, 2, 3])
def test_fused_panel_solve_every_in_group_schedule(ingroup):
    old = engine.nat.tune("ingroup", ingroup)
    try:
        a, b = _both(_plain(2100, 100, 2, tree=MAT52, hyps=[[0.2], [0.4]]))
    finally:
        engine.nat.tune("ingroup", old)
    _assert_bitwise(a, b)


def test_fused_panel_solve_identity_augmented():
    """The gradient / K^-1 path: identity extra rows, whose zero band the fused tiles skip."""
    x, y = o.make_inputs("C1", n=1100, seed=21)
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    H = torch.tensor([[0.07]], dtype=torch.float64, device=dev)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)

    def run():
        f = engine.InverseFactorization(len(x), 1, 1)
        f.W.zero_()
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        return [f.W, f.out, f.gradient()]
    a, b = _both(run)
    _assert_bitwise(a, b)


def test_fused_panel_solve_ragged():
    """Ragged members: per-member padding / unused test rows are skipped as zero rows."""
    sizes, tsz = [300, 1000, 129, 1], [10, 0, 33, 5]
    members, _ = ragged_members([(SE, [0.1]), (MAT52, [0.3])], sizes, tsz)

    def run():
        f = engine.RaggedFactorization(sizes, 1, tsz)
        f.W.zero_()
        f.run(members, 1e-2)
        return [f.W, f.out, f.mu, f.var]
    a, b = _both(run)
    _assert_bitwise(a, b)


def test_fused_panel_solve_not_positive_definite_reports_info():
    """A K that is not PD: the fused launch reports the same first bad pivot (info) as the separate one."""
    x = np.linspace(0, 1, 600).reshape(-1, 1)
    x[300] = x[299]  # duplicate point, noise 0: singular K
    y = np.sin(6 * x[:, 0])
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    X = torch.tensor(x, dtype=torch.float64, device=dev).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    H = torch.tensor([[0.3]], dtype=torch.float64, device=dev)
    NZ = torch.tensor([0.0], dtype=torch.float64, device=dev)
    infos = {}
    for fuse in (0, 1):
        old = engine.nat.tune("fuse_trsm", fuse)
        try:
            f = engine.AugmentedFactorization(600, 1, 0, 1).run(kd, H, 1, NZ, 0, X, 0, Y, 0)
            infos[fuse] = int(f.info[0])
        finally:
            engine.nat.tune("fuse_trsm", old)
    assert infos[0] > 0
    assert infos[0] == infos[1]


def test_fused_panel_solve_beside_a_busy_stream():
    """Workgroups of one fused launch may start far apart when another stream holds the CUs: the block
    must not be overwritten by L while a late workgroup still loads it (the writer is the last
    workgroup to load, DiagArgs::ctr).  Small factorisations run on the caller's stream while a large
    batched one fills the chip from a side stream; every result must equal the quiet run bit for bit."""
    dev = engine.device()
    big_x, big_y = o.make_inputs("C1", n=6000, seed=5)
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    BX = torch.tensor(big_x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    BY = torch.tensor(big_y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    BH = torch.tensor([[0.05], [0.1], [0.2], [0.3]], dtype=torch.float64, device=dev)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    small = _plain(700, 0, 5, hyps=[[c] for c in np.geomspace(0.2, 0.5, 5)], seed=6)
    quiet = [np.array(r.cpu().numpy(), copy=True) for r in small()]
    side = torch.cuda.Stream(dev)
    big = engine.AugmentedFactorization(6000, 1, 0, 4)
    for _ in range(3):
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            big.run(kd, BH, 1, NZ, 0, BX, 0, BY, 0)
        for _ in range(4):
            res = [np.array(r.cpu().numpy(), copy=True) for r in small()]
            _assert_bitwise(quiet, res)
        torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize()


def test_fused_panel_solve_beside_the_lookahead_bulk_stream():
    """fuse_trsm = 2 also fuses with the panel look-ahead on: the fused launches then run beside the bulk
    trailing updates of the CU-masked stream (late-starting workgroups, the ticket counter under real
    concurrency) and must still give the separate launch's bits."""
    old_la = engine.nat.tune("lookahead", 1)
    try:
        out = {}
        for fuse in (0, 2):
            old = engine.nat.tune("fuse_trsm", fuse)
            try:
                res = _plain(6300, 0, 1, hyps=[[0.07]], seed=9)()
                torch.cuda.synchronize()
                out[fuse] = [np.array(r.cpu().numpy(), copy=True) for r in res]
            finally:
                engine.nat.tune("fuse_trsm", old)
        _assert_bitwise(out[0], out[2])
    finally:
        engine.nat.tune("lookahead", old_la)
