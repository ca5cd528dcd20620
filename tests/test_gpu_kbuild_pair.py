"""K build of two-leaf SE + periodic trees on f64 MFMA (gpk_assemble.hip: pair_feat_kernel + pair_mfma_tile), the
C5 kernel (BASELINE configs[4]: SE-ARD + PER, N = 16384, D = 8).  Needs the MI355X.

The tile evaluates |u_i - u_j|^2 as |u_i|^2 + |u_j|^2 - 2 u_i.u_j and sum_k sin^2(pi (x_ik - x_jk) / p) as
D / 2 - (sum_k C_ik C_jk + S_ik S_jk) / 2 (C = cos(2 pi x / p), S = sin(2 pi x / p)) on the matrix cores.  The
reference evaluates the differences directly (KernelBasics/BaseKernels.py:277-294, :440-457), so the MFMA forms
are admitted per tile only while the cancellation they suffer is bounded: (max |u_i|^2 + max |u_j|^2) / l^2 <=
512 and D / l_per^2 <= 128 keep the exponents' absolute error below ~1e-12 (then the entries' relative error is
too); tiles outside the bounds (far-from-origin points, |x / p| > 4) take the direct loop.

  * the oracle kernel matrix (oracle/gp_oracle.py:kernel_matrix) on the training block, the test rows and
    the y row of the augmented matrix: rel 1e-12 of the largest entry (the bound above, with margin);
  * the per-point features of the pre-pass (gpk_tune("asm_feat", 1), the default) write the same bits as
    the per-tile staging (asm_feat 0), with test rows, batches, SE first or second, ADD and MUL;
  * inputs that put some tiles outside the bounds: the mixture still matches the oracle.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import gp_oracle as o
from tests.helpers import make_kernel

from gaussianprocessfundamentals_amd import _native as nat
from gaussianprocessfundamentals_amd import engine

pytestmark = pytest.mark.gpu

F64 = torch.float64


def _tree(op, se_first, ard):
    se = ("SE", {"ard": True}) if ard else ("SE", {})
    per = ("PER", {"standard": True})
    return (op, [se, per] if se_first else [per, se])


def _hyp(d, se_first, ard, rng):
    se = [list(0.5 + 0.5 * rng.uniform(0, 1, d))] if ard else [0.7]
    per = [0.9, 1.3]
    return se + per if se_first else per + se


def _flat(hyp):
    return np.concatenate([np.asarray(h, dtype=np.float64).reshape(-1) for h in hyp])


def _assemble(tree, hyp, d, x, xs, y, noise, batch=1):
    """Augmented matrix of each member (the same inputs, the member's hyperparameters scaled by 1 + 0.1 b)."""
    k = make_kernel(tree, d)
    kd = engine.kernel_descriptor(k, d)
    dev = engine.device()
    n, m = x.shape[0], (0 if xs is None else xs.shape[0])
    H = torch.stack([torch.as_tensor(_flat(hyp) * (1 + 0.1 * b)) for b in range(batch)]).to(dev).contiguous()
    assert H.shape[1] == kd.n_hyp
    f = engine.AugmentedFactorization(n, d, m, batch)
    f.W.zero_()
    L = nat.lib()
    X = torch.as_tensor(x, device=dev).contiguous()
    Xs = torch.as_tensor(xs, device=dev).contiguous() if m else None
    Y = torch.as_tensor(y, device=dev).reshape(1, -1).contiguous()
    NZ = torch.tensor([noise], dtype=F64, device=dev)
    nat.check(L.gpk_assemble(ctypes.byref(kd), ctypes.byref(f.layout), nat.ptr(H), kd.n_hyp, nat.ptr(NZ), 0,
                             nat.ptr(X), 0, nat.ptr(Xs) if Xs is not None else None, 0, None, 0,
                             nat.ptr(Y), 0, nat.ptr(f.W), nat.stream_handle(f.W.device)), "gpk_assemble")
    torch.cuda.synchronize()
    return f, [f.w(b).cpu().numpy().copy() for b in range(batch)]


def _check_against_oracle(tree, hyp, d, x, xs, y, noise, W, lay):
    n, m = x.shape[0], xs.shape[0]
    K = o.kernel_matrix(tree, hyp, x, x) + noise * np.eye(n)
    Ks = o.kernel_matrix(tree, hyp, xs, x)
    scale = np.abs(K).max()
    tr = np.tril(W[:n, :n])
    err_k = np.abs(tr - np.tril(K)).max() / scale
    err_s = np.abs(W[lay.n_pad:lay.n_pad + m, :n] - Ks).max() / scale
    err_y = np.abs(W[lay.y_row, :n] - y).max()
    print("pair MFMA K build: max rel err K %.2e, K_s %.2e, y %.1e" % (err_k, err_s, err_y))
    assert err_k <= 1e-12 and err_s <= 1e-12 and err_y == 0.0


@pytest.mark.parametrize("d", [4, 8])
@pytest.mark.parametrize("op,se_first,ard", [("ADD", True, True), ("MUL", True, False), ("ADD", False, True),
                                             ("MUL", False, True)])
def test_pair_mfma_matches_the_oracle(d, op, se_first, ard):
    rng = np.random.default_rng(40 + d)
    n, m = 333, 45                     # edge tiles, test rows, the y row
    x, xs = rng.uniform(0, 1, (n, d)), rng.uniform(0, 1, (m, d))
    y = rng.standard_normal(n)
    tree, hyp = _tree(op, se_first, ard), _hyp(d, se_first, ard, rng)
    f, Ws = _assemble(tree, hyp, d, x, xs, y, 1e-2)
    _check_against_oracle(tree, hyp, d, x, xs, y, 1e-2, Ws[0], f.layout)


@pytest.mark.parametrize("d", [4, 8])
@pytest.mark.parametrize("op,se_first,ard", [("ADD", True, True), ("MUL", False, False)])
def test_pair_features_prepass_is_bitwise_the_staged_path(d, op, se_first, ard):
    rng = np.random.default_rng(7 + d)
    n, m = 517, 70
    x, xs = rng.uniform(-2, 2, (n, d)), rng.uniform(-2, 2, (m, d))
    y = rng.standard_normal(n)
    tree, hyp = _tree(op, se_first, ard), _hyp(d, se_first, ard, rng)
    out = []
    for feat in (1, 0):
        old = nat.tune("asm_feat", feat)
        try:
            _, Ws = _assemble(tree, hyp, d, x, xs, y, 1e-2, batch=2)
            out.append([np.tril(w) for w in Ws])
        finally:
            nat.tune("asm_feat", old)
    for a, b in zip(*out):
        assert np.array_equal(a, b)


def test_pair_tiles_outside_the_bounds_take_the_direct_loop():
    """Row blocks far from the origin (|u|^2 / l^2 above the bound) and beyond |x / p| = 4 (no sin / cos form):
    their tiles fall back, the others stay on MFMA; every entry still matches the oracle."""
    d = 8
    rng = np.random.default_rng(99)
    n, m = 400, 20
    x = rng.uniform(0, 1, (n, d))
    x[128:192] += 9.0                  # one 64-point block: |u|^2 ~ 8 * 90 > 512 l^2, |x / p| > 4
    x[256:320, 0] += 3.0               # another: the SE bound holds, |x / p| ~ 3.1 still in the sin / cos range
    xs = rng.uniform(0, 1, (m, d))
    y = rng.standard_normal(n)
    tree, hyp = _tree("ADD", True, True), _hyp(d, True, True, rng)
    f, Ws = _assemble(tree, hyp, d, x, xs, y, 1e-2)
    _check_against_oracle(tree, hyp, d, x, xs, y, 1e-2, Ws[0], f.layout)


@pytest.mark.parametrize("op", ["ADD", "MUL"])
def test_pair_diagonal_tiles_symmetric_with_exact_diagonal(op):
    """Diagonal tiles take the symmetric form of the SE exponent (|u_i|^2 + |u_j|^2 summed first): each is bitwise
    symmetric, and its diagonal is k(x, x) + noise exactly (sg_se + sg_per for ADD, their product for MUL)."""
    d = 8
    rng = np.random.default_rng(3)
    n = 320
    x = rng.uniform(0, 1, (n, d))
    y = rng.standard_normal(n)
    tree, hyp = _tree(op, True, True), _hyp(d, True, True, rng)
    noise = 0.0123
    _, Ws = _assemble(tree, hyp, d, x, None, y, noise)
    W = Ws[0]
    kself = (1.0 * 1.0 if op == "MUL" else 1.0 + 1.0) + noise     # unscaled leaves: sg = 1
    for t in range(n // 64):
        T = W[64 * t:64 * t + 64, 64 * t:64 * t + 64]
        assert np.array_equal(T.view(np.uint64), T.T.view(np.uint64)), t
        assert np.all(np.diag(T) == kself), (t, np.diag(T)[:4])


def test_pair_path_ragged_members_bitwise_vs_staging():
    """Ragged batches (gpk_*_ragged, members of different sizes): the pre-pass classifies each member's rows with its
    own n, so the interior / edge split and the padding rows match the per-tile staging bit for bit."""
    d = 8
    tree = _tree("ADD", True, True)
    k = make_kernel(tree, d)
    kd = engine.kernel_descriptor(k, d)
    rng = np.random.default_rng(17)
    dev = engine.device()
    sizes = [300, 130, 257]
    members = []
    for nb in sizes:
        x = torch.as_tensor(rng.uniform(0, 1, (nb, d)), device=dev)
        y = torch.as_tensor(rng.standard_normal(nb), device=dev)
        h = torch.as_tensor(_flat(_hyp(d, True, True, rng)), device=dev)
        members.append((kd, h, x, y, None))
    res = []
    for feat in (1, 0):
        old = nat.tune("asm_feat", feat)
        try:
            f = engine.RaggedFactorization(sizes, d).run(members, 1e-2)
            assert int(f.info.abs().max()) == 0
            res.append((f.nlml().cpu().clone(), [f.cholesky(b).cpu().clone() for b in range(len(sizes))]))
        finally:
            nat.tune("asm_feat", old)
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)


def test_pair_path_gradient_matches_the_oracle():
    """The identity-augmented build (value + gradient, gpk_nlml_grad) of the C5 tree at D = 8 goes through the pair
    path too (the identity rows through the tile list): -LML and its gradient against the oracle's autodiff tape."""
    from oracle import gp_autodiff as ad
    d = 8
    tree = _tree("ADD", True, True)
    rng = np.random.default_rng(23)
    hyp = [[0.6 + 0.05 * i for i in range(d)], 1.0, 0.5]
    xs = rng.uniform(0, 1, (300, d))
    ys = np.sin(xs.sum(1)) + 0.1 * rng.standard_normal(300)
    nl, grads, gnoise = ad.nlml_and_grad(tree, hyp, 0.05, xs, ys)
    kd = engine.kernel_descriptor(make_kernel(tree, d), d)
    dev = engine.device()
    f = engine.InverseFactorization(300, d, 1)
    H = torch.as_tensor(_flat(hyp)).to(dev).reshape(1, -1).contiguous()
    f.run(kd, H, kd.n_hyp, torch.tensor([0.05], dtype=F64, device=dev), 0,
          torch.tensor(xs, device=dev).contiguous(), 0, torch.tensor(ys, device=dev).reshape(1, -1).contiguous(), 0)
    g = f.gradient()[0].cpu().numpy()
    exp = np.concatenate([np.asarray(v, dtype=np.float64).reshape(-1) for v in grads] + [[gnoise]])
    assert abs(float(f.nlml().cpu()[0]) - nl) <= 1e-10 * abs(nl)
    assert np.max(np.abs(g - exp)) <= 1e-8 * np.max(np.abs(exp))
