"""K build (gpk_assemble): the interior-tile loop (compile-time dimension, column point in registers) against
the generic per-element loop, which the oracle parity tests pin (tests/test_gpu_parity.py).

gpk_tune("asm_generic", 1) sends every tile through the generic loop; both must write the same bits for
every kernel op, tree shape, dimension (the specialised D = 1, 2, 3, 4, 8 and a generic one), the scaled /
expanded-norm flags, with test rows and ragged members (edge tiles) and in fp32.  Needs the MI355X.
"""
import ctypes

import numpy as np
import pytest
import torch

from tests.helpers import make_kernel, set_flags

from gaussianprocessfundamentals_amd import _native as nat
from gaussianprocessfundamentals_amd import engine

pytestmark = pytest.mark.gpu

TREES = [("SE", {}), ("SE", {"ard": True}), ("MAT52", {"ard": True, "standard": True}), ("MAT32", {}),
         ("PER", {}), ("PER", {"standard": True}), ("ADD", [("SE", {"ard": True}), ("PER", {"standard": True})]),
         ("MUL", [("SE", {}), ("MAT32", {"standard": True})])]


def _assemble(kd, lay, H, NZ, X, Xs, Y, W):
    L = nat.lib()
    s = nat.stream_handle(W.device)
    nat.check(L.gpk_assemble(ctypes.byref(kd), ctypes.byref(lay), nat.ptr(H), kd.n_hyp, nat.ptr(NZ), 0,
                             nat.ptr(X), 0, nat.ptr(Xs) if Xs is not None else None, 0, None, 0,
                             nat.ptr(Y), 0, nat.ptr(W), s), "gpk_assemble")
    torch.cuda.synchronize()


def _build_both(tree, d, n, m, batch, dtype, scaled=False, expanded=False):
    set_flags(scaled=scaled, expanded=expanded)
    try:
        k = make_kernel(tree, d)
        kd = engine.kernel_descriptor(k, d)
    finally:
        set_flags()
    rng = np.random.default_rng(d * 100 + n)
    dev = engine.device()
    X = torch.as_tensor(rng.uniform(0, 1, (n, d)), device=dev).contiguous()
    Xs = torch.as_tensor(rng.uniform(0, 1, (m, d)), device=dev).contiguous() if m else None
    Y = torch.as_tensor(rng.standard_normal(n), device=dev).reshape(1, -1).contiguous()
    H = torch.as_tensor(0.3 + rng.uniform(0, 1, (batch, kd.n_hyp)), device=dev).contiguous()
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    out = []
    for generic in (1, 0):
        old = nat.tune("asm_generic", generic)
        try:
            f = engine.AugmentedFactorization(n, d, m, batch, dtype)
            f.W.zero_()
            _assemble(kd, f.layout, H, NZ, X, Xs, Y, f.W)
            out.append(torch.stack([torch.tril(f.w(b)) for b in range(batch)]).cpu())
        finally:
            nat.tune("asm_generic", old)
    return out


@pytest.mark.parametrize("tree", TREES)
@pytest.mark.parametrize("d", [1, 2, 3, 4, 5, 8])
def test_interior_loop_is_bitwise_the_generic_loop(tree, d):
    gen, fast = _build_both(tree, d, 300, 40, 2, torch.float64)
    assert torch.equal(gen, fast)


@pytest.mark.parametrize("tree", [("SE", {}), ("PER", {}), ("MAT52", {"ard": True, "standard": True})])
def test_interior_loop_flags_and_fp32(tree):
    for scaled, expanded in ((True, False), (False, True)):
        gen, fast = _build_both(tree, 4, 200, 0, 1, torch.float64, scaled=scaled, expanded=expanded)
        assert torch.equal(gen, fast)
    # (fp32 single nodes take f32_fast_kernel by default -- its own f32 arithmetic, tested below; the interior loop
    # of the general instantiation, with it off, is bitwise the generic loop in fp32 too)
    old = nat.tune("asm_f32_fast", 0)
    try:
        gen, fast = _build_both(tree, 4, 200, 30, 1, torch.float32)
    finally:
        nat.tune("asm_f32_fast", old)
    assert torch.equal(gen, fast)


F32_TREES = [("SE", {}), ("SE", {"ard": True}), ("MAT32", {}), ("MAT32", {"ard": True, "standard": True}),
             ("MAT52", {"ard": True, "standard": True}), ("MAT52", {})]


def _build_f32(tree, d, n, m, batch, scaled):
    """The augmented matrix of `tree` in f32 with asm_f32_fast on and off, and in f64 (the general path, which the
    oracle tests pin): three [batch, p, p] CPU tensors (untriangled: diagonal tiles hold both triangles)."""
    set_flags(scaled=scaled)
    try:
        kd = engine.kernel_descriptor(make_kernel(tree, d), d)
    finally:
        set_flags()
    rng = np.random.default_rng(d * 1000 + n + m)
    dev = engine.device()
    X = torch.as_tensor(rng.uniform(0, 1, (n, d)), device=dev).contiguous()
    Xs = torch.as_tensor(rng.uniform(0, 1, (m, d)), device=dev).contiguous() if m else None
    Y = torch.as_tensor(rng.standard_normal(n), device=dev).reshape(1, -1).contiguous()
    H = torch.as_tensor(0.2 + rng.uniform(0, 1, (batch, kd.n_hyp)), device=dev).contiguous()
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    out = []
    for dtype, fast in ((torch.float32, 1), (torch.float32, 0), (torch.float64, 0)):
        old = nat.tune("asm_f32_fast", fast)
        try:
            f = engine.AugmentedFactorization(n, d, m, batch, dtype)
            f.W.fill_(7.0)
            _assemble(kd, f.layout, H, NZ, X, Xs, Y, f.W)
            out.append(torch.stack([f.w(b) for b in range(batch)]).cpu())
        finally:
            nat.tune("asm_f32_fast", old)
    return out, f.layout


@pytest.mark.parametrize("tree", F32_TREES)
@pytest.mark.parametrize("d", [1, 2, 3, 4, 8])
def test_f32_fast_kbuild_against_the_f64_build(tree, d):
    """f32 K build of one SE / MAT32 / MAT52 node (f32_fast_kernel: f64 distances, the f32 hardware sqrt / exp): its
    interior tiles within 4e-6 of max|K| of the f64 build of the same inputs (C3's fp32 config); every other tile --
    test rows, the padding block, the y row and the zero rows -- bitwise the general path's f32 values; the training
    diagonal exactly (f32)(sg + noise) and the diagonal tiles exactly symmetric."""
    n, m = 300, 37
    (fast, gen, ref), lay = _build_f32(tree, d, n, m, 2, scaled=(d % 2 == 0))
    n64 = 64 * (n // 64)
    lower = torch.tril(torch.ones(lay.p, lay.p, dtype=torch.bool))
    interior = torch.zeros(lay.p, lay.p, dtype=torch.bool)
    interior[:n64, :n64] = True
    interior &= lower
    # (lower 64-tiles only are written; compare the lower triangle plus the diagonal tiles' upper halves)
    written = lower.clone()
    for t in range(lay.p // 64):
        written[64 * t:64 * t + 64, 64 * t:64 * t + 64] = True
    for b in range(2):
        err = float((fast[b].double() - ref[b])[interior].abs().max())
        scale = float(ref[b][interior].abs().max())
        assert err <= 4e-6 * scale, (err, scale)
        outside = written & ~interior
        for t in range(n64 // 64):   # (diagonal tiles' upper halves are interior too)
            outside[64 * t:64 * t + 64, 64 * t:64 * t + 64] = False
        assert torch.equal(fast[b][outside], gen[b][outside])
        dg = torch.arange(n)
        assert torch.equal(fast[b][dg, dg], gen[b][dg, dg])
        for t in range(n64 // 64):
            blk = fast[b][64 * t:64 * t + 64, 64 * t:64 * t + 64]
            assert torch.equal(blk, blk.T)


def test_interior_loop_ragged_members_bitwise():
    """Ragged batches (members of different sizes): the interior test uses each member's own n."""
    d = 3
    k = make_kernel(("ADD", [("SE", {"ard": True}), ("PER", {"standard": True})]), d)  # positive definite
    kd = engine.kernel_descriptor(k, d)
    rng = np.random.default_rng(5)
    dev = engine.device()
    sizes = [300, 130, 257]
    members = []
    for b, nb in enumerate(sizes):
        x = torch.as_tensor(rng.uniform(0, 1, (nb, d)), device=dev)
        y = torch.as_tensor(rng.standard_normal(nb), device=dev)
        h = torch.as_tensor(0.3 + rng.uniform(0, 1, kd.n_hyp), device=dev)
        members.append((kd, h, x, y, None))
    res = []
    for generic in (1, 0):
        old = nat.tune("asm_generic", generic)
        try:
            f = engine.RaggedFactorization(sizes, d).run(members, 1e-2)
            assert int(f.info.abs().max()) == 0
            res.append((f.nlml().cpu().clone(), [f.cholesky(b).cpu().clone() for b in range(len(sizes))]))
        finally:
            nat.tune("asm_generic", old)
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert torch.equal(a, b)


LDS16_TREES = [("ADD", [("SE", {"ard": True}), ("PER", {"standard": True})]),
               ("ADD", [("MUL", [("SE", {"ard": True}), ("PER", {"standard": True})]),
                        ("MAT52", {"ard": True, "standard": True})])]


@pytest.mark.parametrize("tree", LDS16_TREES)
def test_d16_ard_periodic_assembly_above_64kb_lds(tree):
    """d = 16 with ARD nodes beside a standard PER node: the K build needs 71 / 87 KB of dynamic LDS (per-point
    sin / cos slots), which gpk_assemble raises the kernel's limit for; both loops agree bitwise, and the
    factorisation of the assembled matrix succeeds."""
    gen, fast = _build_both(tree, 16, 200, 24, 2, torch.float64)
    assert torch.equal(gen, fast)
    assert torch.isfinite(fast).all() and float(fast[0, 0, 0]) > 0.0


@pytest.mark.parametrize("tree", LDS16_TREES)
def test_d16_ard_vjp_and_gradient_above_64kb_lds(tree):
    """The reverse-mode kernels of the same trees at d = 16 (gpk_kernel_vjp: 118 KB of LDS with two ARD nodes;
    gpk_nlml_grad's per-tile kernel: 86 KB) against torch autograd of the oracle's kernel program."""
    from oracle import gp_autodiff as ad
    d = 16
    rng = np.random.default_rng(16)
    x, z = rng.uniform(0, 1, (70, d)), rng.uniform(0, 1, (45, d))
    kern = make_kernel(tree, d)
    kd = engine.kernel_descriptor(kern, d)
    hyp = ([[0.6 + 0.05 * i for i in range(d)], 1.0, 0.5] if len(tree[1]) == 2 and tree[1][0][0] == "SE"
           else [[0.6 + 0.05 * i for i in range(d)], 1.0, 0.5, [0.9 + 0.03 * i for i in range(d)]])
    params = [torch.tensor(np.asarray(h, dtype=np.float64), requires_grad=True) for h in hyp]
    assert sum(p.numel() for p in params) == kd.n_hyp
    Zt = torch.tensor(z, requires_grad=True)
    K = ad.kernel_matrix_t(tree, params, torch.tensor(x), Zt, False)
    G = rng.standard_normal((70, 45))
    gref = torch.autograd.grad(torch.sum(torch.tensor(G) * K), params + [Zt])
    gh, gz = engine.kernel_vjp(kern, [torch.tensor(h, dtype=torch.float64) for h in hyp], x, z,
                               G=torch.tensor(G, device=engine.device()), want_z=True)
    exp_h = np.concatenate([g.numpy().reshape(-1) for g in gref[:-1]])
    assert np.max(np.abs(gh.cpu().numpy() - exp_h)) <= 1e-11 * np.max(np.abs(exp_h))
    assert np.max(np.abs(gz.cpu().numpy() - gref[-1].numpy())) <= 1e-11 * np.max(np.abs(gref[-1].numpy()))
    # -LML gradient (identity-augmented factorisation + the per-tile gradient kernel) against the oracle's tape
    xs = rng.uniform(0, 1, (150, d))
    ys = np.sin(xs.sum(1)) + 0.1 * rng.standard_normal(150)
    nl, grads, gnoise = ad.nlml_and_grad(tree, hyp, 0.05, xs, ys)
    dev = engine.device()
    f = engine.InverseFactorization(150, d, 1)
    H = torch.cat([torch.as_tensor(np.asarray(h, dtype=np.float64)).reshape(-1) for h in hyp]).to(dev).reshape(1, -1)
    f.run(kd, H.contiguous(), kd.n_hyp, torch.tensor([0.05], dtype=torch.float64, device=dev), 0,
          torch.tensor(xs, device=dev).contiguous(), 0, torch.tensor(ys, device=dev).reshape(1, -1).contiguous(), 0)
    g = f.gradient()[0].cpu().numpy()
    exp = np.concatenate([np.asarray(v, dtype=np.float64).reshape(-1) for v in grads] + [[gnoise]])
    assert abs(float(f.nlml().cpu()[0]) - nl) <= 1e-10 * abs(nl)
    assert np.max(np.abs(g - exp)) <= 1e-8 * np.max(np.abs(exp))


@pytest.mark.parametrize("tree", [("MAT52", {"ard": True, "standard": True}), ("SE", {})])
def test_f32_fast_kbuild_without_edge_tiles(tree):
    """n a multiple of 128, no test rows: every tile is interior or a y / zero tail tile, so f32_fast_kernel runs
    alone (no tile list, no general launch) -- C3's shape in miniature.  Interior within 4e-6 of max|K| of the f64
    build, the tail rows bitwise the general path's."""
    n = 512
    (fast, gen, ref), lay = _build_f32(tree, 4, n, 0, 1, scaled=False)
    err = float((torch.tril(fast[0][:n, :n]).double() - torch.tril(ref[0][:n, :n])).abs().max())
    assert err <= 4e-6 * float(ref[0][:n, :n].abs().max())
    assert torch.equal(torch.tril(fast[0])[n:], torch.tril(gen[0])[n:])
