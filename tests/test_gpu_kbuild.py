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
    gen, fast = _build_both(tree, 4, 200, 30, 1, torch.float32)
    assert torch.equal(gen, fast)


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
