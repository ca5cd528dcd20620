"""Generate the golden vectors under tests/golden/ from the CPU oracle (oracle/gp_oracle.py).

    python tests/golden/make_golden.py            # all fixtures (a few minutes, ~8 GB RAM)
    python tests/golden/make_golden.py --small    # skip C4 / C5

The reference (gpbasics) cannot run here (TensorFlow absent), so these vectors pin the
restatement, which is itself pinned by closed-form answers (tests/test_oracle.py).
Inputs follow SURVEY §8(d); generator: numpy default_rng(seed).
"""
from __future__ import annotations

import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import gp_oracle as o  # noqa: E402

SE = ("SE", {"ard": False})


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    print("wrote %s (%d bytes)" % (path, os.path.getsize(path)))


def c1():
    x, y = o.make_inputs("C1")
    c = o.nlml_components(SE, [0.1], 1e-8, x, y)
    save("c1_se_n256", x=x, y=y, l=0.1, noise=1e-8, nlml=c["nlml"], fit=c["fit"], logdet=c["logdet"],
         L=c["L"], alpha=c["alpha"].reshape(-1))


def c2():
    x, y = o.make_inputs("C2")
    xs = np.linspace(-0.05, 1.05, 512).reshape(-1, 1)
    c = o.nlml_components(SE, [0.1], 1e-2, x, y)
    mu, var = o.posterior(SE, [0.1], 1e-2, x, y, xs)
    save("c2_se_n4096", x=x, y=y, xs=xs, l=0.1, noise=1e-2, nlml=c["nlml"], fit=c["fit"], logdet=c["logdet"],
         mu=mu, var_diag=np.diag(var).copy(), var_block=var[:64, :64].copy(), alpha_head=c["alpha"].reshape(-1)[:64])


def c3():
    x, y = o.make_inputs("C3")
    # the reference's L1 Matern is indefinite for D=4 (its Cholesky fails); C3 uses the Euclidean form
    tree = ("MAT52", {"ard": True, "standard": True})
    ls = [0.25, 0.5, 0.75, 1.0]
    c = o.nlml_components(tree, [ls], 1e-1, x, y)
    save("c3_mat52ard_n8192", x_sha256=digest(x), y_sha256=digest(y), ls=np.array(ls), noise=1e-1,
         nlml=c["nlml"], fit=c["fit"], logdet=c["logdet"])


def c4():
    x, y = o.make_inputs("C4")
    ls = np.geomspace(0.02, 0.5, 16)
    sg = np.geomspace(0.25, 4.0, 8)
    cands = np.array([[a, b] for a in ls for b in sg])
    out = np.empty(len(cands))
    for i, (a, b) in enumerate(cands):
        out[i] = o.nlml(SE, [a, b], 1e-2, x, y, scaled=True)
    save("c4_sweep128_n4096", x=x, y=y, cands=cands, noise=1e-2, nlml=out)


def c5():
    x, y = o.make_inputs("C5")
    tree = ("ADD", [("SE", {"ard": True}), ("PER", {"standard": True})])
    ls = list(np.linspace(0.4, 1.1, 8))
    c = o.nlml_components(tree, [ls, 1.0, 0.5], 1e-2, x, y)
    save("c5_seard_per_n16384", x_sha256=digest(x), y_sha256=digest(y), ls=np.array(ls), per=np.array([1.0, 0.5]),
         noise=1e-2, nlml=c["nlml"], fit=c["fit"], logdet=c["logdet"])


def small_trees():
    """Composite trees, scaled kernels, the expanded SE norm and batch mode at small N."""
    rng = np.random.default_rng(11)
    # 1-D inputs: PER on an L1 distance is only guaranteed positive definite in one dimension
    x = rng.uniform(-1, 1, (300, 1))
    y = np.sin(3 * x[:, 0]) + 0.05 * rng.standard_normal(300)
    tree = ("MUL", [("ADD", [SE, ("MAT32", {"ard": False})]), ("PER", {})])
    hyp = [0.6, 1.3, 0.8, 0.9, 1.1, 2.5, 0.7]  # scaled: SE [l, sg], MAT32 [l, sg], PER [l, p, sg]
    nl_scaled = o.nlml(tree, hyp, 1e-3, x, y, scaled=True)
    nl_exp = o.nlml(SE, [0.3], 1e-3, x, y, se_expanded=True)
    xb = rng.uniform(0, 1, (3, 64, 1))
    yb = np.sin(6 * xb[..., 0]) + 0.1 * rng.standard_normal((3, 64))
    nl_batch = o.batch_nlml(SE, [0.2], 1e-2, xb, yb)
    save("small_trees", x=x, y=y, hyp=np.array(hyp), nlml_scaled_tree=nl_scaled, nlml_se_expanded=nl_exp,
         xb=xb, yb=yb, nlml_batch=nl_batch)


if __name__ == "__main__":
    t0 = time.time()
    c1()
    small_trees()
    c2()
    c3()
    if "--small" not in sys.argv:
        c4()
        c5()
    print("done in %.1f s" % (time.time() - t0))
