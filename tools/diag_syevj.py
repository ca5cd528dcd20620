"""gpk_syevj convergence vs the absolute rotation threshold (tune key syevj_abs_tol_e3): sweeps,
time and eigenvalue / pinv accuracy against numpy on kernel Gram matrices and a random symmetric one.

usage: python tools/diag_syevj.py"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402
from gaussianprocessfundamentals_amd import engine  # noqa: E402
from oracle import gp_oracle as o  # noqa: E402

SE = ("SE", {"ard": False})
rng = np.random.default_rng(2)
G = rng.standard_normal((300, 300))
mats = {
    "grid409_l0.01": o.kernel_matrix(SE, [0.01], np.linspace(0, 1, 409).reshape(-1, 1), np.linspace(0, 1, 409).reshape(-1, 1)),
    "grid409_l0.05": o.kernel_matrix(SE, [0.05], np.linspace(0, 1, 409).reshape(-1, 1), np.linspace(0, 1, 409).reshape(-1, 1)),
    "rand300": (G + G.T) / 2,
}
for tol in (1000, 10000, 100000):
    nat.tune("syevj_abs_tol_e3", tol)
    for name, K in mats.items():
        Kd = torch.tensor(K, device="cuda")
        engine.syevj(Kd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lam, V, sweeps = engine.syevj(Kd)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        lam, V = lam.cpu().numpy(), V.cpu().numpy()
        ref = np.linalg.eigvalsh(K)
        scale = np.max(np.abs(ref))
        P = engine.pinv_sym(Kd).cpu().numpy()
        Pref = o.tf_pinv(K)
        print("tol_e3 %5d %-14s sweeps %2d  %7.1f ms  eig err %.2e  recon %.2e  orth %.2e  pinv rel %.2e" % (
            tol, name, sweeps, ms, np.max(np.abs(np.sort(lam) - ref)) / scale,
            np.max(np.abs(V @ np.diag(lam) @ V.T - K)) / scale, np.max(np.abs(V.T @ V - np.eye(len(K)))),
            np.max(np.abs(P - Pref)) / np.max(np.abs(Pref))))
nat.tune("syevj_abs_tol_e3", 1000)
