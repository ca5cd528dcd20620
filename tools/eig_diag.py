import sys, time, numpy as np, torch
sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp
gp.init(0)
from gaussianprocessfundamentals_amd import engine
from oracle import gp_oracle as o
for m in [409, 700, 1000, 1023, 1024, 1100, 2000]:
    rng = np.random.default_rng(m)
    for kind in ("rand", "kern"):
        if kind == "rand":
            A = rng.standard_normal((m, m)); A = 0.5 * (A + A.T)
        else:
            x = rng.uniform(0, 1, (m, 1)); A = o.k_noised(("SE", {}), [0.1], -0.3, x)
        At = torch.tensor(A, device="cuda")
        engine.syevd(At); torch.cuda.synchronize()
        t0 = time.perf_counter(); lam, V = engine.syevd(At); torch.cuda.synchronize(); dt = time.perf_counter() - t0
        ref = np.linalg.eigvalsh(A); l = lam.cpu().numpy(); Vn = V.cpu().numpy()
        print(m, kind, "ms %.1f" % (dt * 1e3), "lam err %.2e" % np.abs(l - ref).max(), "max %.3f/%.3f" % (l.max(), ref.max()),
              "orth %.2e" % np.abs(Vn.T @ Vn - np.eye(m)).max(), "res %.2e" % np.abs(A @ Vn - Vn * l).max(), flush=True)
