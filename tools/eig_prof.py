"""Run gpk_syevd a few times on one matrix (for rocprofv3 --kernel-trace --stats): python tools/eig_prof.py [m] [reps]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gaussianprocessfundamentals_amd import engine  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 409
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rng = np.random.default_rng(0)
z = rng.uniform(0, 1, (m, 1))
K = np.exp(-0.5 * (z - z.T) ** 2 / 0.01 ** 2)
A = torch.tensor(K, device="cuda")
engine.syevd(A)
torch.cuda.synchronize()
for _ in range(reps):
    t = time.perf_counter()
    lam, V = engine.syevd(A)
    torch.cuda.synchronize()
    print("m %d syevd %.2f ms" % (m, 1e3 * (time.perf_counter() - t)), flush=True)
