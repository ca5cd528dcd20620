"""Fused panel solve with W pre-filled with NaN / huge garbage: does any uninitialised element leak in?"""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp
gp.init(0)
from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd import _native as nat
from oracle import gp_oracle as o
from tests.helpers import make_kernel
SE = ("SE", {"ard": False})
x, y = o.make_inputs("C1", n=700, seed=6)
dev = engine.device()
kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
cands = np.geomspace(0.02, 0.5, 23)
NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
nat.tune("lookahead", 0)
for fill in (float("nan"), 1e300, 0.0):
    for fuse in (0, 1):
        nat.tune("fuse_trsm", fuse)
        H = torch.tensor([[c] for c in cands[15:20]], dtype=torch.float64, device=dev)
        f = engine.AugmentedFactorization(700, 1, 0, 5)
        f.W.fill_(fill)
        f.Winv.fill_(fill)
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        W = f.w(0).cpu().numpy()
        lay = f.layout
        bad_rows = [r for r in range(int(lay.p)) if not np.all(np.isfinite(W[r, :min(r + 1, int(lay.n_pad))]))]
        print("fill", fill, "fuse", fuse, "info", f.info.tolist(), "nlml", [round(v, 6) for v in f.nlml().tolist()],
              "nonfinite rows (lower, K cols)", bad_rows[:5], len(bad_rows), flush=True)
