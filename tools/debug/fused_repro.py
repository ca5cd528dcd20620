"""Fused panel solve vs separate launch on the sweep that failed (N=700, SE l up to 0.5)."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp
gp.init(0)
from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd import _native as nat
from gaussianprocessfundamentals_amd.sweep import native_batched_evaluator
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
for la in (0, 2):
    nat.tune("lookahead", la)
    for fuse in (0, 1):
        nat.tune("fuse_trsm", fuse)
        for b0, b1 in ((15, 20), (20, 23), (17, 18)):
            H = torch.tensor([[c] for c in cands[b0:b1]], dtype=torch.float64, device=dev)
            f = engine.AugmentedFactorization(700, 1, 0, b1 - b0)
            f.W.zero_()
            f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
            torch.cuda.synchronize()
            print("la", la, "fuse", fuse, "cands", b0, b1, "info", f.info.tolist(), "nlml", [round(v, 6) for v in f.nlml().tolist()],
                  "exp", [round(o.nlml(SE, [c], 1e-2, x, y), 6) for c in cands[b0:b1]], flush=True)
nat.tune("lookahead", 2)
for fuse in (0, 1):
    nat.tune("fuse_trsm", fuse)
    for P in (1, 2):
        ev = native_batched_evaluator(make_kernel(SE, 1), x, y, 1e-2, max_batch=5, pipeline=P)
        r = ev(torch.tensor([[c] for c in cands], dtype=torch.float64))
        torch.cuda.synchronize()
        print("fuse", fuse, "P", P, "info", r[:, 1].tolist(), flush=True)
