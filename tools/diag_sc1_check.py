"""Debug: the write-through (SC1) diagonal-block body as a plain launch (gpk_tune diag_version 3, chain and
fused panel solve off) against the default body, one f64 evaluation per n.  Exits 3 if a run does not finish.
usage: python tools/diag_sc1_check.py n [n ...]"""
import os
import sys
import threading

import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402
from gaussianprocessfundamentals_amd import engine  # noqa: E402
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk  # noqa: E402

nat.tune("chain", 0)
nat.tune("fuse_trsm", 0)
nat.tune("lookahead", 0)
dev = torch.device("cuda", 0)
kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
for n in [int(a) for a in sys.argv[1:]] or [1, 4096]:
    X = torch.sort(torch.rand(n, 1, dtype=torch.float64, device=dev), dim=0).values.contiguous()
    Y = torch.rand(1, n, dtype=torch.float64, device=dev)
    H = torch.full((1, 1), 0.1, dtype=torch.float64, device=dev)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    res = {}
    for ver in (2, 3):
        nat.tune("diag_version", ver)
        f = engine.AugmentedFactorization(n, 1, 0, 1)
        done = threading.Event()

        def work():
            f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
            torch.cuda.synchronize()
            done.set()

        threading.Thread(target=work, daemon=True).start()
        if not done.wait(15.0):
            print("n", n, "diag_version", ver, "NOT FINISHED", flush=True)
            os._exit(3)
        res[ver] = (float(f.out.cpu()[0]), int(f.info.cpu()[0]), f.W.clone())
    d = (res[2][2] - res[3][2]).abs().max().item()
    print("n", n, "nlml v2 %.15g v3 %.15g info %d %d max|dW| %.3g" % (res[2][0], res[3][0], res[2][1], res[3][1], d),
          flush=True)
os._exit(0)
