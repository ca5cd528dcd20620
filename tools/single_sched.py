"""Single-evaluation (batch 1) device time of the fused -LML path under schedule knobs.

usage: GPK_RESERVE_CUS=R python tools/single_sched.py n [n ...]
For every n and every knob set below: median over 30 calls of the HIP-event span of one
AugmentedFactorization.run (K build + factorisation + read-out) on the caller's stream.
"""
import itertools
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402
from gaussianprocessfundamentals_amd import engine  # noqa: E402

engine.CHAIN_VERIFY = os.environ.get("VERIFY", "0") == "1"  # (device span only: no info read-back per call)
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk  # noqa: E402

SETS = [dict(lookahead=0, fuse_trsm=1, group=8)]
for la, fu, g in itertools.product((1,), (1, 2), (4, 8)):
    SETS.append(dict(lookahead=la, fuse_trsm=fu, group=g))
if os.environ.get("SETS"):
    SETS = [json.loads(s) for s in os.environ["SETS"].split(";")]


def main():
    dev = torch.device("cuda", 0)
    kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
    for n in [int(a) for a in sys.argv[1:]] or [4096, 8192]:
        f = engine.AugmentedFactorization(n, 1, 0, 1)
        X = torch.sort(torch.rand(n, 1, dtype=torch.float64, device=dev), dim=0).values.contiguous()
        Y = torch.rand(1, n, dtype=torch.float64, device=dev)
        H = torch.full((1, 1), 0.1, dtype=torch.float64, device=dev)
        NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
        for ks in SETS:
            for k, v in ks.items():
                nat.tune(k, v)
            ts = []
            for i in range(33):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
                e1.record()
                e1.synchronize()
                if i >= 3:
                    ts.append(e0.elapsed_time(e1))
            print(json.dumps({"n": n, "reserve": os.environ.get("GPK_RESERVE_CUS", "32"), **ks,
                              "ms": round(statistics.median(ts), 4), "min": round(min(ts), 4)}), flush=True)


if __name__ == "__main__":
    main()
