"""Small batches: the persistent launch over every member (gpk_tune chain 2, chain_max_batch) against the
launch path, HIP-event span of AugmentedFactorization.run (K build + factorisation + read-out), median of 20.

usage: python tools/chain_batch_ab.py [n ...]   -> one JSON line per (n, batch, path)"""
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402
from gaussianprocessfundamentals_amd import engine  # noqa: E402
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk  # noqa: E402

engine.CHAIN_VERIFY = False
dev = torch.device("cuda", 0)
kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
for n in [int(a) for a in sys.argv[1:]] or [2048, 4096]:
    X = torch.sort(torch.rand(n, 1, dtype=torch.float64, device=dev), dim=0).values.contiguous()
    Y = torch.rand(1, n, dtype=torch.float64, device=dev)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    for batch in (1, 2, 4, 8, 16):
        H = torch.linspace(0.08, 0.12, batch, dtype=torch.float64, device=dev).reshape(batch, 1).contiguous()
        f = engine.AugmentedFactorization(n, 1, 0, batch)
        for mode in (0, 2):
            with nat.thread_tune(chain=mode, chain_max_batch=64, chain_batch_max_rows=100000):
                ts = []
                for i in range(23):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
                    e1.record()
                    e1.synchronize()
                    if i >= 3:
                        ts.append(e0.elapsed_time(e1))
            ms = statistics.median(ts)
            print(json.dumps({"n": n, "batch": batch, "path": "chain" if mode else "launch", "ms": round(ms, 4),
                              "evals_per_s": round(batch / ms * 1e3, 1)}), flush=True)
