"""Ragged-batch factorisation time (segmented / blockwise models: one batched factorisation of
members of different sizes, gpk_*_ragged) against the time of a uniform batch of the largest size.

usage: python tools/bench_ragged.py [n_max] [members]
Cases: one member of n_max plus (members - 1) of n_max / 2; all members n_max / 2 except the last;
a uniform batch of n_max.  Prints ms per call (HIP-synchronised wall time, median of 5) and the
algorithmic -LML work rate (sum of n_b^3 / 3 over the members).
"""
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import engine  # noqa: E402
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk  # noqa: E402


def run_case(sizes):
    dev = torch.device("cuda", 0)
    kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
    members = []
    for b, nb in enumerate(sizes):
        x = torch.sort(torch.rand(nb, 1, dtype=torch.float64, device=dev), dim=0).values.contiguous()
        y = torch.sin(12.0 * x[:, 0]).contiguous()
        members.append((kd, torch.tensor([0.05 + 0.01 * b], dtype=torch.float64, device=dev), x, y, None))
    f = engine.RaggedFactorization(sizes, 1)
    for _ in range(2):
        f.run(members, 1e-2)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        f.run(members, 1e-2)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    ms = statistics.median(ts)
    flops = sum(float(nb) ** 3 / 3.0 for nb in sizes)
    return {"sizes": "%d x %d + %d x %d" % (sizes.count(sizes[0]), sizes[0], len(sizes) - sizes.count(sizes[0]),
                                              sizes[-1]) if len(set(sizes)) > 1 else "%d x %d" % (len(sizes), sizes[0]),
            "ms": round(ms, 3), "work_tflops": round(flops / (ms * 1e-3) / 1e12, 2),
            "info": int(f.info.abs().max().item())}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    for sizes in ([n] + [n // 2] * (k - 1), [n // 2] * (k - 1) + [n], [n] * k, [n // 2] * k):
        print(json.dumps(run_case(sizes)), flush=True)
