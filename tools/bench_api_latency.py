"""Latency of the drop-in API as a reference user calls it: LogLikelihood.get_metric(hyp, noise) once per
candidate, float() of the result (a host synchronisation) after each call -- the pattern of the
reference's fitters (gpbasics/Optimizer/Fitter.py:91-167) -- and get_metric_and_gradient likewise.

usage: python tools/bench_api_latency.py [--no-grad] [n ...]
Prints one JSON line per N with the per-call milliseconds (median of 20 calls, distinct lengthscales).
"""
import json
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd.DataHandling.DataInput import DataInput  # noqa: E402
from gaussianprocessfundamentals_amd.KernelBasics.BaseKernels import SquaredExponentialKernel  # noqa: E402
from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction  # noqa: E402
from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type  # noqa: E402
from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType  # noqa: E402
from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import GaussianProcess  # noqa: E402


def run(n, grad=True):
    rng = np.random.default_rng(1)
    x = np.sort(rng.uniform(0.0, 1.0, n)).reshape(n, 1)
    y = np.sin(4.0 * np.pi * x[:, 0]) + 0.1 * rng.standard_normal(n)
    di = DataInput(x, y.reshape(-1, 1), x[:16], y[:16].reshape(-1, 1))
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(SquaredExponentialKernel(1), ZeroMeanFunction(1))
    g.set_data_input(di)
    m = get_metric_by_type(MetricType.LL, g)
    noise = torch.tensor(1e-2, dtype=torch.float64)
    cands = [0.08 + 0.002 * i for i in range(23)]
    times, gtimes = [], []
    for i, c in enumerate(cands):
        t0 = time.perf_counter()
        v = float(m.get_metric([torch.tensor(c, dtype=torch.float64)], noise))
        t1 = time.perf_counter()
        if i >= 3:
            times.append((t1 - t0) * 1e3)
    for i, c in enumerate(cands if grad else []):
        t0 = time.perf_counter()
        nl, grads, gn = m.get_metric_and_gradient([torch.tensor(c, dtype=torch.float64)], noise)
        float(nl), float(grads[0]), float(gn)
        t1 = time.perf_counter()
        if i >= 3:
            gtimes.append((t1 - t0) * 1e3)
    return {"n": n, "get_metric_ms": round(statistics.median(times), 3),
            "get_metric_and_gradient_ms": round(statistics.median(gtimes), 3) if gtimes else None, "last_nlml": v}


if __name__ == "__main__":
    grad = "--no-grad" not in sys.argv
    for n in [int(a) for a in sys.argv[1:] if not a.startswith("--")] or [4096, 8192]:
        print(json.dumps(run(n, grad)), flush=True)
