"""Sweep of the identity-augmented persistent launch's planner knobs (value + gradient):
chain_group (deferred-update depth), chain_group_corner / chain_corner_tail (the -K^-1 corner's groups) and
chain_group_la, through the drop-in API's get_metric_and_gradient (median of 15 calls, a host synchronisation after
each, as tools/bench_api_latency.py).  Every combination's -LML and gradient are compared with the first one's.

usage: python tools/grad_knob_sweep.py N [quick]
Prints one JSON line per combination.
"""
import itertools
import json
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402
from gaussianprocessfundamentals_amd.DataHandling.DataInput import DataInput  # noqa: E402
from gaussianprocessfundamentals_amd.KernelBasics.BaseKernels import SquaredExponentialKernel  # noqa: E402
from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction  # noqa: E402
from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type  # noqa: E402
from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType  # noqa: E402
from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import GaussianProcess  # noqa: E402


def metric(n):
    rng = np.random.default_rng(1)
    x = np.sort(rng.uniform(0.0, 1.0, n)).reshape(n, 1)
    y = np.sin(4.0 * np.pi * x[:, 0]) + 0.1 * rng.standard_normal(n)
    di = DataInput(x, y.reshape(-1, 1), x[:16], y[:16].reshape(-1, 1))
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(SquaredExponentialKernel(1), ZeroMeanFunction(1))
    g.set_data_input(di)
    return get_metric_by_type(MetricType.LL, g)


def timed(m, calls=15):
    noise = torch.tensor(1e-2, dtype=torch.float64)
    ts, last = [], None
    for i in range(calls + 3):
        c = torch.tensor(0.08 + 0.002 * (i % 7), dtype=torch.float64)
        t0 = time.perf_counter()
        nl, grads, gn = m.get_metric_and_gradient([c], noise)
        last = (float(nl), float(grads[0]), float(gn))
        t1 = time.perf_counter()
        if i >= 3:
            ts.append((t1 - t0) * 1e3)
    return statistics.median(ts), min(ts), last


if __name__ == "__main__":
    n = int(sys.argv[1])
    quick = len(sys.argv) > 2
    m = metric(n)
    groups = [0, 6, 8, 12, 16] if not quick else [0, 8]
    corners = [8, 16]
    tails = [4, 8, 16] if not quick else [8]
    las = [1, 2, 3] if not quick else [2]
    ref = None
    for g, gc, tl, la in itertools.product(groups, corners, tails, las):
        with nat.thread_tune(chain_group_eye=g, chain_group_corner=gc, chain_corner_tail=tl, chain_group_la=la):
            med, mn, last = timed(m)
        if ref is None:
            ref = last
        dev = max(abs(a - b) / max(abs(b), 1e-300) for a, b in zip(last, ref))
        print(json.dumps({"n": n, "chain_group": g, "chain_group_corner": gc, "chain_corner_tail": tl,
                          "chain_group_la": la, "ms_median": round(med, 3), "ms_min": round(mn, 3),
                          "max_rel_vs_first": dev}), flush=True)
