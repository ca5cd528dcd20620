"""Timing of the approximation paths on one GPU, with the oracle on the host beside it.

usage: python tools/bench_approx.py [n] [reps]
Prints one JSON line: per-metric device ms (median of reps after one warm-up; every metric is built
fresh per repetition so no cache carries over), the building blocks' rates (gpk_dgemm TF/s on an
n x n x m product, gpk_syevj ms and sweeps and gpk_syevd ms on K_mm) and the numpy/SciPy oracle's ms for the same
metric (one evaluation, 16 threads)."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import engine  # noqa: E402
from gaussianprocessfundamentals_amd.DataHandling.DataInput import DataInput  # noqa: E402
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk  # noqa: E402
from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction  # noqa: E402
from gaussianprocessfundamentals_amd.Metrics import MatrixHandlingTypes as mht  # noqa: E402
from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type  # noqa: E402
from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType  # noqa: E402
from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import GaussianProcess  # noqa: E402
from oracle import gp_oracle as o  # noqa: E402

A, H = mht.MatrixApproximations, mht.NumericalMatrixHandlingType
SE = ("SE", {"ard": False})


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    m = int(n * 0.1)
    rng = np.random.default_rng(1)
    x = np.sort(rng.uniform(0, 1, (n, 1)), axis=0)
    y = np.sin(4 * np.pi * x[:, 0]) + 0.1 * rng.standard_normal(n)
    z = np.linspace(0, 1, m).reshape(-1, 1)
    l, noise = 0.01, 1e-2      # lengthscale ~ the inducing spacing: K_mm of full numerical rank
    out = {"n": n, "m": m, "kernel": "SE", "lengthscale": l, "noise": noise, "device_ms": {}, "oracle_ms": {}}

    def gp_obj():
        di = DataInput(x, y.reshape(-1, 1), x[:8], y[:8].reshape(-1, 1))
        di.set_mean_function(ZeroMeanFunction(1))
        g = GaussianProcess(bk.SquaredExponentialKernel(1), ZeroMeanFunction(1))
        g.set_data_input(di)
        return g

    hyp = [torch.tensor([l], dtype=torch.float64)]
    nz = torch.tensor(noise, dtype=torch.float64)
    zt = torch.tensor(z)
    cases = [
        ("exact_cholesky", A.NONE, H.CHOLESKY_BASED, None),
        ("nystroem_cholesky", A.BASIC_NYSTROEM, H.CHOLESKY_BASED, zt),
        ("nystroem_strict", A.BASIC_NYSTROEM, H.STRICT_INVERSE, zt),
        ("skc_lower_cholesky", A.SKC_LOWER_BOUND, H.CHOLESKY_BASED, zt),
        ("skc_upper", A.SKC_UPPER_BOUND, H.LINEAR_CONJUGATE_GRADIENT, zt),
        ("ski_strict", A.SKI, H.STRICT_INVERSE, None),
        ("ski_lcg", A.SKI, H.LINEAR_CONJUGATE_GRADIENT, None),
    ]
    values = {}
    for name, approx, handling, ind in cases:
        ts = []
        for r in range(reps + 1):
            g = gp_obj()
            met = get_metric_by_type(MetricType.LL, g, approx, handling, subset_size=None if approx is A.SKC_UPPER_BOUND else m)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            v = met.get_metric(hyp, nz, ind)
            val = float(v.reshape(-1)[0])
            torch.cuda.synchronize()
            if r:
                ts.append((time.perf_counter() - t0) * 1e3)
        out["device_ms"][name] = round(float(np.median(ts)), 3)
        values[name] = val
    out["values"] = values
    # building blocks
    knm = torch.tensor(o.kernel_matrix(SE, [l], x, z), device="cuda")
    for _ in range(2):
        engine.dgemm(knm, knm, trans_b=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        engine.dgemm(knm, knm, trans_b=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    out["dgemm_nxnxm"] = {"ms": round(dt * 1e3, 3), "tflops": round(2.0 * n * n * m / dt / 1e12, 2)}
    kmm = torch.tensor(o.kernel_matrix(SE, [l], z, z), device="cuda")
    engine.syevj(kmm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, _, sweeps = engine.syevj(kmm)
    torch.cuda.synchronize()
    out["syevj_m"] = {"ms": round((time.perf_counter() - t0) * 1e3, 2), "sweeps": sweeps}
    engine.syevd(kmm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    engine.syevd(kmm)
    torch.cuda.synchronize()
    out["syevd_m"] = {"ms": round((time.perf_counter() - t0) * 1e3, 2)}
    # oracle (host)
    for name, fn in (("exact_cholesky", lambda: o.nlml(SE, [l], noise, x, y)),
                     ("nystroem_cholesky", lambda: o.nystroem_nlml(SE, [l], noise, x, y, z)),
                     ("skc_upper", lambda: o.skc_upper_bound(SE, [l], noise, x, y, z)),
                     ("ski_strict", lambda: o.ski_nlml(SE, [l], noise, x, y, m, handling="STRICT_INVERSE"))):
        t0 = time.perf_counter()
        ref = fn()
        out["oracle_ms"][name] = round((time.perf_counter() - t0) * 1e3, 1)
        out.setdefault("rel_err_vs_oracle", {})[name] = abs(values[name] - ref) / abs(ref)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
