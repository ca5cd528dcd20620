"""Posterior mean / variance through the drop-in API on the device vs the oracle on the host.

usage: python tools/bench_posterior.py [n] [m] [reps]

GaussianProcess.predict (mu, S/GaussianProcess.py:42-85) and aux.get_posterior_var (full M x M
covariance, S/Auxiliary.py:83-93) of the SE kernel at C2's inputs (N training points, M test points
drawn from the same range), noise 1e-2: one augmented factorisation with M extra rows per call
(gpk_assemble + gpk_potrf_aug + gpk_finalize).  Timed per call with a host synchronisation (what a
caller of predict sees); the oracle restates the reference (numpy/SciPy, explicit inv(L)).
Prints one JSON line; also checks mu and diag(Sigma) against the oracle.
"""
import json
import os
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
from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import GaussianProcess  # noqa: E402
from oracle import gp_oracle as o  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    m = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    x, y = o.make_inputs("C2", n=n)
    rng = np.random.default_rng(9)
    xs = np.sort(rng.uniform(0.0, 1.0, m)).reshape(m, 1)
    di = DataInput(x, y.reshape(-1, 1), xs, np.zeros((m, 1)))
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(SquaredExponentialKernel(1), ZeroMeanFunction(1))
    g.set_data_input(di)
    hyp = [torch.tensor(0.1, dtype=torch.float64)]
    noise = torch.tensor(1e-2, dtype=torch.float64)

    def call():
        _, _, mu = g.predict(hyp, noise=noise)
        var = g.aux.get_posterior_var(hyp, noise)
        torch.cuda.synchronize()
        return mu, var

    for _ in range(3):
        call()
    t0 = time.perf_counter()
    for _ in range(reps):
        mu, var = call()
    gpu_ms = (time.perf_counter() - t0) * 1e3 / reps

    threads = int(os.environ.get("GPK_CPU_THREADS", min(16, os.cpu_count() or 1)))
    from threadpoolctl import threadpool_limits
    with threadpool_limits(limits=threads):
        o.posterior(("SE", {}), [0.1], 1e-2, x[:512], y[:512], xs[:64])  # warm
        t0 = time.perf_counter()
        mu_ref, var_ref = o.posterior(("SE", {}), [0.1], 1e-2, x, y, xs)
        cpu_ms = (time.perf_counter() - t0) * 1e3
    err_mu = float(np.max(np.abs(mu.cpu().numpy() - mu_ref)))
    err_var = float(np.max(np.abs(np.diag(var.cpu().numpy()) - np.diag(var_ref))))
    flops = n ** 3 / 3.0 + n * n * m + n * m * m  # factor + V = L^-1 K_s + Sigma = K_ss - V^T V
    print(json.dumps({"what": "posterior mu + full covariance via predict / get_posterior_var", "n": n, "m": m,
                      "gpu_ms_per_call": round(gpu_ms, 3), "gpu_tflops": round(flops / (gpu_ms * 1e-3) / 1e12, 2),
                      "cpu_oracle_ms": round(cpu_ms, 1), "cpu_threads": threads,
                      "speedup": round(cpu_ms / gpu_ms, 1), "max_abs_err_mu": err_mu,
                      "max_abs_err_diag_var": err_var}))
    assert err_mu < 1e-8 and err_var < 1e-8


if __name__ == "__main__":
    main()
