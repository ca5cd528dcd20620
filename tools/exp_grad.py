"""Where the time of one -LML + gradient evaluation goes (gpk_nlml_grad: augmented factorisation with
identity extra rows, then the gradient kernel).

usage: python tools/exp_grad.py [value] [n] [batch ...]   ("value": the -LML alone, gpk_nlml)
For each batch: wall time per call (look-ahead on, the default), then a per-class breakdown from the
native launch timer with the look-ahead off (each launch alone on the stream): ms, launches and the
achieved TF/s of the classes that carry algorithmic flops.
"""
import sys
import time

import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402
from gaussianprocessfundamentals_amd import engine  # noqa: E402
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk  # noqa: E402


def main():
    args = sys.argv[1:]
    value = bool(args) and args[0] == "value"
    if value:
        args = args[1:]
    n = int(args[0]) if args else 8192
    batches = [int(a) for a in args[1:]] or [1, 8]
    dev = torch.device("cuda", 0)
    X = torch.sort(torch.rand(n, 1, dtype=torch.float64, device=dev), dim=0).values.contiguous()
    Y = torch.sin(12.0 * X[:, 0]).reshape(1, n).contiguous()
    kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    for batch in batches:
        H = torch.linspace(0.05, 0.2, batch, dtype=torch.float64).reshape(batch, 1).to(dev)
        f = engine.AugmentedFactorization(n, 1, 0, batch) if value else engine.InverseFactorization(n, 1, batch)
        for _ in range(2):
            f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / reps
        print("n %d batch %d: %.3f ms per call (%.2f evals/s, %.1f TF at n^3 (gradient) or n^3/3 (value) flops)"
              % (n, batch, ms, batch * 1e3 / ms, batch * float(n) ** 3 / (3.0 if value else 1.0) / (ms * 1e-3) / 1e12),
              flush=True)
        nat.tune("lookahead", 0)
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        nat.timing_reset()
        nat.timing_enable(True)
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        nat.timing_enable(False)
        nat.tune("lookahead", 1)
        t = nat.timing_read()
        tot = sum(v["ms"] for v in t.values())
        print("   serialised sum %.3f ms" % tot)
        for c, v in t.items():
            if v["launches"]:
                tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["flops"] and v["ms"] else 0.0
                print("   %-10s %8.3f ms  %5d launches  %6.1f TF" % (c, v["ms"], v["launches"], tf), flush=True)


if __name__ == "__main__":
    main()
