"""A/B of the diagonal-block kernel versions (gpk_tune("diag_version", 1 | 2)): per-launch HIP-event
span of the diag / trsm / update classes with the look-ahead off, and the step time of a
single-candidate factorisation with the default schedule.

usage: python tools/exp_diag_ab.py [batch] [n]
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
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    dev = torch.device("cuda", 0)
    f = engine.AugmentedFactorization(n, 1, 0, batch)
    kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
    X = torch.sort(torch.rand(n, 1, dtype=torch.float64, device=dev), dim=0).values.contiguous()
    Y = torch.rand(1, n, dtype=torch.float64, device=dev)
    H = torch.full((batch, 1), 0.1, dtype=torch.float64, device=dev)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    for v in (1, 2, 1, 2):
        nat.tune("diag_version", v)
        nat.tune("lookahead", 0)
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        nat.timing_reset()
        nat.timing_enable(True)
        for _ in range(3):
            f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        nat.timing_enable(False)
        t = nat.timing_read()
        nat.tune("lookahead", 1)
        for _ in range(3):
            f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / reps
        print("diag_version %d: " % v + "  ".join(
            "%s %.1f us x %d" % (c, t[c]["ms"] * 1e3 / max(1, t[c]["launches"]), t[c]["launches"] // 3)
            for c in ("diag", "trsm", "update")) + "   | look-ahead step %.3f ms (batch %d, n %d)" % (ms, batch, n))
    nat.tune("diag_version", 2)


if __name__ == "__main__":
    main()
