"""Diagonal-block kernel timing with the look-ahead off (each launch alone on the stream).

usage: python tools/exp_diag.py [batch] [n]
Prints the average HIP-event span of the diag / trsm / update classes for the timing-only ablations
of gpk_tune("diag_debug", v): 0 full, 1 no inverse, 2 no potf2, 4 no tile ops, 7 nothing but the
block load / store, 15 no stores either, 23 no step loop (load + final row), 63 load only.
"""
import sys

import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402
from gaussianprocessfundamentals_amd import engine  # noqa: E402
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk  # noqa: E402


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    dev = torch.device("cuda", 0)
    f = engine.AugmentedFactorization(n, 1, 0, batch)
    kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
    X = torch.sort(torch.rand(n, 1, dtype=torch.float64, device=dev), dim=0).values.contiguous()
    Y = torch.rand(1, n, dtype=torch.float64, device=dev)
    H = torch.full((batch, 1), 0.1, dtype=torch.float64, device=dev)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    nat.tune("lookahead", 0)
    for dbg in (0, 1, 2, 4, 7, 15, 23, 63):
        nat.tune("diag_debug", dbg)
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        nat.timing_reset()
        nat.timing_enable(True)
        for _ in range(3):
            f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        nat.timing_enable(False)
        t = nat.timing_read()
        print("diag_debug %d: " % dbg + "  ".join(
            "%s %.1f us x %d" % (c, t[c]["ms"] * 1e3 / max(1, t[c]["launches"]), t[c]["launches"] // 3)
            for c in ("diag", "trsm", "update")))
    nat.tune("diag_debug", 0)


if __name__ == "__main__":
    main()
