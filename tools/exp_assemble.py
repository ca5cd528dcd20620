"""Assemble-kernel timing experiment: gpk_assemble of the metric layout vs a plain fill of W.

usage: python tools/exp_assemble.py [batch] [n]
"""
import ctypes
import sys
import time

import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402
from gaussianprocessfundamentals_amd import engine  # noqa: E402
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    kname = sys.argv[3] if len(sys.argv) > 3 else "SE"
    dev = torch.device("cuda", 0)
    f = engine.AugmentedFactorization(n, 1, 0, batch)
    lay = f.layout
    kern = {"SE": bk.SquaredExponentialKernel, "MAT52": bk.MaternKernel5_2, "PER": bk.PeriodicKernel}[kname](1)
    kd = engine.kernel_descriptor(kern, 1)
    X = torch.rand(n, 1, dtype=torch.float64, device=dev)
    Y = torch.rand(1, n, dtype=torch.float64, device=dev)
    H = torch.full((batch, kd.n_hyp), 0.3, dtype=torch.float64, device=dev)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    L = nat.lib()
    s = nat.stream_handle(dev)

    def asm():
        nat.check(L.gpk_assemble(ctypes.byref(kd), ctypes.byref(lay), nat.ptr(H), kd.n_hyp, nat.ptr(NZ), 0, nat.ptr(X), 0,
                                 None, 0, None, 0, nat.ptr(Y), 0, nat.ptr(f.W), s), "asm")

    lower_bytes = batch * lay.p * (lay.p + 64) / 2 * 8
    t_asm = timeit(asm)
    t_fill = timeit(lambda: f.W.fill_(1.0))
    print("%s batch %d n %d p %d: assemble %.3f ms (%.0f GB/s of lower tiles); fill of all W %.3f ms (%.0f GB/s)"
          % (kname, batch, n, lay.p, t_asm, lower_bytes / t_asm / 1e6, t_fill, f.W.numel() * 8 / t_fill / 1e6))


if __name__ == "__main__":
    main()
