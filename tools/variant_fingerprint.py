"""Bitwise fingerprint of the factorisation under the library GPK_LIB points at, for A/B builds that
must not change results: prints one line per case with the hex of every member's -LML and a hash of the
whole augmented factor (W) of member 0.

usage: GPK_LIB=variants/libgpk_x.so python tools/variant_fingerprint.py
"""
import hashlib
import sys

import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402
from gaussianprocessfundamentals_amd import engine  # noqa: E402
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk  # noqa: E402


def case(n, m, batch, ingroup):
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(n + m + batch)
    X = torch.sort(torch.rand(n + m, 1, generator=g, dtype=torch.float64), dim=0).values.to(dev).contiguous()
    Y = torch.sin(12.0 * X[:n, 0]).reshape(1, n).contiguous()
    H = torch.linspace(0.05, 0.2, batch, dtype=torch.float64).reshape(batch, 1).to(dev)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
    nat.tune("ingroup", ingroup)
    f = engine.AugmentedFactorization(n, 1, m, batch)
    if m:
        f.run(kd, H, 1, NZ, 0, X[:n], 0, Y, 0, X[n:], 0)
    else:
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
    torch.cuda.synchronize()
    nl = [float(v).hex() for v in f.nlml().cpu()]
    h = hashlib.sha256(torch.tril(f.w(0)).cpu().numpy().tobytes()).hexdigest()[:16]
    nat.tune("ingroup", 0)
    return "n=%d m=%d batch=%d ingroup=%d w0=%s nlml=%s" % (n, m, batch, ingroup, h, ",".join(nl))


if __name__ == "__main__":
    for args in [(4096, 0, 8, 0), (8192, 0, 16, 3), (3000, 200, 4, 1), (2048, 0, 1, 2), (4096, 0, 1, 0),
                 (3000, 200, 2, 2), (1300, 0, 3, 2)]:
        print(case(*args), flush=True)
