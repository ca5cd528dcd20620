"""Debug: factor one 128 x 128 SPD block through libgpk and compare L / L^-1 with numpy."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
import gaussianprocessfundamentals_amd.global_parameters as gp
gp.init(0)
from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd.KernelBasics.BaseKernels import SquaredExponentialKernel
from oracle import gp_oracle as o

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
x, y = o.make_inputs("C1", n=n, seed=3)
fact = engine.AugmentedFactorization(n, 1, 0, 1, torch.float64)
kd = engine.kernel_descriptor(SquaredExponentialKernel(1), 1)
H = torch.tensor([0.1], dtype=torch.float64, device="cuda")
NZ = torch.tensor([1e-2], dtype=torch.float64, device="cuda")
X = torch.as_tensor(x, device="cuda").contiguous()
Y = torch.as_tensor(y, device="cuda").reshape(1, -1).contiguous()
fact.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
torch.cuda.synchronize()
print("info", fact.info.cpu().numpy())
W = fact.w(0).cpu().numpy()
K = o.k_noised(("SE", {}), [0.1], 1e-2, x)
Lref = np.linalg.cholesky(K)
L = np.tril(W[:n, :n])
err = np.abs(L - Lref)
print("max |L - Lref|", err.max())
bad = np.argwhere(err > 1e-8)
print("first bad entries", bad[:10])
Winv = fact.Winv.cpu().numpy()[:128 * 128].reshape(128, 128)
Linv = np.linalg.inv(Lref[:128, :128])
e2 = np.abs(np.tril(Winv) - Linv)
print("max |Winv - inv(L)| block 0", e2.max(), np.argwhere(e2 > 1e-6)[:10])
for t in range(8):
    blk = (slice(16 * t, 16 * t + 16),) * 2
    print("tile", t, "L err %.2e  Dinv err %.2e" % (err[blk].max(), e2[blk].max()))
