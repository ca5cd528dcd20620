"""Phase timeline of the persistent factorisation's D tasks (a GPK_DIAG_PROF=1 build of libgpk, GPK_LIB):
per step s of the 128 x 128 diagonal body and per wave, the shader-clock cycles of P_s work, the wait at its
barrier, QR_s work and its barrier, averaged over the blocks.  usage: GPK_LIB=variants/libgpk_dprof.so
python tools/diag_phase_prof.py n"""
import ctypes
import os
import sys

os.environ["GPK_CHAIN_TIMES"] = "1"
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402
from gaussianprocessfundamentals_amd import engine  # noqa: E402
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
nat.tune("chain", 2)
dev = torch.device("cuda", 0)
kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
X = torch.sort(torch.rand(n, 1, dtype=torch.float64, device=dev), dim=0).values.contiguous()
Y = torch.rand(1, n, dtype=torch.float64, device=dev)
H = torch.full((1, 1), 0.1, dtype=torch.float64, device=dev)
NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
f = engine.AugmentedFactorization(n, 1, 0, 1)
for _ in range(3):
    f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
torch.cuda.synchronize()
lay = f.layout
nblk = lay.n_pad // 128
tasks = nat.chain_plan(lay.n_pad, lay.y_row, torch.cuda.get_device_properties(0).multi_processor_count)
nt = len(tasks)
tot = nt + nblk * 64
buf = (ctypes.c_uint64 * (6 * tot))()
rc = nat.load_library().gpk_chain_times(buf, tot)
assert rc == 0, rc
P = np.frombuffer(buf, dtype=np.uint64)[6 * nt:].reshape(nblk, 8, 8, 6).astype(np.float64)  # [k][s][wave][ph]
ks = range(2, nblk - 1)
print("n %d: D phases in shader cycles, mean over blocks %d..%d" % (n, 2, nblk - 2))
base = P[:, 0, :, 0].min(axis=1)   # first P_0 stamp per block
load = np.mean([P[k, 0, :, 5].max() - P[k, 0, :, 0].min() for k in ks])
print("P_0 start -> loaded (max wave): stamp order only; block end - P_0 start: %.0f cycles" %
      np.mean([P[k, 7, :, 4].max() - P[k, 0, :, 0].min() for k in ks]))
for s in range(8):
    pw = np.mean([P[k, s, :, 1] - P[k, s, :, 0] for k in ks], axis=0)     # P work per wave
    pb = np.mean([P[k, s, :, 2] - P[k, s, :, 1] for k in ks], axis=0)     # P barrier wait
    qw = np.mean([P[k, s, :, 3] - P[k, s, :, 2] for k in ks], axis=0)
    nxt = [(P[k, s + 1, :, 0] if s < 7 else P[k, 7, :, 4]) - P[k, s, :, 3] for k in ks]
    qb = np.mean(nxt, axis=0)
    step = np.mean([(P[k, s + 1, 0, 0] if s < 7 else P[k, 7, 0, 4]) - P[k, s, 0, 0] for k in ks])
    print("s %d step %5.0f | P work w0 %5.0f  w1-7 %s | P bar w0 %4.0f | QR work %s | QR bar+ w0 %4.0f" % (
        s, step, pw[0], " ".join("%4.0f" % v for v in pw[1:]), pb[0], " ".join("%4.0f" % v for v in qw), qb[0]))
print("waves 1-7, P work split (cycles, steps 1..6): inverse tile | trailing tiles | HBM stores of L / L^-1 rows")
for s in range(1, 7):
    inv = np.mean([P[k, s, 1:, 5] - P[k, s, 1:, 0] for k in ks], axis=0)
    trl = np.mean([P[k, s, 1:, 4] - P[k, s, 1:, 5] for k in ks], axis=0)
    sto = np.mean([P[k, s, 1:, 1] - P[k, s, 1:, 4] for k in ks], axis=0)
    print("s %d inv %s | trail %s | store %s" % (s, " ".join("%4.0f" % v for v in inv), " ".join("%4.0f" % v for v in trl),
                                                " ".join("%4.0f" % v for v in sto)))
