"""Where the workgroups of one persistent factorisation spend the launch (GPK_CHAIN_TIMES=1): per task type the
summed run time (inputs ready -> published) and wait time (claimed -> inputs ready) as fractions of grid x span,
the claim gaps, the tail after the last diagonal task, and the fraction of workgroups running a task in 10 time
bins.  usage: python tools/chain_util.py n [eye] [f32] [grid=G]   (eye: the identity-augmented value + gradient
factorisation; f32: chain_kernel<float>, whose plans take one slice-update task per slice; grid: workgroups)"""
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

n = int(sys.argv[1])
eye = "eye" in sys.argv[2:]
f32 = "f32" in sys.argv[2:]
nat.tune("chain", 2)
dev = torch.device("cuda", 0)
grid = torch.cuda.get_device_properties(0).multi_processor_count
for a in sys.argv[2:]:
    if a.startswith("grid="):
        grid = int(a[5:])
        nat.tune("chain_grid", grid)
dt = torch.float32 if f32 else torch.float64
kd = engine.kernel_descriptor(bk.SquaredExponentialKernel(1), 1)
X = torch.sort(torch.rand(n, 1, dtype=torch.float64, device=dev), dim=0).values.contiguous()
Y = torch.rand(1, n, dtype=torch.float64, device=dev)
H = torch.full((1, 1), 0.1, dtype=torch.float64, device=dev)
NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
f = engine.InverseFactorization(n, 1, 1, dt) if eye else engine.AugmentedFactorization(n, 1, 0, 1, dt)
for _ in range(3):
    f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
torch.cuda.synchronize()
lay = f.layout
tasks = nat.chain_plan(lay.n_pad, lay.y_row, grid, eye, f32).copy()
gsz = ((tasks[:, 0] >> 2) & 15) + 1
ty = tasks[:, 0] & 3
nt = len(tasks)
buf = (ctypes.c_uint64 * (6 * nt))()
rc = nat.load_library().gpk_chain_times(buf, nt)
T = np.frombuffer(buf, dtype=np.uint64).reshape(nt, 6).astype(np.float64)[:, :4] / 100.0
T -= T[:, 0].min()
span = T[:, 3].max()
names = ["D", "S", "U32", "BLK"]
print("rc %d n %d eye %d %s tasks %d grid %d span %.1f us" % (rc, n, eye, "f32" if f32 else "f64", nt, grid, span))
tot = grid * span
for t in range(4):
    m = ty == t
    if not m.any():
        continue
    run = (T[m, 3] - T[m, 1]).sum()
    wait = (T[m, 1] - T[m, 0]).sum()
    print("%-4s n %5d  run %5.1f %%  wait %5.1f %%  (run mean %.1f us)" % (names[t], m.sum(), 100 * run / tot,
                                                                        100 * wait / tot, (T[m, 3] - T[m, 1]).mean()))
    if t == 3:
        for g in sorted(set(gsz[m].tolist())):
            mm = m & (gsz == g)
            r = T[mm, 3] - T[mm, 1]
            print("     g=%2d: n %5d  run %5.1f %%  mean %.1f us = %.1f GF/s per CU" % (
                g, mm.sum(), 100 * r.sum() / tot, r.mean(), 2 * 128 ** 3 * g / (r.mean() * 1e3)))
# claim gaps: per workgroup, publish -> next claim is not measured per workgroup (the stamps are per task); the
# remainder of grid x span is time between tasks (claim latency, the drain of the list, the launch ramp)
busy = (T[:, 3] - T[:, 0]).sum()
print("between tasks / idle: %.1f %%" % (100 * (tot - busy) / tot))
d = np.where(ty == 0)[0]
print("last D done at %.1f us, tail %.1f us (%.1f %% of the span)" % (T[d, 3].max(), span - T[d, 3].max(),
                                                                      100 * (span - T[d, 3].max()) / span))
edges = np.linspace(0, span, 11)
frac = []
for a, b in zip(edges[:-1], edges[1:]):
    ov = np.clip(np.minimum(T[:, 3], b) - np.maximum(T[:, 1], a), 0, None).sum()
    frac.append(ov / (grid * (b - a)))
print("running fraction by tenth of the span:", " ".join("%.2f" % v for v in frac))
