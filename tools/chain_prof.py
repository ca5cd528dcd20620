"""Per-task timing of one persistent factorisation (GPK_CHAIN_TIMES=1): for each task type the mean wait
(claimed -> inputs ready) and run (ready -> published) time, the critical chain D(k) -> D(k+1) spacing, and
the span.  usage: python tools/chain_prof.py n [grid]"""
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
grid = int(sys.argv[2]) if len(sys.argv) > 2 else 0
nat.tune("chain", 1)
nat.tune("chain_grid", grid)
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
tasks = nat.chain_plan(lay.n_pad, lay.y_row, grid if grid > 0 else torch.cuda.get_device_properties(0).multi_processor_count)
nt = len(tasks)
buf = (ctypes.c_uint64 * (3 * nt))()
rc = nat.load_library().gpk_chain_times(buf, nt)
T = np.frombuffer(buf, dtype=np.uint64).reshape(nt, 3).astype(np.float64) / 100.0  # us
t0 = T[:, 0].min()
T -= t0
print("rc", rc, "tasks", nt, "span %.1f us" % (T[:, 2].max()), flush=True)
names = ["D", "S", "U32", "BLK"]
for ty in range(4):
    m = tasks[:, 0] == ty
    if m.any():
        w = T[m, 1] - T[m, 0]
        r = T[m, 2] - T[m, 1]
        print("%-4s n %5d  wait mean %.1f  run mean %.1f  min %.1f  max %.1f us" % (names[ty], m.sum(), w.mean(), r.mean(),
                                                                             r.min(), r.max()), flush=True)
d = np.where(tasks[:, 0] == 0)[0]
print("D(k) ready / done (us):", [(int(tasks[i, 1]), round(T[i, 1], 1), round(T[i, 2], 1)) for i in d[:8]], flush=True)
gaps = np.diff(T[d, 2])
print("D done spacing mean %.1f us, first %s" % (gaps.mean(), np.round(gaps[:10], 1).tolist()), flush=True)
# for step 5: the chain tasks' ready/done
k = min(5, len(d) - 1)
for ty in (1, 2):
    m = (tasks[:, 0] == ty) & (tasks[:, 1] == k) & (tasks[:, 2] // 4 == k + 1)
    print(names[ty], "k=%d block k+1 slices: ready %s done %s" % (k, np.round(T[m, 1], 1).tolist(), np.round(T[m, 2], 1).tolist()))
