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
tyraw = tasks[:, 0].copy()
gsz = ((tyraw >> 2) & 15) + 1   # BLK over g panels
tasks = tasks.copy()
tasks[:, 0] &= 3
nt = len(tasks)
buf = (ctypes.c_uint64 * (6 * nt))()
rc = nat.load_library().gpk_chain_times(buf, nt)
Traw = np.frombuffer(buf, dtype=np.uint64).reshape(nt, 6).astype(np.float64)
T = Traw / 100.0  # us
t0 = T[:, 0].min()
T[:, :4] -= t0
T[:, 4:] = np.where((T[:, 4:] > 0) & (tasks[:, :1] != 0) & (tasks[:, :1] != 3), T[:, 4:] - t0, np.nan)
print("rc", rc, "tasks", nt, "span %.1f us" % (T[:, 3].max()), flush=True)
names = ["D", "S", "U32", "BLK"]
for ty in range(4):
    m = tasks[:, 0] == ty
    if m.any():
        w = T[m, 1] - T[m, 0]
        r = T[m, 3] - T[m, 1]
        b = T[m, 2] - T[m, 1]
        print("%-4s n %5d  wait mean %.1f  run mean %.1f  min %.1f  max %.1f us (wave 0 body %.1f, drain + barrier %.1f)" % (
            names[ty], m.sum(), w.mean(), r.mean(), r.min(), r.max(), b.mean(), (r - b).mean()), flush=True)
        if ty == 3:
            for gv in sorted(set(gsz[m].tolist())):
                mm = m & (gsz == gv)
                print("     g=%d: n %d run mean %.1f us = %.1f GF/s per CU" % (
                    gv, mm.sum(), (T[mm, 3] - T[mm, 1]).mean(), 2 * 128 ** 3 * gv / ((T[mm, 3] - T[mm, 1]).mean() * 1e3)),
                    flush=True)
        if ty in (1, 2):
            print("     wave 0: operands in place %.1f, MFMAs retired %.1f, body done %.1f us after ready" % (
                np.nanmean(T[m, 4] - T[m, 1]), np.nanmean(T[m, 5] - T[m, 1]), b.mean()), flush=True)
d = np.where(tasks[:, 0] == 0)[0]
print("D(k) ready / done (us):", [(int(tasks[i, 1]), round(T[i, 1], 1), round(T[i, 3], 1)) for i in d[:8]], flush=True)
gaps = np.diff(T[d, 3])
print("D done spacing mean %.1f us, first %s" % (gaps.mean(), np.round(gaps[:10], 1).tolist()), flush=True)
# for step 5: the chain tasks' ready/done
k = min(5, len(d) - 1)
for ty in (1, 2):
    m = (tasks[:, 0] == ty) & (tasks[:, 1] == k) & (tasks[:, 2] // 4 == k + 1)
    print(names[ty], "k=%d block k+1 slices: ready %s done %s" % (k, np.round(T[m, 1], 1).tolist(), np.round(T[m, 3], 1).tolist()))

# the critical chain of steps 4..9: D(k) run, hand-off to the first S of block k + 1, S run, hand-off to
# the U32 of those slices, U32 run, hand-off to D(k + 1)
idx = {tuple(t[:4]): i for i, t in enumerate(tasks.tolist())}
for k in range(4, min(10, len(d) - 1)):
    i_d, i_d1 = d[k], d[k + 1]
    sl = [idx.get((1, k, s, 0)) for s in range(4 * (k + 1), 4 * (k + 1) + 4)]
    ul = [idx.get((2, k, s, k + 1)) for s in range(4 * (k + 1), 4 * (k + 1) + 4)]
    if None in sl or None in ul:
        continue
    s_rdy, s_done = max(T[sl, 1]), max(T[sl, 3])
    u_rdy, u_done = max(T[ul, 1]), max(T[ul, 3])
    print("step %d: D %.1f | ->S %.1f | S %.1f | ->U %.1f | U %.1f | ->D %.1f  (total %.1f)" % (
        k, T[i_d, 3] - T[i_d, 1], s_rdy - T[i_d, 3], s_done - s_rdy, u_rdy - s_done, u_done - u_rdy,
        T[i_d1, 1] - u_done, T[i_d1, 1] - T[i_d, 1]), flush=True)

# effective shader clock over the D and BLK bodies (s_memtime cycles / s_memrealtime at 100 MHz)
for ty in (0, 3):
    m = tasks[:, 0] == ty
    cyc = Traw[m, 5] - Traw[m, 4]
    us = (Traw[m, 2] - Traw[m, 1]) / 100.0
    ok = (cyc > 0) & (us > 0)
    print("%s body: shader clock %.2f GHz (median over %d tasks)" % (names[ty], np.median(cyc[ok] / us[ok]) / 1e3, ok.sum()), flush=True)

# every step: the hand-off gaps of the chain and how much of each is a late claim (the task's ticket was drawn
# only after its inputs were published: its workgroup was still busy with an earlier task)
rows = []
for k in range(1, len(d) - 1):
    i_d, i_d1 = d[k], d[k + 1]
    sl = [i for i in range(nt) if tasks[i, 0] == 1 and tasks[i, 1] == k and tasks[i, 2] // 4 == k + 1]
    ul = [i for i in range(nt) if tasks[i, 0] == 2 and tasks[i, 1] == k and tasks[i, 2] // 4 == k + 1]
    if not sl or not ul:
        continue
    d_done = T[i_d, 3]
    s_rdy, s_done = max(T[sl, 1]), max(T[sl, 3])
    u_rdy, u_done = max(T[ul, 1]), max(T[ul, 3])
    late_s = max(0.0, max(T[sl, 0]) - d_done)
    late_u = max(0.0, max(T[ul, 0]) - s_done)
    late_d = max(0.0, T[i_d1, 0] - u_done)
    rows.append((T[i_d, 3] - T[i_d, 1], s_rdy - d_done, late_s, s_done - s_rdy, u_rdy - s_done, late_u,
                 u_done - u_rdy, T[i_d1, 1] - u_done, late_d, T[i_d1, 1] - T[i_d, 1]))
if rows:
    r = np.array(rows).mean(axis=0)
    print("mean over %d steps: D %.1f | ->S %.1f (late claim %.1f) | S %.1f | ->U %.1f (late %.1f) | U %.1f | "
          "->D %.1f (late %.1f) | step %.1f us" % ((len(rows),) + tuple(r)), flush=True)

# chain_uq 2 (SQ tasks: S type with bit 7): D(k) | -> SQ ready | SQ run | -> D(k + 1) ready
sqm = ((tyraw & 3) == 1) & (((tyraw >> 7) & 1) == 1)
if sqm.any():
    rows = []
    for k in range(1, len(d) - 1):
        i_d, i_d1 = d[k], d[k + 1]
        sl = np.where(sqm & (tasks[:, 1] == k))[0]
        if len(sl) == 0:
            continue
        s_rdy, s_done = max(T[sl, 1]), max(T[sl, 3])
        rows.append((T[i_d, 3] - T[i_d, 1], s_rdy - T[i_d, 3], s_done - s_rdy, T[i_d1, 1] - s_done,
                     max(0.0, T[i_d1, 0] - s_done), T[i_d1, 1] - T[i_d, 1]))
    r = np.array(rows).mean(axis=0)
    print("SQ mean over %d steps: D %.1f | ->SQ %.1f | SQ %.1f | ->D %.1f (late %.1f) | step %.1f us" % (
        (len(rows),) + tuple(r)), flush=True)
