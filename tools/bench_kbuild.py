"""Kernel-matrix build (gpk_assemble into the augmented layout) on its own: time, HBM rate of the lower
tiles written, and element rate, for the SURVEY configs whose K build is not fused into the first
trailing update.

usage: python tools/bench_kbuild.py [case ...]   (cases: C5, C3, SE8192; default all)
C5: ADD(SE-ARD, PER standard) D=8, N=16384 fp64; C3: MAT52-ARD D=4, N=8192 fp32; SE8192: SE D=1, N=8192
fp64 batch 32 (the metric's inputs, built unfused).  Median of 10 launches, HIP events on the stream.
"""
import ctypes
import hashlib
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
import bench  # noqa: E402
from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402
from gaussianprocessfundamentals_amd import engine  # noqa: E402


def run(case):
    cfg = {"C5": ("C5", 1), "C3": ("C3", 1), "SE8192": ("metric", 32)}[case]
    name, batch = cfg
    kname, d, n, noise, dtn, hyp = bench.CONFIGS[name]
    dtype = torch.float32 if dtn == "f32" else torch.float64
    dev = torch.device("cuda", 0)
    kern = bench.build_kernel(kname, d)
    kd = engine.kernel_descriptor(kern, d)
    f = engine.AugmentedFactorization(n, d, 0, batch, dtype)
    lay = f.layout
    g = torch.Generator().manual_seed(7)
    X = torch.rand(n, d, generator=g, dtype=torch.float64).to(dev).contiguous()
    Y = torch.rand(1, n, generator=g, dtype=torch.float64).to(dev).contiguous()
    H = (0.3 + torch.rand(batch, kd.n_hyp, generator=g, dtype=torch.float64)).to(dev).contiguous()
    NZ = torch.tensor([noise], dtype=torch.float64, device=dev)
    L = nat.lib()
    s = nat.stream_handle(dev)

    def asm():
        nat.check(L.gpk_assemble(ctypes.byref(kd), ctypes.byref(lay), nat.ptr(H), kd.n_hyp, nat.ptr(NZ), 0,
                                 nat.ptr(X), 0, None, 0, None, 0, nat.ptr(Y), 0, nat.ptr(f.W), s), "gpk_assemble")

    for _ in range(3):
        asm()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        asm()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = statistics.median(ts)
    w0 = f.w(0)
    digest = hashlib.sha256(torch.tril(w0[:lay.p, :lay.p]).cpu().numpy().tobytes()).hexdigest()[:16]
    es = 4 if dtype == torch.float32 else 8
    lower = batch * lay.p * (lay.p + 64) / 2
    return {"case": case, "n": n, "d": d, "batch": batch, "kernel": kname, "dtype": dtn, "ms": round(ms, 3),
            "GBps_lower_tiles": round(lower * es / (ms * 1e-3) / 1e9, 1),
            "Gelem_per_s": round(batch * n * (n + 1) / 2 / (ms * 1e-3) / 1e9, 2), "w0": digest}


if __name__ == "__main__":
    for c in sys.argv[1:] or ["C5", "C3", "SE8192"]:
        print(json.dumps(run(c)), flush=True)
