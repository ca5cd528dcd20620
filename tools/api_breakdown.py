import sys, time, statistics
import numpy as np, torch
sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp
gp.init(0)
from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd.Statistics.CovarianceMatrix import noise_vector
from gaussianprocessfundamentals_amd.KernelBasics.BaseKernels import SquaredExponentialKernel
for n in (1024, 4096):
    rng = np.random.default_rng(1)
    x = torch.tensor(np.sort(rng.uniform(0, 1, n)).reshape(n, 1), device="cuda")
    y = torch.tensor(np.sin(4 * np.pi * x.cpu().numpy()[:, 0]), device="cuda").reshape(1, n).contiguous()
    k = SquaredExponentialKernel(1)
    f = engine.AugmentedFactorization(n, 1, 0, 1)
    res = {"kd": [], "hyp": [], "noise": [], "run": [], "sync": [], "total": []}
    for i in range(30):
        t0 = time.perf_counter()
        kd = engine.kernel_descriptor(k, 1); t1 = time.perf_counter()
        hyp = engine.pack_hyper_parameter([torch.tensor(0.1 + 0.001 * i, dtype=torch.float64)], kd.n_hyp); t2 = time.perf_counter()
        nz = noise_vector(torch.tensor(1e-2, dtype=torch.float64)); t3 = time.perf_counter()
        f.run(kd, hyp, 0, nz, 0, x, 0, y, 0); t4 = time.perf_counter()
        v = float(f.nlml()[0]); t5 = time.perf_counter()
        if i >= 5:
            for key, a, b in (("kd", t0, t1), ("hyp", t1, t2), ("noise", t2, t3), ("run", t3, t4), ("sync", t4, t5), ("total", t0, t5)):
                res[key].append((b - a) * 1e3)
    print(n, {k_: round(statistics.median(v_), 4) for k_, v_ in res.items()})
