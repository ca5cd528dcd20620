"""get_metric_and_gradient alone (the reference fitter's value + gradient call, Optimizer/Fitter.py:155-158) for
rocprofv3: `calls` evaluations at N, a host synchronisation after each.  usage: python tools/grad_profile.py [n] [calls]"""
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from grad_knob_sweep import metric  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 20
m = metric(n)
noise = torch.tensor(1e-2, dtype=torch.float64)
ts = []
for i in range(calls):
    c = torch.tensor(0.08 + 0.002 * (i % 7), dtype=torch.float64)
    t0 = time.perf_counter()
    nl, grads, gn = m.get_metric_and_gradient([c], noise)
    float(nl)
    ts.append((time.perf_counter() - t0) * 1e3)
ts = sorted(ts[3:])
print("n %d get_metric_and_gradient median %.3f ms" % (n, ts[len(ts) // 2]))
