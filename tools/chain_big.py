"""Persistent factorisation above the default chain_max_p: -LML / L against the launch path at large n.
usage: python tools/chain_big.py n [n ...]"""
import sys

import numpy as np

sys.path.insert(0, ".")
import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)
from gaussianprocessfundamentals_amd import engine  # noqa: E402
from tests.test_gpu_chain import _lower, _run  # noqa: E402

print("old chain_max_p", engine.nat.tune("chain_max_p", 100000), flush=True)
for n in [int(a) for a in sys.argv[1:]]:
    fc, _ = _run(n, 0, 1)
    fl, _ = _run(n, 0, 0)
    a, b = _lower(fc), _lower(fl)
    print("n %d info %d/%d  L max rel diff %.2e  nlml %.15g vs %.15g (rel %.2e)" % (
        n, int(fc.info.cpu()[0]), int(fl.info.cpu()[0]), np.abs(a - b).max() / np.abs(b).max(),
        fc.out.cpu().numpy()[0], fl.out.cpu().numpy()[0],
        abs(fc.out.cpu().numpy()[0] / fl.out.cpu().numpy()[0] - 1)), flush=True)
