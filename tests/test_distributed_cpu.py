"""The sharded sweep under torch.distributed with the gloo backend, world sizes 1, 2, 3 and 8 (CPU; SURVEY §4
plans 1-8): contiguous, uneven shards.

The per-rank evaluator here is the CPU oracle (test infrastructure), injected explicitly; the
product's default evaluator is the native batched device path (tested on the GPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import gp_oracle as o


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gaussianprocessfundamentals_amd.global_parameters as gp
    gp.init(0)
    from gaussianprocessfundamentals_amd.sweep import HyperparameterSweep
    x, y = o.make_inputs("C1", n=64, seed=1)
    calls = []

    def evaluator(c):
        calls.append(int(c.shape[0]))
        res = []
        for row in c.tolist():
            try:
                res.append([o.nlml(("SE", {}), [row[0]], 1e-2, x, y), 0.0])
            except np.linalg.LinAlgError:
                res.append([float("inf"), 1.0])
        return torch.tensor(res, dtype=torch.float64).reshape(-1, 2)

    cands = torch.tensor([[v] for v in np.geomspace(0.02, 0.5, 13)], dtype=torch.float64)
    sw = HyperparameterSweep(evaluator, comm_device=torch.device("cpu"))
    nlml, info, best = sw.run(cands)
    out_q.put((rank, nlml.tolist(), info.tolist(), best, calls))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_gloo_sweep_matches_serial(world):
    from gaussianprocessfundamentals_amd.sweep import shard_range
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    x, y = o.make_inputs("C1", n=64, seed=1)
    exp = [o.nlml(("SE", {}), [v], 1e-2, x, y) for v in np.geomspace(0.02, 0.5, 13)]
    for rank, nlml, info, best, calls in res:
        np.testing.assert_allclose(nlml, exp, rtol=1e-12)
        assert info == [0] * 13
        assert best == int(np.argmin(exp))
        a, b = shard_range(13, rank, world)
        assert calls == [b - a]   # contiguous shards: 7 + 6 at world 2, 5 + 4 + 4 at 3, 2 2 2 2 2 1 1 1 at 8
