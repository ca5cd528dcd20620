"""Sharded hyperparameter sweeps: the multi-GPU form of the LML hot path.

The reference evaluates independent likelihoods in Python loops (k-fold lists,
gpbasics/Optimizer/Fitter.py:27-33 / :97-98; blockwise sub-GPs,
gpbasics/Metrics/LogLikelihood.py:85-104; any user sweep).  Here one process per GPU takes a
contiguous slice of the candidate list, evaluates the slice as ONE batched factorisation
(every launch of gpk_potrf_aug factors all of its members), and a single all-gather of
(nlml, info) pairs -- 16 bytes per candidate over RCCL/xGMI -- gives every rank the full result.
X and y are replicated (each rank holds its own copy); there is no other collective.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

from . import engine
from . import global_parameters as gp


def shard_range(n_items: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous balanced slice [start, stop) of n_items for rank (the first n % world ranks
    take one extra item)."""
    if world <= 0 or rank < 0 or rank >= world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def native_batched_evaluator(kernel, X: torch.Tensor, y: torch.Tensor, noise, dtype=None,
                             max_batch: Optional[int] = None,
                             pipeline: int = 1) -> Callable[[torch.Tensor], torch.Tensor]:
    """Evaluator running gpk_assemble/gpk_potrf_aug/gpk_finalize over candidate batches.

    Candidates are factored in chunks of ``max_batch`` (all at once when None).  With
    ``pipeline`` = P > 1 the chunks rotate over P factorisation buffers on P HIP streams, so one
    chunk's exposed panel chain overlaps the next chunk's trailing updates (the panel look-ahead
    is then left to the pipelining: each chunk runs its kernels on its own stream).  The result is
    ordered on the caller's stream.

    Returns f(cands [c, n_hyp] fp64) -> [c, 2] fp64 device tensor of (nlml, info)."""
    X = engine.as_device_f64(X)
    yv = engine.as_device_f64(y).reshape(1, -1).contiguous()
    n, d = int(X.shape[0]), int(X.shape[1])
    kd = engine.kernel_descriptor(kernel, d)
    from .Statistics.CovarianceMatrix import noise_vector
    nv = noise_vector(noise)
    dt = dtype or gp.p_dtype
    cache = {}
    P = max(1, int(pipeline))
    streams = [torch.cuda.Stream(X.device) for _ in range(P - 1)] if P > 1 else []

    def evaluate(cands: torch.Tensor) -> torch.Tensor:
        cands = cands.to(device=X.device, dtype=torch.float64).contiguous()
        c = int(cands.shape[0])
        out = torch.empty((c, 2), dtype=torch.float64, device=X.device)
        if c == 0:
            return out
        if cands.shape[1] != kd.n_hyp:
            raise ValueError("candidate rows must have %d hyperparameter values" % kd.n_hyp)
        step = c if max_batch is None else max(1, int(max_batch))
        caller = torch.cuda.current_stream(X.device)
        slots = [caller] + streams
        for st in streams:
            st.wait_stream(caller)
        # the chunks' factorisations overlap on P streams: no look-ahead side streams, no panel solve fused
        # into the diagonal-block launch (its redundant workgroups would take CUs from the other chunks'
        # updates: C5 38.2 -> 36.4 evals/s at 3 in flight) and no persistent launch (it would claim every
        # CU) -- pinned for this thread's calls only (gpk_tune_thread), not for other threads
        from . import _native as nat
        knobs = nat.thread_tune(lookahead=0, fuse_trsm=0, chain=0) if P > 1 else nat.thread_tune()
        with knobs:
            for i, s0 in enumerate(range(0, c, step)):
                s1 = min(c, s0 + step)
                b = s1 - s0
                slot = i % P
                f = cache.get((b, slot))
                if f is None:
                    f = engine.AugmentedFactorization(n, d, 0, b, dt)
                    cache[(b, slot)] = f
                with torch.cuda.stream(slots[slot]):
                    f.run(kd, cands[s0:s1], kd.n_hyp, nv, 0, X, 0, yv, 0)
                    out[s0:s1, 0] = f.nlml()
                    out[s0:s1, 1] = f.info.to(torch.float64)
        for st in streams:
            caller.wait_stream(st)
        return out

    return evaluate


class HyperparameterSweep:
    """Evaluate -LML for every row of a candidate matrix across the ranks of ``group``.

    ``evaluator(cands [c, n_hyp]) -> [c, 2]`` (nlml, info); by default the native batched
    device evaluator.  Works with world size 1 and without an initialised process group."""

    def __init__(self, evaluator: Callable[[torch.Tensor], torch.Tensor], group=None,
                 comm_device: Optional[torch.device] = None):
        self.evaluator = evaluator
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.world = dist.get_world_size(group) if self.distributed else 1
        if comm_device is None:
            backend = dist.get_backend(group) if self.distributed else "none"
            comm_device = engine.device() if backend == "nccl" else torch.device("cpu")
        self.comm_device = comm_device

    def local_slice(self, n_candidates: int) -> Tuple[int, int]:
        return shard_range(n_candidates, self.rank, self.world)

    def run(self, candidates: torch.Tensor):
        """Returns (nlml [C], info [C] int32, argmin index) on every rank."""
        C = int(candidates.shape[0])
        s0, s1 = self.local_slice(C)
        local = self.evaluator(candidates[s0:s1])
        if not self.distributed or self.world == 1:
            allv = local.to(self.comm_device)
        else:
            chunk = -(-C // self.world)
            buf = torch.full((chunk, 2), float("nan"), dtype=torch.float64, device=self.comm_device)
            buf[:s1 - s0] = local.to(self.comm_device)
            gathered = torch.empty((self.world * chunk, 2), dtype=torch.float64, device=self.comm_device)
            dist.all_gather_into_tensor(gathered, buf, group=self.group)
            parts = []
            for r in range(self.world):
                a, b = shard_range(C, r, self.world)
                parts.append(gathered[r * chunk:r * chunk + (b - a)])
            allv = torch.cat(parts, dim=0)
        nlml = allv[:, 0]
        info = allv[:, 1].to(torch.int32)
        masked = torch.where(info == 0, nlml, torch.full_like(nlml, float("inf")))
        best = int(torch.argmin(masked).item()) if C else -1
        return nlml, info, best
