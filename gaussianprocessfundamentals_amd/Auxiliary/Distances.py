"""Pairwise distances (gpbasics/Auxiliary/Distances.py:4-12) on the device (gpk_distance_matrix).

``euclidian_distance`` keeps the reference's expanded norm sqrt(|a|^2 - 2 a.b + |b|^2) without a
clamp, so it returns NaN exactly where rounding makes the argument negative (exact for
D = 1, NaN on parts of the diagonal for D > 1); ``manhattan_distance`` is the L1 sum.  Inputs are
[n, d] / [m, d] or batched [B, n, d] / [B, m, d] (a batch of 1 broadcasts, as TensorFlow's matmul
and broadcasting subtraction do); outputs [n, m] / [B, n, m] fp64 on the device.  The kernel
matrices never go through these: the kernel build evaluates its distances in registers.

Parity note: for D > 1 WHERE the expanded norm turns NaN is parity unpinned -- the reference ships
no fixture for it, and the rounding shape used here (norms from rounded squares, the cross term as
an FMA chain, the shape TensorFlow's reduce_sum / matmul are assumed to have) is this build's
restatement; only the D = 1 result (exact, no NaN) is guaranteed.  Callers that need finite
distances use ``euclidean_distance_direct``.
"""
from __future__ import annotations

import torch

from .. import _native as nat
from .. import engine

EXPANDED_EUCLIDEAN, MANHATTAN, EUCLIDEAN = 0, 1, 2


def _distance(a, b, mode: int) -> torch.Tensor:
    A, B = engine.as_device_f64(a), engine.as_device_f64(b)
    batched = A.dim() == 3 or B.dim() == 3
    A3 = A if A.dim() == 3 else A.reshape(1, A.shape[0], -1)
    B3 = B if B.dim() == 3 else B.reshape(1, B.shape[0], -1)
    if A3.shape[2] != B3.shape[2]:
        raise ValueError("inputs differ in their last dimension: %d vs %d" % (A3.shape[2], B3.shape[2]))
    batch = max(A3.shape[0], B3.shape[0])
    if A3.shape[0] not in (1, batch) or B3.shape[0] not in (1, batch):
        raise ValueError("batch sizes %d and %d do not broadcast" % (A3.shape[0], B3.shape[0]))
    A3, B3 = A3.contiguous(), B3.contiguous()
    n, m, d = int(A3.shape[1]), int(B3.shape[1]), int(A3.shape[2])
    out = torch.empty((batch, n, m), dtype=torch.float64, device=A3.device)
    nat.check(nat.lib().gpk_distance_matrix(mode, nat.ptr(A3), n, n * d if A3.shape[0] > 1 else 0, nat.ptr(B3), m,
                                            m * d if B3.shape[0] > 1 else 0, d, batch, nat.ptr(out), m, n * m,
                                            nat.stream_handle(A3.device)), "gpk_distance_matrix")
    return out if batched else out[0]


def euclidian_distance(a, b) -> torch.Tensor:
    """sqrt(rowsum(a^2) - 2 a b^T + rowsum(b^2)^T), unclamped (Distances.py:4-7)."""
    return _distance(a, b, EXPANDED_EUCLIDEAN)


def manhattan_distance(a, b) -> torch.Tensor:
    """sum_d |a_d - b_d| (Distances.py:10-12)."""
    return _distance(a, b, MANHATTAN)


def euclidean_distance_direct(a, b) -> torch.Tensor:
    """sqrt(sum_d (a_d - b_d)^2): the Euclidean distance without the expanded norm's cancellation."""
    return _distance(a, b, EUCLIDEAN)
