"""Linear conjugate gradients (gpbasics/Auxiliary/LinearConjugateGradients.py:9-71) on the device.

Same iteration and the same stopping rule as the reference: start from x, r_0 = A x - b,
p_0 = -r_0; continue while |max(r_k)| > 1e-2 (note: the reference takes the absolute value of the
MAXIMUM, not the maximum absolute value); stop early (returning the previous x) when an update
turns NaN; give up after more than n iterations (checked when k is a multiple of n / 4).  The
matrix-vector product of every iteration is the HBM-bound device GEMV (gpk_gemv); the O(n)
vector updates are device tensor operations.  The host reads one scalar per iteration (the
stopping test), as the reference's Python loop does.
"""
from __future__ import annotations

import logging

import torch

from .. import global_parameters as global_param

global_param.ensure_init()


def linear_cg(matrix: torch.Tensor, vector: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    from .. import engine
    n = int(matrix.shape[0])
    b = vector.reshape(-1, 1).to(torch.float64)
    x = x.reshape(-1, 1).to(torch.float64).clone()
    r = engine.gemv(matrix, x) - b                       # :11
    p = -r                                               # :12
    k = 0
    first_run = True
    while first_run or float(torch.abs(torch.max(r))) > 1e-2:   # :17
        Apk = engine.gemv(matrix, p)                     # get_Apk :44-45
        rr = torch.sum(r * r)
        alpha_k = rr / torch.sum(p * Apk)                # get_alpha_k :48-52
        next_x = x + alpha_k * p                         # :55-56
        if bool(torch.any(torch.isnan(next_x))):         # :21-22
            return x
        x = next_x
        r_next = r + alpha_k * Apk                       # :59-60
        beta = torch.sum(r_next * r_next) / rr           # :63-67
        p = -r_next + beta * p                           # :70-71
        r = r_next
        k += 1
        first_run = False
        if k % (n / 4) == 0 and k > n:                   # :35-39
            logging.debug("Linear Conjugate Gradient cannot be determined. Amount of iterations exceeds n (=%i)." % n)
            break
    return x
