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


def linear_cg(matrix: torch.Tensor, vector: torch.Tensor, x: torch.Tensor, tape: list = None) -> torch.Tensor:
    """tape: if a list, one record (p_k, A p_k, r_k, r_{k+1}, alpha_k, beta_k) per iteration whose update was
    kept -- what tf.GradientTape records through the loop -- for linear_cg_backward."""
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
        if tape is not None:
            tape.append((p, Apk, r, r_next, alpha_k, beta))
        p = -r_next + beta * p                           # :70-71
        r = r_next
        k += 1
        first_run = False
        if k % (n / 4) == 0 and k > n:                   # :35-39
            logging.debug("Linear Conjugate Gradient cannot be determined. Amount of iterations exceeds n (=%i)." % n)
            break
    return x


def linear_cg_backward(matrix: torch.Tensor, tape: list, x_bar: torch.Tensor):
    """Reverse mode of linear_cg from x_0 = 0 through the recorded iterations: given the adjoint of the
    returned x, returns (P, Q) [n, iterations] with the adjoint of the matrix = Q P^T (the Ap_k = A p_k
    products are the loop's only use of the matrix; r_0 = A x_0 - b carries none for x_0 = 0).  Per iteration,
    in reverse: p_{k+1} = -r_{k+1} + beta p_k, beta = r_{k+1}^T r_{k+1} / r_k^T r_k, r_{k+1} = r_k + alpha Ap,
    x_{k+1} = x_k + alpha p_k, alpha = r_k^T r_k / p_k^T Ap; one GEMV per iteration (A^T = A)."""
    from .. import engine
    xb = x_bar.reshape(-1, 1).to(torch.float64)
    rb = torch.zeros_like(xb)        # adjoint of r_{k+1}
    pb = torch.zeros_like(xb)        # adjoint of p_{k+1}
    Ps, Qs = [], []
    for (p, Ap, r, r_next, a, beta) in reversed(tape):
        rr = torch.sum(r * r)
        rrn = torch.sum(r_next * r_next)
        pAp = torch.sum(p * Ap)
        # p_{k+1} = -r_{k+1} + beta p_k
        rb = rb - pb
        beta_b = torch.sum(pb * p)
        pkb = beta * pb
        # beta = rrn / rr
        rrn_b = beta_b / rr
        rr_b = -beta_b * rrn / (rr * rr)
        rb = rb + 2.0 * rrn_b * r_next
        # r_{k+1} = r_k + a Ap ; x_{k+1} = x_k + a p_k
        a_b = torch.sum(rb * Ap) + torch.sum(xb * p)
        Apb = a * rb
        pkb = pkb + a * xb
        # a = rr / pAp
        rr_b = rr_b + a_b / pAp
        pAp_b = -a_b * rr / (pAp * pAp)
        pkb = pkb + pAp_b * Ap
        Apb = Apb + pAp_b * p
        # Ap = A p_k
        Ps.append(p)
        Qs.append(Apb)
        pkb = pkb + engine.gemv(matrix, Apb.contiguous())
        # rr = r_k^T r_k ; r_k feeds r_{k+1} too
        rb = rb + 2.0 * rr_b * r
        pb = pkb
        # x_k's adjoint is x_{k+1}'s (x_{k+1} = x_k + ...)
    # p_0 = -r_0: r_0's adjoint gains -p_0's; r_0 = A x_0 - b with x_0 = 0 gives the matrix nothing
    if not Ps:
        z = torch.zeros((xb.shape[0], 0), dtype=torch.float64, device=xb.device)
        return z, z
    return torch.cat(Ps, dim=1).contiguous(), torch.cat(Qs, dim=1).contiguous()
