"""Accuracy study for emulating the fp64 trailing updates on the int8 MFMA (Ozaki scheme I).

usage: python tools/ozaki_study.py [n] [cfg]

A blocked right-looking Cholesky of the metric-style augmented matrix [K + noise I; y^T] (numpy, fp64)
whose trailing updates C -= P P^T are computed from int8 slices of P: every row of P is scaled by a
power of two so that its largest entry is < 1, then split into S slices of 7 bits
(P = sum_s 2^-7(s+1) P_s, P_s integer in [-127, 127]); the product keeps the slice pairs s + t < S, each
an exact int8 x int8 -> int32 GEMM (K <= 2^17 cannot overflow), accumulated in fp64.  Prints the
relative NLL error against the plain fp64 factorisation for S = 3 .. 8 and the int8 GEMM count
S (S + 1) / 2 per update.  CPU only; no device code involved.
"""
import math
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle import gp_oracle as o  # noqa: E402

NB = 128


def split_rows(P, S):
    """Row-scaled 7-bit slices: P = diag(sc) sum_s 2^-7(s+1) Q_s."""
    mx = np.max(np.abs(P), axis=1)
    e = np.where(mx > 0, np.ceil(np.log2(np.where(mx > 0, mx, 1.0))), 0.0)
    sc = np.exp2(e)
    R = P / sc[:, None]            # |R| <= 1
    slices = []
    for s in range(S):
        q = np.round(R * 2.0 ** (7 * (s + 1)))
        q = np.clip(q, -127, 127)
        slices.append(q)
        R = R - q * 2.0 ** (-7 * (s + 1))
    return sc, slices


def emulated_syrk(P, S):
    sc, sl = split_rows(P, S)
    out = np.zeros((P.shape[0], P.shape[0]))
    for s in range(S):
        for t in range(S - s):
            prod = sl[s] @ sl[t].T  # integer-valued: exact in fp64 BLAS while k 127^2 < 2^53 (int32 on the MFMA)
            out += prod * 2.0 ** (-7 * (s + t + 2))
    return out * np.outer(sc, sc)


def cholesky_nll(A, y, S=None, G=8):
    """-LML from a blocked right-looking factorisation of [A; y^T] with K = G NB trailing updates."""
    n = A.shape[0]
    W = np.zeros((n + 1, n + 1))
    W[:n, :n] = np.tril(A)
    W[n, :n] = y
    for g0 in range(0, n, G * NB):
        g1 = min(n, g0 + G * NB)
        # panel group: unblocked within (fp64), then one trailing update of everything below / right
        for j in range(g0, g1):
            W[j, j] = math.sqrt(W[j, j] - W[j, g0:j] @ W[j, g0:j])
            W[j + 1:, j] = (W[j + 1:, j] - W[j + 1:, g0:j] @ W[j, g0:j]) / W[j, j]
        P = W[g1:, g0:g1]
        if P.shape[0] == 0:
            continue
        upd = P @ P.T if S is None else emulated_syrk(P, S)
        W[g1:, g1:] -= np.tril(upd)
    logdet = 2.0 * np.sum(np.log(np.diag(W[:n, :n])))
    fit = float(W[n, :n] @ W[n, :n])
    return 0.5 * fit + 0.5 * logdet + 0.5 * n * math.log(2 * math.pi)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    cfg = sys.argv[2] if len(sys.argv) > 2 else "metric"
    x, y = o.make_inputs("C2" if cfg == "c2" else "metric", n)
    tree = ("SE", {"ard": False})
    K = o.k_noised(tree, [0.1], 1e-2, x)
    ref = cholesky_nll(K, y[:, 0] if y.ndim == 2 else y)
    print("n %d  fp64 NLL %.12f  (oracle %.12f)" % (n, ref, o.nlml(tree, [0.1], 1e-2, x, y)))
    for S in range(3, 9):
        got = cholesky_nll(K, y[:, 0] if y.ndim == 2 else y, S=S)
        print("S = %d  int8 GEMMs per update %2d  NLL rel err %.3e" % (S, S * (S + 1) // 2, abs(got - ref) / abs(ref)))


if __name__ == "__main__":
    main()
