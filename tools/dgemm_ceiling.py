"""Vendor f64 GEMM rate on this box (torch.matmul -> hipBLASLt / rocBLAS), as a practical ceiling
for the trailing update (a K = 1024 SYRK-shaped product of 8192-row panels).

usage: python tools/dgemm_ceiling.py
Prints one JSON line per shape: TF/s of C = A B (A m x k, B k x n, f64), batched and single.
"""
import json

import torch


def rate(b, m, n, k, reps=10):
    dev = torch.device("cuda", 0)
    a = torch.randn(b, m, k, dtype=torch.float64, device=dev)
    bt = torch.randn(b, k, n, dtype=torch.float64, device=dev)
    c = torch.empty(b, m, n, dtype=torch.float64, device=dev)
    for _ in range(3):
        torch.matmul(a, bt, out=c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.matmul(a, bt, out=c)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return {"batch": b, "m": m, "n": n, "k": k, "ms": round(ms, 3), "tflops": round(2.0 * b * m * n * k / (ms * 1e-3) / 1e12, 2)}


if __name__ == "__main__":
    for shape in [(1, 8192, 8192, 1024), (1, 16384, 16384, 1024), (1, 8192, 8192, 8192), (8, 8192, 8192, 1024),
                  (16, 4096, 4096, 1024)]:
        print(json.dumps(rate(*shape)), flush=True)
