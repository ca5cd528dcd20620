"""Device write / copy ceilings of this MI355X for the K build's roofline: torch fill_ (write only) and copy_
(read + write) on 1 GiB f64 buffers, and a strided fill of the lower-triangle-sized region of an N x N matrix by
64-row tiles (the K build's store pattern: 64 rows x 512 B per tile).  Median of 20, HIP events.

usage: python tools/probe/write_ceiling.py
"""
import json
import statistics

import torch


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts) * 1e-3


def main():
    dev = torch.device("cuda", 0)
    n = 1 << 27  # 1 GiB of f64
    a = torch.empty(n, dtype=torch.float64, device=dev)
    b = torch.empty(n, dtype=torch.float64, device=dev)
    t = timed(lambda: a.fill_(1.0))
    print(json.dumps({"op": "fill_", "bytes": 8 * n, "s": t, "GBps": round(8 * n / t / 1e9, 1)}), flush=True)
    t = timed(lambda: b.copy_(a))
    print(json.dumps({"op": "copy_", "bytes": 16 * n, "s": t, "GBps": round(16 * n / t / 1e9, 1)}), flush=True)
    N = 16384
    W = torch.empty(N, N + 64, dtype=torch.float64, device=dev)
    t = timed(lambda: W.fill_(0.5))
    by = 8 * N * (N + 64)
    print(json.dumps({"op": "fill_ W 16384 x 16448", "bytes": by, "s": t, "GBps": round(by / t / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
