"""A/B of the persistent launch's two-list mode (gpk_tune "chain_xcd": the diagonal chain's D / S / UQ tasks claimed
first by workgroups of XCD 0) against the one-list default, through the drop-in API as tools/bench_api_latency.py
measures it (median of 20 calls of get_metric / get_metric_and_gradient, a host synchronisation after each),
alternating the modes twice per size.

usage: python tools/chain_xcd_ab.py [n ...]   (seats: GPK_CHAIN_XCD_SEATS, default 16)
"""
import json
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from bench_api_latency import run  # noqa: E402

from gaussianprocessfundamentals_amd import _native as nat  # noqa: E402

if __name__ == "__main__":
    ns = [int(a) for a in sys.argv[1:]] or [2048, 4096, 8192]
    for n in ns:
        for rep in range(2):
            for xcd in (0, 1):
                with nat.thread_tune(chain_xcd=xcd):
                    r = run(n, grad=True)
                r.update({"chain_xcd": xcd, "rep": rep})
                print(json.dumps(r), flush=True)
