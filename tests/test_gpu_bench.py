"""bench.py's multi-GPU code path at world size 1 (`--dist`: RCCL process group, per-step
all-gather of every rank's (nlml, info), barriers, MAX over ranks) and its JSON contract, run as a
child process at small N.  The reported nlml of the first candidate is checked against the oracle
(rel <= 1e-9, the C2 tolerance of SURVEY §8d)."""
import json
import os
import subprocess
import sys

import pytest

from oracle import gp_oracle as o

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, timeout=100):
    env = dict(os.environ)
    env.setdefault("MASTER_PORT", "29563")
    cp = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                        capture_output=True, text=True, timeout=timeout)
    assert cp.returncode == 0, cp.stdout[-2000:] + cp.stderr[-4000:]
    lines = [l for l in cp.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, cp.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_dist_rehearsal_metric():
    n = 1024
    d = run_bench("--dist", "--n", str(n), "--batch", "4", "--steps", "2", "--warmup", "1",
                  "--roofline-steps", "1", "--no-cpu-baseline")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["scaling"] == "weak" and d["dtype"] == "f64"
    assert d["value"] > 0 and d["config"]["batches_in_flight"] == 2  # bench.DEFAULT_PIPELINE_METRIC
    assert d["check"]["info"] == 0 and d["check"]["allgather_ok"] is True
    r = d["roofline"]
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s" and 0 < r["frac"] < 1.0
    x, y = o.make_inputs("metric", n=n)
    exp = o.nlml(("SE", {}), [0.1], 1e-2, x, y)
    assert abs(d["check"]["nlml"] - exp) <= 1e-9 * abs(exp)
    assert d["check"]["rel_vs_oracle"] <= 1e-9


def test_bench_dist_rehearsal_sweep():
    d = run_bench("--dist", "--config", "C4", "--n", "512", "--steps", "1", "--warmup", "1",
                  "--roofline-steps", "1", "--no-cpu-baseline")
    assert d["scaling"] == "strong" and d["config"]["candidates_per_rank_step"] == 128
    assert d["check"]["info"] == 0 and d["check"]["allgather_ok"] is True
    assert d["check"]["rel_vs_oracle"] <= 1e-9


def test_bench_headline_schedule_full_size_parity():
    """The exact headline schedule at full size -- N = 8192, 64 candidates per batch, 2 batches in flight,
    panel look-ahead off, panel solve unfused (bench.py defaults) -- with 4 spread candidates' -LML checked
    against the oracle inside the bench run (rel <= 1e-9, SURVEY §8d fp64 bar; M/LogLikelihood.py:30-65)."""
    d = run_bench("--steps", "1", "--warmup", "1", "--roofline-steps", "1", "--no-cpu-baseline",
                  "--check-candidates", "0,21,42,63", timeout=110)
    assert d["config"]["n"] == 8192 and d["config"]["candidates_per_rank_step"] == 64
    assert d["config"]["batches_in_flight"] == 2 and "look-ahead off" in d["config"]["schedule"]
    chk = d["check"]
    assert chk["info"] == 0 and [c["candidate"] for c in chk["candidates"]] == [0, 21, 42, 63]
    for c in chk["candidates"]:
        assert abs(c["hyp"][0] - 0.1 * (1.0 + 0.01 * c["candidate"])) < 1e-15
    assert chk["rel_vs_oracle"] <= 1e-9, chk


def test_bench_c4_slice_mode():
    """--slice-of W: rank 0's share of the W-way sharded C4 sweep on one GPU (the per-rank work of the
    W-GPU run), values checked against the oracle."""
    d = run_bench("--config", "C4", "--n", "1024", "--slice-of", "8", "--steps", "2", "--warmup", "1",
                  "--roofline-steps", "1", "--no-cpu-baseline")
    assert d["config"]["candidates_per_rank_step"] == 16 and d["slice"]["of_world"] == 8
    assert d["check"]["info"] == 0 and d["check"]["rel_vs_oracle"] <= 1e-9
