"""bench.py's launcher contract on the CPU (no GPU touched; gloo): `--gpus N` without a launcher starts N
ranks itself (torch.distributed.run, 127.0.0.1 rendezvous), and a launcher world size that disagrees with
--gpus is refused with a non-zero exit (the driver's N-GPU runs)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _line(cp):
    lines = [l for l in cp.stdout.splitlines() if l.startswith("{")]
    assert cp.returncode == 0 and len(lines) == 1, cp.stdout[-2000:] + cp.stderr[-2000:]
    return json.loads(lines[0])


def test_gpus_2_starts_two_ranks():
    d = _line(_run(["--gpus", "2", "--launch-dry"]))
    assert d["launch_dry"] and d["n_gpus"] == 2 and d["gpus_flag"] == 2
    assert d["ranks"] == [0, 1] and d["local_ranks"] == [0, 1] and d["distinct_pids"] == 2


def test_gpus_1_is_one_rank():
    d = _line(_run(["--launch-dry"]))
    assert d["n_gpus"] == 1 and d["ranks"] == [0]


def test_world_size_mismatch_exits_nonzero():
    cp = _run(["--gpus", "1", "--launch-dry"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert cp.returncode != 0 and "WORLD_SIZE=2" in cp.stderr
    cp = _run(["--gpus", "4", "--launch-dry"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert cp.returncode != 0


def test_slice_mode_needs_c4():
    cp = _run(["--slice-of", "8", "--launch-dry"])
    assert cp.returncode == 0  # the dry launcher ignores the workload
    cp = _run(["--slice-of", "8", "--config", "metric"])
    assert cp.returncode == 2 and "C4" in cp.stderr
