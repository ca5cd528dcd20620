#!/usr/bin/env python3
"""Benchmark of the GP log-marginal-likelihood hot path on MI355X.

Metric (BASELINE.json): LML evaluations per second at N = 8192, fp64, SE kernel, D = 1
(SURVEY §8d "Metric" row).  One step = one full evaluation -- kernel-matrix build, blocked
Cholesky with the fused forward solve, read-out of -LML -- from inputs already resident in HBM.
With --gpus N (torchrun, one process per GPU) every rank evaluates its own hyperparameter
candidate per step (weak scaling) and the step ends with the sweep's one collective, an
all-gather of the per-rank (nlml, info) pairs over RCCL.

Prints ONE JSON line on rank 0 (fields per the driver contract) including
  roofline      the trailing-update MFMA kernel (the dominant one): algorithmic flops of the
                lower-triangular SYRK ÷ its HIP-event time over the timed region, vs the fp64
                (or fp32) MFMA peak
  cpu_baseline  the numpy/SciPy restatement of the reference path (oracle/) timed on this host
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK = {"f64": 78.6, "f32": 157.3}   # TFLOP/s dense MFMA (AMD MI355X spec; microarch guide for f32)
HBM_PEAK = 8000.0                      # GB/s spec
# candidates per rank per step on the metric config, and batches in flight there: 64 x 2 (128 candidates,
# 71 GB of augmented matrices of the 288 GB) measured 352.3 / 351.7 evals/s against 348.4 / 349.3 for 32 x 2
# and 350.9 / 351.4 for 48 x 2 (two alternating passes on one box, tools/batch_ab.sh); 16 x 3 337.8 --
# larger launches of the short trailing updates at the end of each factorisation
DEFAULT_BATCH = 64
# --mode grad (identity-augmented, p ~ 2N: 2.2 GB per candidate at N = 8192): 16 x 2 (70 GB), 106.3 / 106.3
# evals/s against 104.9 / 104.4 for 8 x 2 (two alternating passes on one box)
DEFAULT_BATCH_GRAD = 16
DEFAULT_PIPELINE_METRIC = 2
# the other configs (one candidate per step except C4): 4 buffers / streams -- C2 1091 -> 1289, C3 403 -> 436,
# C5 38.2 -> 38.7 evals/s against 3, C4 flat; 5, 6 and 8 measured slower than 4 on C2 (785, 924, 1135) with 4, 8
# or 16 hardware queues alike
DEFAULT_PIPELINE_OTHER = 4
# one f64 candidate per step where the persistent factorisation applies (C2, N <= 12288): 8 persistent launches in
# flight, each with a quarter of the CUs as its grid (chain_grid 64 of 256: four run at a time, the next ones start
# as CUs free up) -- 1695-1714 evals/s against 1343-1347 for the launch path at 4 in flight; 8 x 48 1594-1619,
# 8 x 56 / 80 / 96 / 128 1582 / 1614 / 1623 / 1562, 6 x 64 1707, 4 x 64 1549, 10 / 12 / 16 in flight collapse to
# ~850 (more streams than the 8 hardware queues), profiles/r05u_*, r05v_*, r05ac_*, r05ad_*.  (Before round 5
# every persistent run was verified with a host synchronisation inside run(), which serialised them: r04ae
# measured no overlap.)
PERSIST_PIPELINE = int(os.environ.get("GPK_BENCH_PERSIST_P", "8"))
PERSIST_CU_SHARE = 1.0 / float(os.environ.get("GPK_BENCH_PERSIST_SHARE", "4"))

CONFIGS = {
    # name: (kernel, d, n, noise, dtype, hyp)
    "metric": ("SE", 1, 8192, 1e-2, "f64", [0.1]),
    "C2": ("SE", 1, 4096, 1e-2, "f64", [0.1]),
    "C3": ("MAT52-ARD", 4, 8192, 1e-1, "f32", [[0.25, 0.5, 0.75, 1.0]]),
    # C4: the 128-candidate (lengthscale, signal variance) sweep, sharded over the ranks (strong
    # scaling: one step = the whole sweep, every rank factorises its slice as one batch)
    "C4": ("SE-SCALED", 1, 4096, 1e-2, "f64", None),
    "C5": ("SE-ARD+PER", 8, 16384, 1e-2, "f64", None),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="nlml", choices=["nlml", "grad"],
                    help="nlml: -LML only (the headline metric); grad: -LML + its gradient w.r.t. every "
                         "hyperparameter and the noise (identity-augmented factorisation + gradient pass)")
    ap.add_argument("--n", type=int, default=None, help="override N")
    ap.add_argument("--batch", type=int, default=None,
                    help="hyperparameter candidates factorised together per rank per step "
                         "(default: %d for the metric config, %d with --mode grad, 1 otherwise)"
                         % (DEFAULT_BATCH, DEFAULT_BATCH_GRAD))
    ap.add_argument("--pipeline", type=int, default=None,
                    help="factorisation buffers / streams that consecutive steps rotate over (overlap of batches); "
                         "default %d for the metric config, %d otherwise" % (DEFAULT_PIPELINE_METRIC, DEFAULT_PIPELINE_OTHER))
    ap.add_argument("--lookahead", type=int, default=None,
                    help="panel look-ahead on side streams: 1 on, 0 off, 2 auto (libgpk: off below 64 128-blocks "
                         "of the augmented matrix); default 2, 0 when --pipeline > 1")
    ap.add_argument("--fuse-trsm", type=int, default=None,
                    help="panel solve inside the diagonal-block launch (libgpk fuse_trsm); default 0 when "
                         "--pipeline > 1, else the library default (1)")
    ap.add_argument("--chain", type=int, default=None,
                    help="single-member factorisations as one persistent launch (libgpk chain); default 0 when "
                         "--pipeline > 1, else the library default")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-events", action="store_true", help="time without per-kernel HIP events")
    ap.add_argument("--roofline-steps", type=int, default=3, help="steps of the look-ahead-off roofline pass")
    ap.add_argument("--dist", action="store_true",
                    help="run the multi-GPU code path (RCCL process group, per-step all-gather, barriers, MAX "
                         "over ranks) even at world size 1: the rehearsal of the N > 1 bench on a 1-GPU box")
    ap.add_argument("--launch-dry", action="store_true",
                    help="launcher check without a GPU: every rank joins a gloo group, all-gathers its rank and "
                         "rank 0 prints the ranks it saw (no HIP call)")
    ap.add_argument("--slice-of", type=int, default=1, metavar="W",
                    help="C4 only: time on this GPU the slice rank 0 evaluates when the 128-candidate sweep is "
                         "sharded over W ranks (128 / W candidates per step) -- the per-rank work of the W-GPU run")
    ap.add_argument("--check-candidates", default=None,
                    help="comma-separated batch indices whose -LML is checked against the oracle after the "
                         "timed region (default: first, middle, last)")
    ap.add_argument("--no-check", action="store_true", help="skip the oracle check of the bench's own values")
    return ap.parse_args()


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: start N ranks, one process per GPU, through
    torch.distributed.run (127.0.0.1 rendezvous) as a child process -- nothing in this process has
    touched the GPU -- and return its exit code."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # the box supports dmabuf IPC only (RCCL)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def launch_dry(args):
    """Every rank: a gloo group, all-gather of (rank, local rank, pid); rank 0 prints them."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    mine = torch.tensor([rank, int(os.environ.get("LOCAL_RANK", "0")), os.getpid()], dtype=torch.int64)
    got = [torch.zeros_like(mine) for _ in range(world)]
    if world > 1:
        dist.all_gather(got, mine)
    else:
        got = [mine]
    if rank == 0:
        print(json.dumps({"launch_dry": True, "n_gpus": world, "gpus_flag": args.gpus,
                          "ranks": [int(g[0]) for g in got], "local_ranks": [int(g[1]) for g in got],
                          "distinct_pids": len({int(g[2]) for g in got})}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic(cfg, batch):
    """HBM bytes per update launch from the committed PMC pass (profiles/pmc_traffic.json:
    2 x FETCH_SIZE + WRITE_SIZE per the gfx950 corrections, averaged over the update dispatches of
    `tools/pmc_pass.sh` on the same config); None when no pass for this config is on file."""
    path = os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f).get("%s_b%d" % (cfg, batch))
    except (OSError, ValueError):
        return None
    return rec


def synthetic_inputs(cfg, n):
    """SURVEY §8(d) synthetic inputs (numpy default_rng): the generator the golden vectors and the oracle
    use (oracle.gp_oracle.make_inputs), restated here so that the measured path imports nothing from oracle/
    (only the cpu_baseline leg does)."""
    import numpy as np
    if cfg in ("C2", "C4", "metric"):
        seed = {"C2": 1, "C4": 3, "metric": 5}[cfg]
        rng = np.random.default_rng(seed)
        x = np.sort(rng.uniform(0.0, 1.0, n)).reshape(n, 1)
        return x, np.sin(4.0 * math.pi * x[:, 0]) + 0.1 * rng.standard_normal(n)
    d, seed = {"C3": (4, 2), "C5": (8, 4)}[cfg]
    rng = np.random.default_rng(seed)
    x = rng.uniform(0.0, 1.0, (n, d))
    return x, np.sum(np.sin(2.0 * math.pi * x), axis=1) + 0.1 * rng.standard_normal(n)


def c4_candidates():
    """lengthscale geomspace(0.02, 0.5, 16) x signal variance geomspace(0.25, 4, 8)
    (the grid of tests/golden/make_golden.py)."""
    import numpy as np
    return [[float(a), float(b)] for a in np.geomspace(0.02, 0.5, 16) for b in np.geomspace(0.25, 4.0, 8)]


def build_kernel(name, d):
    from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk
    from gaussianprocessfundamentals_amd.KernelBasics import Operators as ops
    if name in ("SE", "SE-SCALED"):
        return bk.SquaredExponentialKernel(d)
    if name == "MAT52-ARD":
        return bk.MaternKernel5_2(d, ard=True, standard=True)
    if name == "SE-ARD+PER":
        return ops.AdditionOperator(d, [bk.SquaredExponentialKernel(d, ard=True), bk.PeriodicKernel(d, standard=True)])
    raise ValueError(name)


def cpu_baseline_grad(cfg_name, n):
    """-LML + gradient by the autodiff oracle (torch CPU reverse mode through Cholesky), one warm
    evaluation on this host's threads."""
    import numpy as np
    import torch
    from oracle import gp_autodiff as ad
    from oracle import gp_oracle as o
    threads, _ = host_threads()
    torch.set_num_threads(threads)
    kname, d, _, noise, _, hyp = CONFIGS[cfg_name]
    tree = {"SE": ("SE", {}), "SE-SCALED": ("SE", {})}.get(kname)
    if tree is None or hyp is None:
        return None
    x, y = o.make_inputs("metric" if cfg_name == "metric" else cfg_name, n=n)
    ad.nlml_and_grad(tree, hyp, noise, x[:512], y[:512])  # warm
    t0 = time.perf_counter()
    ad.nlml_and_grad(tree, hyp, noise, x, y)
    t1 = time.perf_counter() - t0
    return {"value": 1.0 / t1, "unit": "LML+gradient evals/s", "cores": threads, "kind": "port",
            "sample": "one warm -LML + gradient evaluation of the %s workload (N=%d, fp64) by the autodiff "
                      "oracle (oracle/gp_autodiff.py: torch CPU reverse mode through cholesky / "
                      "triangular_solve, as tf.GradientTape in the reference), %d threads (%.1f s)"
                      % (cfg_name, n, threads, t1)}


def host_threads():
    """Host threads of the CPU baseline: the CPUs this process may run on (sched_getaffinity), capped
    by the cgroup CPU quota and by OMP_NUM_THREADS when either is set (the GPU box exposes the whole
    machine's CPUs but grants one GPU's share).  GPK_CPU_THREADS overrides.  Returns (threads, facts)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:  # cgroup v2
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = aff
    if quota:
        threads = min(threads, max(1, int(math.ceil(quota))))
    if omp and omp.isdigit() and int(omp) > 0:
        threads = min(threads, int(omp))
    if os.environ.get("GPK_CPU_THREADS"):
        threads = int(os.environ["GPK_CPU_THREADS"])
    return threads, {"sched_getaffinity": aff, "cgroup_cpu_quota": quota, "omp_num_threads": omp,
                     "os_cpu_count": os.cpu_count()}


def oracle_tree(kname):
    return {"SE": ("SE", {}), "SE-SCALED": ("SE", {}), "MAT52-ARD": ("MAT52", {"ard": True, "standard": True}),
            "SE-ARD+PER": ("ADD", [("SE", {"ard": True}), ("PER", {"standard": True})])}[kname]


def oracle_hyp(row, kname, d):
    """A flat device hyperparameter row -> the oracle's nested list (ARD length scales as one list)."""
    if kname == "MAT52-ARD":
        return [list(row[:d])]
    if kname == "SE-ARD+PER":
        return [list(row[:d])] + list(row[d:])
    return list(row)


def cpu_baseline(cfg_name, n, budget_s, row):
    """Time the oracle (numpy/SciPy restatement of the reference path, oracle/gp_oracle.nlml_stages) on
    this host for the device's candidate `row` (a flat hyperparameter row): K build on a thread pool
    (TF's intra-op pool spreads the reference's), dpotrf / 2 x dtrtrs through MKL (torch's CPU LAPACK --
    here faster than scipy's OpenBLAS build, so the stronger baseline), stage by stage, with all host
    threads and with one.  Returns (record, nlml of the evaluated candidate)."""
    from oracle import gp_oracle as o
    threads, facts = host_threads()
    kname, d, _, noise, _, _ = CONFIGS[cfg_name]
    tree = oracle_tree(kname)
    scaled = kname == "SE-SCALED"
    hyp = oracle_hyp(row, kname, d)
    x, y = o.make_inputs("metric" if cfg_name == "metric" else cfg_name, n=n)
    # median of >= 5 warm repetitions with the host threads, plus one 1-thread figure
    runs = []
    o.nlml_stages(tree, hyp, noise, x[:1024], y[:1024], threads, scaled)  # warm (pools, page-in)
    t_all = time.perf_counter()
    while len(runs) < 5 or (time.perf_counter() - t_all < budget_s and len(runs) < 9):
        runs.append(o.nlml_stages(tree, hyp, noise, x, y, threads, scaled))
        if time.perf_counter() - t_all > 3 * budget_s:
            break
    runs.sort(key=lambda r: r[1]["total"])
    nl, med = runs[len(runs) // 2]
    one = None
    if threads == 1:
        one = med
    elif med["total"] * min(threads, 16) < 2.0 * budget_s:
        one = o.nlml_stages(tree, hyp, noise, x, y, 1, scaled)[1]
    try:
        cpu_model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:  # noqa: BLE001
        cpu_model = "unknown"
    stages = {k: round(v, 4) for k, v in med.items()}
    rec = {"value": 1.0 / med["total"], "unit": "LML evals/s", "cores": threads, "kind": "port",
           "value_1_thread": (1.0 / one["total"]) if one else None,
           "stages_s": stages,
           "stages_s_1_thread": {k: round(v, 4) for k, v in one.items()} if one else None,
           "host": dict(facts, cpu_model=cpu_model, lapack="MKL (torch CPU) dpotrf / dtrtrs",
                        kbuild="numpy, row chunks of 256 on %d threads" % threads),
           "sample": "median of %d warm full evaluations of the %s workload (N=%d, fp64: K build, dpotrf, "
                     "2 x dtrtrs, read-out) by the oracle (oracle/gp_oracle.nlml_stages), %d threads = "
                     "min(sched_getaffinity %d, cgroup quota %s, OMP_NUM_THREADS %s), %s; plus one 1-thread "
                     "evaluation" % (len(runs), cfg_name, n, threads, facts["sched_getaffinity"],
                                     facts["cgroup_cpu_quota"], facts["omp_num_threads"], cpu_model)}
    return rec, nl


def oracle_check(cfg_name, n, rows, idx, kname, d, noise, got, known=None):
    """-LML of device candidates `idx` (rows of the hyperparameter batch) against the oracle on the
    same inputs (`known`: oracle values already computed, by candidate); returns the check record
    (bar: rel <= 1e-9, the fp64 tolerance of SURVEY §8d; fp32 C3: 1e-3)."""
    from oracle import gp_oracle as o
    threads, _ = host_threads()
    x, y = o.make_inputs("metric" if cfg_name == "metric" else cfg_name, n=n)
    tree = oracle_tree(kname)
    out = []
    for c in idx:
        if known and c in known:
            exp = known[c]
        else:
            exp, _ = o.nlml_stages(tree, oracle_hyp(rows[c], kname, d), noise, x, y, threads, kname == "SE-SCALED")
        out.append({"candidate": int(c), "hyp": [round(v, 12) for v in rows[c]], "nlml": got[c], "oracle": exp,
                    "rel": abs(got[c] - exp) / abs(exp)})
    return {"candidates": out, "rel_vs_oracle": max(r["rel"] for r in out)}


# Hardware queues per process: HIP multiplexes streams onto GPU_MAX_HW_QUEUES in-order hardware queues
# (4 by default). P pipelined factorisation streams + torch's default stream + the comm stream + RCCL's stream
# share them, and two streams sharing a queue serialise.  Measured with the RCCL path on (--dist, N = 8192,
# P = 3): 321.7 evals/s with 4 queues, 338.1 with 8 (P = 2: 302.1 / 329.5).  Round 6: C2 (8 persistent launches in
# flight) 1675 / 1706 evals/s with 8 / 16 queues, its --dist rehearsal 1430 / 1684, the metric 357.3 / 357.3
# (profiles/r06d_hw_queues.txt) -- 16.
HW_QUEUES = int(os.environ.get("GPK_BENCH_HW_QUEUES", "16"))  # 0: leave the runtime default


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) != args.gpus:
        sys.stderr.write("bench.py: --gpus %d but the launcher started WORLD_SIZE=%s ranks; refusing to report "
                         "a %d-GPU number from a %s-rank job\n" % (args.gpus, env_world, args.gpus, env_world))
        sys.exit(2)
    if env_world is None and args.gpus > 1:
        # no launcher: start the N ranks here, before anything touches the GPU
        sys.exit(launch_ranks(args.gpus))
    if args.launch_dry:
        launch_dry(args)
        return
    if args.slice_of != 1 and (args.config != "C4" or args.slice_of < 1 or args.gpus != 1):
        sys.stderr.write("bench.py: --slice-of W needs --config C4 on one GPU\n")
        sys.exit(2)
    # before the first HIP call of the process (torch initialises HIP lazily)
    if HW_QUEUES and int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < HW_QUEUES:
        os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if torch.cuda.device_count() < world:
        sys.stderr.write("bench.py: %d ranks but only %d GPUs visible\n" % (world, torch.cuda.device_count()))
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    use_dist = world > 1 or args.dist
    if use_dist:
        if world == 1:  # no launcher: a one-rank group of our own (127.0.0.1 rendezvous)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import gaussianprocessfundamentals_amd.global_parameters as gp
    gp.init(0)
    if CONFIGS[args.config][0] == "SE-SCALED":
        gp.p_scaled_base_kernel = True  # hyp = [lengthscale, signal variance]
    from gaussianprocessfundamentals_amd import _native as nat
    from gaussianprocessfundamentals_amd import engine

    kname, d, n, noise, dtn, hyp = CONFIGS[args.config]
    n = args.n or n
    if kname == "SE-SCALED":
        hyp = c4_candidates()[0]
    elif hyp is None:
        hyp = [[0.4 + 0.1 * i for i in range(d)], 1.0, 0.5]
    dt = torch.float64 if dtn == "f64" else torch.float32
    x, y = synthetic_inputs(args.config, n)
    dev = torch.device("cuda", local)
    X = torch.as_tensor(x, dtype=torch.float64, device=dev).contiguous()
    Y = torch.as_tensor(y, dtype=torch.float64, device=dev).reshape(1, n).contiguous()
    kernel = build_kernel(kname, d)
    kd = engine.kernel_descriptor(kernel, d)
    flat_h = []
    for h in hyp:
        flat_h.extend(h if isinstance(h, list) else [h])
    sweep = kname == "SE-SCALED"
    if sweep:
        # C4 (strong scaling): the 128 candidates are split contiguously over the ranks
        from gaussianprocessfundamentals_amd.sweep import shard_range
        cands = c4_candidates()
        # --slice-of W (one GPU): rank 0's slice of a W-way sharding, i.e. one rank's work in the W-GPU run
        shards = world if args.slice_of == 1 else args.slice_of
        s0, s1 = shard_range(len(cands), rank, shards)
        rows = cands[s0:s1]
        batch = len(rows)
        chunk = -(-len(cands) // shards)
    else:
        batch = args.batch or ((DEFAULT_BATCH_GRAD if args.mode == "grad" else DEFAULT_BATCH)
                               if args.config == "metric" else 1)
        chunk = batch
        # weak scaling: every rank evaluates its own `batch` candidates (a sweep over the first
        # hyperparameter: candidate c of rank r scales it by 1 + 0.01 (r * batch + c))
        rows = []
        for c in range(batch):
            h = list(flat_h)
            if not isinstance(hyp[0], list):
                h[0] = h[0] * (1.0 + 0.01 * (rank * batch + c))
            rows.append(h)
    H = torch.tensor(rows, dtype=torch.float64, device=dev).contiguous()
    NZ = torch.tensor([noise], dtype=torch.float64, device=dev)
    grad_mode = args.mode == "grad"
    # --pipeline P: P factorisation buffers on P streams, consecutive steps round-robin over them,
    # so that one batch's exposed panel chain (start and tail of the factorisation) overlaps the
    # trailing updates of the next (the batches are independent candidate sets of the sweep)
    # (f32 too since the block-row updates: C3 on 8 f32 persistent launches side by side 474.1-474.8 evals/s against
    # 472.4-472.8 for the f32 launch path at 4 in flight, profiles/r06s_defaults.txt; GPK_BENCH_PERSIST_F32=0 keeps
    # the launch path for f32)
    persist = (args.pipeline is None and args.chain is None and not grad_mode and not sweep and batch == 1 and
               (dtn == "f64" or os.environ.get("GPK_BENCH_PERSIST_F32", "1") == "1") and n <= 12288)
    P = max(1, args.pipeline if args.pipeline is not None else
            (DEFAULT_PIPELINE_METRIC if args.config == "metric" else
             PERSIST_PIPELINE if persist else DEFAULT_PIPELINE_OTHER))
    la = args.lookahead if args.lookahead is not None else (0 if P > 1 else 2)
    nat.tune("lookahead", la)
    # batches overlapping on P > 1 streams: the panel solve stays a separate launch (fused, its redundant
    # workgroups take CUs from the other batches' updates: C5 at 3 in flight 38.2 -> 36.4 evals/s)
    if args.fuse_trsm is not None or P > 1:
        nat.tune("fuse_trsm", args.fuse_trsm if args.fuse_trsm is not None else 0)
    # the persistent factorisation keeps one workgroup per CU for the whole evaluation: with P > 1
    # batches in flight the launch path's kernels share the chip better
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    chain_grid = 0
    if persist:
        # P persistent launches side by side, each claiming its share of the CUs (no launch waits for another's
        # workgroups: each one's tasks only ever wait for tasks claimed earlier in its own list)
        chain_grid = max(1, int(round(ncu * PERSIST_CU_SHARE)))
        nat.tune("chain", 2)
        nat.tune("chain_grid", chain_grid)
    elif args.chain is not None or P > 1:
        nat.tune("chain", args.chain if args.chain is not None else 0)
    if grad_mode:
        facts = [engine.InverseFactorization(n, d, batch, dt) for _ in range(P)]
    else:
        facts = [engine.AugmentedFactorization(n, d, 0, batch, dt) for _ in range(P)]
    fact = facts[0]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(P - 1)]
    step_no = [0]
    # The sweep's collective, kept off the factorisation streams: every P steps (one per slot in flight) a comm
    # stream waits for those steps' factorisations, packs their (nlml, info) and issues ONE all-gather over RCCL
    # for all of them (asynchronous; two alternating buffers, reused only after the gather that read them).  Per
    # step on the factorisation streams this leaves one event record instead of two copy kernels and a collective
    # whose stream ordering tied every factorisation queue to RCCL's.
    comm = torch.cuda.Stream(dev) if use_dist else None
    done_ev = [torch.cuda.Event() for _ in range(P)] if use_dist else None
    mine = [torch.full((P, 2 * chunk), float("nan"), dtype=torch.float64, device=dev) for _ in range(2)]
    gathered = [torch.empty(world * P * 2 * chunk, dtype=torch.float64, device=dev) if use_dist else None
                for _ in range(2)]
    works = [None, None]
    pending = []
    flushes = [0]

    def flush():
        if not pending:
            return None
        u = flushes[0] % 2
        flushes[0] += 1
        with torch.cuda.stream(comm):
            if works[u] is not None:
                works[u].wait()   # (device-side: the gather that read this buffer two flushes ago is done)
            buf = mine[u]
            for row, j in enumerate(pending):
                comm.wait_event(done_ev[j])
                # (device views, no settle: a persistent run is not waited for here; a timed-out one would
                # arrive as info = -1 and fail the all-gather check)
                nl_dev, info_dev = facts[j].unsettled_results()
                nl_dev.record_stream(comm)
                info_dev.record_stream(comm)
                buf[row, :batch] = nl_dev
                buf[row, chunk:chunk + batch] = info_dev.to(torch.float64)
            works[u] = dist.all_gather_into_tensor(gathered[u], buf.reshape(-1), async_op=True)
        pending.clear()
        return u

    def step(slot=None):
        i = step_no[0] % P if slot is None else slot
        step_no[0] += 1
        f = facts[i]
        with torch.cuda.stream(streams[i]):
            if grad_mode:
                f.run(kd, H, H.shape[1], NZ, 0, X, 0, Y, 0, gradient=True)
            else:
                f.run(kd, H, H.shape[1], NZ, 0, X, 0, Y, 0)
            if use_dist:
                done_ev[i].record(streams[i])
        if use_dist:
            if i in pending:
                flush()
            pending.append(i)
            if len(pending) == P:
                flush()

    # every slot once before the warm-up (setup, not a warm-up step): a stream's first launch allocates libgpk's
    # per-stream scratch, a device synchronisation that would otherwise land in the timed region whenever the
    # warm-up has fewer steps than there are slots (C2 at 8 in flight: 198 instead of 1715 evals/s with 3)
    for i in range(P):
        step(slot=i)
    if use_dist:
        flush()
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    if use_dist:
        flush()
    torch.cuda.synchronize()
    # persistent launches are not verified inside the timed region (no step reads a result): a launch whose waits
    # timed out (info = -1, its candidates not evaluated) is counted on the device (gpk_chain_stats) and its
    # candidates are left out of `value` below
    timeouts0 = nat.chain_timeouts()
    # timed region: no per-launch HIP events (they would add a marker packet to every launch)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if use_dist:
        flush()   # (the last steps' results: every evaluation of the timed region is gathered inside it)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if use_dist:
        dist.barrier()
    el = t1 - t0
    timed_out = nat.chain_timeouts() - timeouts0
    if timed_out:
        sys.stderr.write("bench.py: %d persistent launches timed out in the timed region; their candidates are not "
                         "counted\n" % timed_out)
    if use_dist:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
        to = torch.tensor([timed_out], dtype=torch.int64, device=dev)
        dist.all_reduce(to, op=dist.ReduceOp.SUM)
        timed_out = int(to.item())
    # per-class kernel spans of the production schedule (look-ahead on): a separate events pass
    use_events = not args.no_events
    timing = None
    if use_events:
        nat.timing_reset()
        nat.timing_enable(True)
        for _ in range(args.roofline_steps):
            step()
        torch.cuda.synchronize()
        nat.timing_enable(False)
        timing = nat.timing_read()
    # Roofline pass: a few more steps with the look-ahead off, so that every kernel runs alone on
    # the caller's stream and its HIP-event duration is its own (in the timed region above the
    # bulk update shares the chip with the panel chain, which stretches each launch's span).
    iso = None
    if use_events:
        old_la = nat.tune("lookahead", 0)
        step(slot=0)
        torch.cuda.synchronize()
        nat.timing_reset()
        nat.timing_enable(True)
        for _ in range(args.roofline_steps):
            step(slot=0)
        torch.cuda.synchronize()
        nat.timing_enable(False)
        iso = nat.timing_read()
        nat.tune("lookahead", old_la)
    nl_all = [float(v) for v in fact.nlml().cpu().tolist()]
    nl = nl_all[0]
    info = int(fact.info.abs().max().item())
    gathered_ok = None
    if use_dist:
        # one more step on slot 0, gathered on its own: every rank's (nlml, info) pairs must have arrived via RCCL
        torch.cuda.synchronize()   # (the events passes' gathers are done with both buffers)
        pending.clear()
        mine[flushes[0] % 2].fill_(float("nan"))
        step(slot=0)
        u = flush()
        torch.cuda.synchronize()
        g = gathered[u].view(world, P, 2 * chunk)[:, 0, :].cpu()
        total = len(c4_candidates()) if sweep else world * batch
        vals = g[:, :chunk].reshape(-1)
        gathered_ok = bool(int(torch.isfinite(vals).sum()) == total and float(g[:, chunk:].nan_to_num(0).abs().max()) == 0.0)

    if rank == 0:
        evals = args.steps * ((len(c4_candidates()) if args.slice_of == 1 else batch) if sweep else world * batch)
        # (a timed-out persistent launch evaluated none of its batch's candidates; summed over the ranks)
        evals -= timed_out * batch
        value = evals / el
        ms = el / args.steps * 1000.0
        lay = fact.layout
        # algorithmic flops per evaluation: potrf + 2 trsv; with the gradient, potrf + trtri + lauum
        # (n^3: the inverse from the identity-augmented factorisation) + the O(n^2) gradient pass
        f_lml = float(n) ** 3 if grad_mode else n ** 3 / 3.0 + 2.0 * n * n
        roof = None
        roof_k = None
        breakdown = None
        if timing:
            pmc = pmc_traffic(args.config + ("_grad" if grad_mode else ""), batch)
            up = iso["update"]
            ach = up["flops"] / (up["ms"] * 1e-3) / 1e12 if up["ms"] > 0 else 0.0
            ov = timing["update"]
            roof = {"bound": "mfma", "achieved": round(ach, 3), "peak": PEAK[dtn], "unit": "TFLOP/s",
                    "frac": round(ach / PEAK[dtn], 4), "traffic": (pmc.get("hbm_bytes_per_launch") if pmc else None),
                    "traffic_source": (pmc.get("source") if pmc else None),
                    "kernel": "gemm_kernel<UPDATE> (trailing SYRK, %s MFMA 16x16x4)" % dtn,
                    "measured_in": "%d-step post-pass with the look-ahead off (kernels serialised on one "
                                   "stream); the rocprof trace's last %d update dispatches" % (
                                       args.roofline_steps, up["launches"]),
                    "launches_per_step": up["launches"] // args.roofline_steps,
                    "avg_launch_us": round(up["ms"] * 1e3 / max(1, up["launches"]), 2),
                    "algorithmic_gflop_per_launch": round(up["flops"] / max(1, up["launches"]) / 1e9, 4),
                    "algorithmic_bytes_per_launch": round(up["bytes"] / max(1, up["launches"])),
                    "overlapped_achieved": round(ov["flops"] / (ov["ms"] * 1e-3) / 1e12, 3) if ov["ms"] > 0 else None}
            if persist and ov["launches"] > 0 and ov["ms"] > 0:
                # the persistent launches (timing class "update": the whole factorisation is one chain_kernel
                # launch) as they run in the timed schedule, P side by side: each launch's algorithmic flops /
                # its own HIP-event span, against the MFMA peak (of the dtype) of the CUs it holds
                ach_l = ov["flops"] / (ov["ms"] * 1e-3) / 1e12
                peak_l = PEAK[dtn] * chain_grid / ncu
                roof.update({"achieved": round(ach_l, 3), "peak": round(peak_l, 3), "frac": round(ach_l / peak_l, 4),
                             "kernel": "chain_kernel (persistent factorisation, %d workgroups = %d of %d CUs, %s "
                                       "MFMA tiles)" % (chain_grid, chain_grid, ncu, dtn),
                             "measured_in": "%d-step events pass of the timed schedule (%d launches in flight); peak "
                                            "scaled to the launch's CU share" % (args.roofline_steps, P),
                             "launches_per_step": ov["launches"] // args.roofline_steps,
                             "avg_launch_us": round(ov["ms"] * 1e3 / ov["launches"], 2),
                             "algorithmic_gflop_per_launch": round(ov["flops"] / ov["launches"] / 1e9, 4),
                             "isolated_achieved": round(ach, 3), "chip_achieved": round(f_lml * value / 1e12, 3)})
            asm = timing["assemble"]
            ia = iso["assemble"]
            if ia["launches"] > 0 and ia["ms"] > 0:
                # the K build (gpk_assemble), isolated: algorithmic bytes (the lower tiles written + the points
                # read, include/gpk.h) per launch / its HIP-event duration, against the HBM peak
                gbs = ia["bytes"] / (ia["ms"] * 1e-3) / 1e9
                roof_k = {"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                          "frac": round(gbs / 8000.0, 4), "kernel": "assemble_kernel (K build)",
                          "launches_per_step": ia["launches"] // args.roofline_steps,
                          "avg_launch_us": round(ia["ms"] * 1e3 / ia["launches"], 2),
                          "algorithmic_bytes_per_launch": round(ia["bytes"] / ia["launches"]),
                          "measured_in": "the same look-ahead-off post-pass"}
            else:
                roof_k = None
            breakdown = {k: round(v["ms"] / args.roofline_steps, 4) for k, v in timing.items()}
            breakdown["kbuild_GBps"] = round(asm["bytes"] / (asm["ms"] * 1e-3) / 1e9, 1) if asm["ms"] > 0 else None
            breakdown["note"] = ("sums of kernel spans per class over a %d-step events pass after the timed region; "
                                 "with the look-ahead the classes overlap" % args.roofline_steps)
        cpu = None
        cpu_nl0 = None
        if not args.no_cpu_baseline and world == 1:
            if grad_mode:
                cpu = cpu_baseline_grad(args.config, n)
            else:
                cpu, cpu_nl0 = cpu_baseline(args.config, n, args.cpu_seconds, rows[0])
        # parity of the bench's own numbers: -LML of spread candidates against the oracle on the same inputs
        check = {"nlml": nl, "info": info, "chain_timeouts_timed": timed_out,
                 **({"allgather_ok": gathered_ok} if use_dist else {})}
        if not args.no_check:
            idx = ([int(v) for v in args.check_candidates.split(",")] if args.check_candidates else
                   sorted({0, batch // 2, batch - 1}))
            check.update(oracle_check(args.config, n, rows, idx, kname, d, noise, nl_all,
                                      known={0: cpu_nl0} if cpu_nl0 is not None else {}))
        line = {
            "metric": ("log-marginal-likelihood%s evals/sec at N=%d %s"
                       % (" + gradient" if grad_mode else "", n, "fp64" if dtn == "f64" else "fp32")),
            "value": round(value, 3),
            "unit": "LML+gradient evals/s" if grad_mode else "LML evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "strong" if sweep else "weak",
            "vs_baseline": None,
            "dtype": dtn,
            "data": "synthetic (SURVEY §8d generator, numpy default_rng seed %d), resident in HBM"
                    % {"metric": 5, "C2": 1, "C3": 2, "C4": 3, "C5": 4}[args.config],
            "config": {"workload": ("%s GP -LML sweep, kernel=SE (scaled), D=%d, N=%d, noise=%g; one step = all %d "
                                    "(lengthscale, variance) candidates, %d per rank as one batched factorisation"
                                    % (args.config, d, n, noise, len(c4_candidates()), batch)) if sweep else
                                   ("%s GP -LML, kernel=%s, D=%d, N=%d, noise=%g; %d candidate evaluations per rank per step (batched factorisation)"
                                    % (args.config, kname, d, n, noise, batch)),
                       "candidates_per_rank_step": batch,
                       "batches_in_flight": P,
                       "schedule": (("consecutive steps rotate over %d factorisation buffers on %d HIP streams, "
                                     "each factorisation ONE persistent launch on %d of the %d CUs (%d in flight side "
                                     "by side)" % (P, P, chain_grid, ncu, P)) if persist else
                                    ("consecutive steps rotate over %d factorisation buffers on %d HIP streams (one "
                                     "batch's panel chain overlaps the next batch's trailing updates), panel "
                                     "look-ahead %s" % (P, P, {0: "off", 1: "on"}.get(la, "auto")))),
                       "n": n, "d": d, "kernel": kname, "panel": int(lay.nb), "parallelism": "dp%d (independent candidates)" % world},
            "roofline": roof,
            "kbuild_roofline": roof_k,
            "cpu_baseline": cpu,
            "lml_tflops": round(f_lml * value / 1e12, 3),
            "lml_frac_of_peak": round(f_lml * value / 1e12 / PEAK[dtn], 4),
            "kernel_ms_per_step": breakdown,
            "check": check,
        }
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        if sweep and args.slice_of != 1:
            line["slice"] = {"of_world": args.slice_of, "candidates": batch,
                             "projected_sweep_evals_per_s": round(len(c4_candidates()) * args.steps / el, 3),
                             "note": "this GPU timed rank 0's slice of a %d-way sharded C4 sweep; value = the slice's "
                                     "candidates / s, projected = all 128 / the slice's step time" % args.slice_of}
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
