"""The persistent single-member factorisation (gpk_tune("chain"), chain_kernel in gpk_potrf.hip; on by default for single f64 evaluations since it measured faster,
DESIGN §4) against the launch-per-panel schedule and the oracle (needs the MI355X).

One f64 member without identity / ragged rows runs as ONE launch whose workgroups claim the tasks of
gpk_chain_plan (tests/test_chain_plan.py checks that list on the host).  Contract with the launch path:
agreement to 1e-12 relative in L, z, -LML, mu and Sigma at every size (N up to 7296 here), at the reference's
1e-8 jitter as well; and bit-identical results (test_chain_bitwise_vs_launch_path, N up to 12288, the
chain_max_p edge): every tile update and panel solve keeps the launch path's MFMA k-order, the deferred tile
updates over g panels included, and an f64 accumulator stored and reloaded between panels rounds nothing.  Between runs of the chain itself the arithmetic order is fixed
(every tile's updates are serialised by its counter), so repeated runs are bitwise equal.  A wait that
times out is recovered on the launch path at the first read of the run's results (engine.AugmentedFactorization._settle).
"""
import threading

import numpy as np
import pytest
import torch

from oracle import gp_oracle as o
from tests.helpers import jitter_nll_bar, make_kernel

from gaussianprocessfundamentals_amd import engine

pytestmark = pytest.mark.gpu

SE = ("SE", {"ard": False})


def _run(n, m, chain, hyp=0.1, noise=1e-2, seed=3, sync=True):
    x, y = o.make_inputs("C1", n=n, seed=seed)
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    H = torch.tensor([[hyp]], dtype=torch.float64, device=dev)
    NZ = torch.tensor([noise], dtype=torch.float64, device=dev)
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    Xs = torch.linspace(-0.1, 1.1, max(m, 1), dtype=torch.float64, device=dev).reshape(-1, 1) if m else None
    # chain 1 -> 2: the persistent launch even if another stream still has work in flight
    with engine.nat.thread_tune(chain=2 if chain else 0):
        f = engine.AugmentedFactorization(n, 1, m, 1)
        f.W.zero_()
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0, Xs, 0)
        if sync:
            torch.cuda.synchronize()
    return f, (x, y)


def _lower(f):
    lay = f.layout
    w = f.w(0).cpu().numpy()
    return np.tril(w[: lay.y_row + 1, : lay.y_row + 1])


@pytest.mark.parametrize("n,m,noise", [(1, 0, 1e-2), (100, 0, 1e-2), (128, 0, 1e-2), (257, 0, 1e-2),
                                       (1000, 37, 1e-2), (2048, 0, 1e-2), (3000, 300, 1e-2), (4096, 0, 1e-2),
                                       (4096, 100, 1e-2), (6144, 0, 1e-2), (7168, 0, 1e-2), (7168, 100, 1e-2),
                                       (7296, 0, 1e-2), (1000, 0, 1e-8), (4096, 0, 1e-8)])
def test_chain_matches_the_launch_path(n, m, noise):
    fc, _ = _run(n, m, 1, noise=noise)
    fl, _ = _run(n, m, 0, noise=noise)
    assert fc.layout.p <= 12416  # (inside chain_max_p: the persistent launch ran)
    assert int(fc.info.cpu()[0]) == 0 and int(fl.info.cpu()[0]) == 0
    a, b = _lower(fc), _lower(fl)
    scale = np.abs(b).max()
    assert np.abs(a - b).max() <= 1e-12 * scale
    oc, ol = fc.out.cpu().numpy(), fl.out.cpu().numpy()
    assert oc[0] == pytest.approx(ol[0], rel=1e-12)
    if m:
        np.testing.assert_allclose(fc.mu.cpu().numpy(), fl.mu.cpu().numpy(), rtol=0, atol=1e-10)
        np.testing.assert_allclose(fc.var.cpu().numpy(), fl.var.cpu().numpy(), rtol=0, atol=1e-10)


@pytest.mark.parametrize("n,m", [(257, 0), (3000, 300), (4096, 0), (7296, 0), (8192, 0), (12288, 0)])
def test_chain_bitwise_vs_launch_path(n, m):
    """Same MFMA k-order in every tile update and panel solve, and an f64 accumulator stored and reloaded
    between panels rounds nothing: the persistent launch reproduces the launch path bit for bit."""
    fc, _ = _run(n, m, 1)
    fl, _ = _run(n, m, 0)
    a, b = _lower(fc), _lower(fl)
    diff = int(np.count_nonzero(a.view(np.uint64) != b.view(np.uint64)))
    assert diff == 0, "%d of %d lower-triangle words differ" % (diff, a.size)
    assert fc.out.cpu()[0].item() == fl.out.cpu()[0].item()


@pytest.mark.parametrize("group,uq", [(1, 0), (1, 1), (4, 0), (8, 1), (4, 2), (1, 2)])
@pytest.mark.parametrize("n,m", [(2100, 40), (5000, 0)])
def test_chain_plan_variants_bitwise_vs_launch_path(n, m, group, uq):
    """Every planner variant (deferred-update depth chain_group, the next diagonal block's update as quarter tasks,
    one task per slice, or inside the slices' panel-solve tasks (SQ, chain_uq 2)) reproduces the launch path bit for
    bit: the same per-tile MFMA k-order in every variant."""
    with engine.nat.thread_tune(chain_group=group, chain_uq=uq):
        before = engine.nat.chain_stats()["launches"]
        fc, _ = _run(n, m, 1)
        assert engine.nat.chain_stats()["launches"] > before
    fl, _ = _run(n, m, 0)
    a, b = _lower(fc), _lower(fl)
    assert int(np.count_nonzero(a.view(np.uint64) != b.view(np.uint64))) == 0
    assert fc.out.cpu()[0].item() == fl.out.cpu()[0].item()


@pytest.mark.parametrize("n,m,uq", [(2100, 40, 1), (4096, 0, 1), (8192, 0, 1), (5000, 0, 0), (5000, 0, 2)])
def test_chain_two_lists_bitwise_vs_launch_path(n, m, uq):
    """gpk_tune("chain_xcd"): the diagonal chain's tasks as a second task list claimed first by workgroups of one
    XCD (tests/test_chain_plan.py simulates its progress and cell order).  Only which workgroup runs a task changes:
    bitwise the launch path's results, and the persistent launch really ran with it."""
    with engine.nat.thread_tune(chain_xcd=1, chain_uq=uq):
        before = engine.nat.chain_stats()["launches"]
        fc, _ = _run(n, m, 1)
        assert engine.nat.chain_stats()["launches"] > before
    fl, _ = _run(n, m, 0)
    a, b = _lower(fc), _lower(fl)
    assert int(np.count_nonzero(a.view(np.uint64) != b.view(np.uint64))) == 0
    assert fc.out.cpu()[0].item() == fl.out.cpu()[0].item()


def test_chain_noise_1e8_matches_the_oracle():
    """The reference's default jitter (1e-8, cond(K) ~ 1e10 at N = 256) through the persistent launch."""
    f, (x, y) = _run(1000, 0, 1, noise=1e-8)
    ref = o.nlml(SE, [0.1], 1e-8, x, y)
    got = float(f.nlml().cpu()[0])
    bar = jitter_nll_bar(o.k_noised(SE, [0.1], 1e-8, x.reshape(-1, 1)), y, ref)   # (~2.2e-5: cond(K) 2.4e10)
    err = abs(got - ref) / abs(ref)
    print("chain N=1000 jitter 1e-8: rel %.3e, bar %.3e" % (err, bar))
    assert err < bar, (got, ref, bar)


@pytest.mark.parametrize("n", [300, 4096, 7296])
def test_chain_nlml_matches_the_oracle(n):
    f, (x, y) = _run(n, 0, 1)
    ref = o.nlml(SE, [0.1], 1e-2, x, y)
    assert float(f.nlml().cpu()[0]) == pytest.approx(ref, rel=1e-9)


def test_chain_runs_as_one_launch():
    engine.nat.timing_reset()
    engine.nat.timing_enable(True)
    try:
        _run(2048, 0, 1)
        t = engine.nat.timing_read()
    finally:
        engine.nat.timing_enable(False)
    assert t["diag"]["launches"] == 0 and t["trsm"]["launches"] == 0
    assert t["update"]["launches"] == 1


def test_chain_is_deterministic():
    a, _ = _run(3000, 64, 1)
    b, _ = _run(3000, 64, 1)
    assert np.array_equal(_lower(a).view(np.uint64), _lower(b).view(np.uint64))


def test_chain_reports_the_first_non_positive_pivot():
    fc, _ = _run(700, 0, 1, hyp=0.3, noise=-0.5)
    fl, _ = _run(700, 0, 0, hyp=0.3, noise=-0.5)
    ic, il = int(fc.info.cpu()[0]), int(fl.info.cpu()[0])
    assert ic > 0 and ic == il
    with pytest.raises(engine.CholeskyError):
        fc.check_info()


def test_chain_on_concurrent_streams():
    ref = {n: _lower(_run(n, 0, 1, hyp=0.05 + 1e-4 * n)[0]) for n in (1500, 2600)}
    streams = [torch.cuda.Stream() for _ in range(2)]
    out = {}
    for s, n in zip(streams, (1500, 2600)):
        with torch.cuda.stream(s):
            out[n] = _run(n, 0, 1, hyp=0.05 + 1e-4 * n, sync=False)[0]
    torch.cuda.synchronize()
    for n in (1500, 2600):
        assert np.array_equal(_lower(out[n]).view(np.uint64), ref[n].view(np.uint64))


def test_persistent_launches_side_by_side_on_cu_shares():
    """bench.py's C2 schedule: 8 persistent launches in flight on 8 streams, each with 3/16 of the CUs as its grid
    (chain_grid), the runs not verified until read (no synchronisation between them).  Each reproduces the launch
    path bit for bit, whatever the others do meanwhile."""
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    n, hyps = 2600, [0.05 + 0.01 * i for i in range(8)]
    ref = [_lower(_run(n, 0, 0, hyp=h)[0]) for h in hyps]
    streams = [torch.cuda.Stream() for _ in hyps]
    runs = []
    with engine.nat.thread_tune(chain_grid=max(1, ncu * 3 // 16)):
        before = engine.nat.chain_stats()["launches"]
        for rep in range(2):
            for s, h in zip(streams, hyps):
                with torch.cuda.stream(s):
                    runs.append(_run(n, 0, 1, hyp=h, sync=False)[0])
        assert engine.nat.chain_stats()["launches"] - before == 2 * len(hyps)
    torch.cuda.synchronize()
    for i, f in enumerate(runs):
        assert int(f.info.cpu()[0]) == 0
        assert np.array_equal(_lower(f).view(np.uint64), ref[i % len(hyps)].view(np.uint64)), i


def test_unsettled_results_are_the_settled_ones():
    """unsettled_results() (bench.py's per-step all-gather) reads the device buffers without waiting for the run:
    after the stream drains they hold what nlml() / info return once settled."""
    f, _ = _run(3000, 0, 1, sync=False)
    nl, info = f.unsettled_results()
    nl, info = nl.clone(), info.clone()   # (stream-ordered copies)
    torch.cuda.synchronize()
    assert torch.equal(nl, f.nlml()) and torch.equal(info, f.info)


def test_timed_out_wait_falls_back_to_the_launch_path():
    """gpk_tune("chain_force_timeout", 1): the next persistent launch reports a timeout at its first wait
    (info = -1, W left half factored).  The same run() call re-assembles and factors on the launch path and
    counts the fallback; the result is the oracle's -LML."""
    before = engine.CHAIN_FALLBACKS
    t_before = engine.nat.chain_timeouts()
    engine.nat.tune("chain_force_timeout", 1)
    try:
        f, (x, y) = _run(2000, 0, 1)
    finally:
        engine.nat.tune("chain_force_timeout", 0)
    assert engine.CHAIN_FALLBACKS == before          # (verified lazily: nothing read yet)
    assert int(f.info.cpu()[0]) == 0                 # the first read re-runs it
    assert engine.CHAIN_FALLBACKS == before + 1
    # the device counts the aborted launch once (gpk_chain_stats out[4], the bench's check of its timed region)
    assert engine.nat.chain_timeouts() == t_before + 1
    assert float(f.nlml().cpu()[0]) == pytest.approx(o.nlml(SE, [0.1], 1e-2, x, y), rel=1e-9)
    # with verification off the timeout surfaces as an infrastructure error, never as "not PD"
    engine.CHAIN_VERIFY = False
    engine.nat.tune("chain_force_timeout", 1)
    try:
        f, _ = _run(2000, 0, 1)
        assert int(f.info.cpu()[0]) == -1
        with pytest.raises(RuntimeError, match="timed out"):
            f.check_info()
    finally:
        engine.CHAIN_VERIFY = True
        engine.nat.tune("chain_force_timeout", 0)


def test_timed_out_wait_through_get_metric():
    """The drop-in API: get_metric / get_metric_checked give the oracle value although the persistent launch
    behind them timed out."""
    from gaussianprocessfundamentals_amd.DataHandling.DataInput import DataInput
    from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type
    from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType
    from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction
    from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import GaussianProcess
    x, y = o.make_inputs("C1", n=1500, seed=8)
    di = DataInput(x.reshape(-1, 1), y.reshape(-1, 1), x.reshape(-1, 1), y.reshape(-1, 1))
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(make_kernel(SE, 1), ZeroMeanFunction(1))
    g.set_data_input(di)
    met = get_metric_by_type(MetricType.LL, g)
    before = engine.CHAIN_FALLBACKS
    engine.nat.tune("chain_force_timeout", 1)
    try:
        with engine.nat.thread_tune(chain=2):
            got = float(met.get_metric_checked([torch.tensor(0.1, dtype=torch.float64)],
                                               torch.tensor(1e-2, dtype=torch.float64)))
    finally:
        engine.nat.tune("chain_force_timeout", 0)
    assert engine.CHAIN_FALLBACKS == before + 1
    assert got == pytest.approx(o.nlml(SE, [0.1], 1e-2, x, y), rel=1e-9)


def test_two_host_threads_on_the_default_stream():
    """Two Python threads (ctypes releases the GIL) run single f64 evaluations of different sizes on the same
    default stream: each thread's persistent launches use their own counter scratch, so every result is
    bitwise the launch path's result for its size."""
    sizes = (1500, 2600)
    ref = {n: _lower(_run(n, 0, 0, hyp=0.05 + 1e-4 * n)[0]) for n in sizes}
    out, errors = {}, []

    def work(n):
        try:
            for rep in range(6):
                f = _run(n, 0, 1, hyp=0.05 + 1e-4 * n, sync=False)[0]
                out[(n, rep)] = f
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    ts = [threading.Thread(target=work, args=(n,)) for n in sizes]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    for (n, rep), f in out.items():
        assert int(f.info.cpu()[0]) == 0
        assert np.array_equal(_lower(f).view(np.uint64), ref[n].view(np.uint64)), (n, rep)


def test_auto_mode_declines_while_another_stream_is_busy():
    """chain = 1 (auto): while a factorisation enqueued on another stream is still running, a single f64
    evaluation takes the launch path (the persistent launch would claim every CU); once the device is idle
    it takes the persistent launch again."""
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    x, y = o.make_inputs("C1", n=4096, seed=3)
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    big = engine.AugmentedFactorization(4096, 1, 0, 16)
    Hb = torch.linspace(0.05, 0.2, 16, dtype=torch.float64, device=dev).reshape(16, 1).contiguous()
    H = torch.tensor([[0.1]], dtype=torch.float64, device=dev)
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    with engine.nat.thread_tune(chain=1):
        with torch.cuda.stream(side):
            big.run(kd, Hb, 1, NZ, 0, X, 0, Y, 0)     # ~10 ms of work on the side stream
        s0 = engine.nat.chain_stats()
        one = engine.AugmentedFactorization(4096, 1, 0, 1)
        one.run(kd, H, 1, NZ, 0, X, 0, Y, 0)            # default stream, side stream still busy
        s1 = engine.nat.chain_stats()
        torch.cuda.synchronize()
        one.run(kd, H, 1, NZ, 0, X, 0, Y, 0)            # idle device
        s2 = engine.nat.chain_stats()
    assert s1["declined_busy"] > s0["declined_busy"] and s1["launches"] == s0["launches"]
    assert s2["launches"] == s1["launches"] + 1 and s2["last_was_chain"]
    assert float(one.nlml().cpu()[0]) == pytest.approx(o.nlml(SE, [0.1], 1e-2, x, y), rel=1e-9)


@pytest.mark.parametrize("n,batch", [(1000, 2), (2048, 3), (700, 5)])
def test_chain_batched_members_bitwise_vs_launch_path(n, batch):
    """A small batch as ONE persistent launch (gpk_tune chain_max_batch): every member's task graph in one
    list, member index in the task word.  Each member -- different hyperparameters, one of them not positive
    definite (negative noise) -- is bitwise the launch path's, info included."""
    x, y = o.make_inputs("C1", n=n, seed=11)
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    H = torch.linspace(0.06, 0.14, batch, dtype=torch.float64, device=dev).reshape(batch, 1).contiguous()
    NZ = torch.full((batch,), 1e-2, dtype=torch.float64, device=dev)
    NZ[1] = -0.5
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    res = []
    for mode in (2, 0):
        before = engine.nat.chain_stats()["launches"]
        with engine.nat.thread_tune(chain=mode, chain_max_batch=8):
            f = engine.AugmentedFactorization(n, 1, 0, batch)
            f.W.zero_()
            f.run(kd, H, 1, NZ, 1, X, 0, Y, 0)
            torch.cuda.synchronize()
        assert (engine.nat.chain_stats()["launches"] > before) == (mode == 2)
        res.append((f.info.cpu().clone(), f.out.cpu().clone(), [_lower_b(f, b) for b in range(batch)]))
    (ic, oc, lc), (il, ol, ll) = res
    assert torch.equal(ic, il) and int(ic[1]) > 0 and int(ic[0]) == 0
    for b in range(batch):
        if b == 1:
            continue
        assert np.array_equal(lc[b].view(np.uint64), ll[b].view(np.uint64)), b
        assert oc[4 * b].item() == ol[4 * b].item()
        assert float(oc[4 * b]) == pytest.approx(o.nlml(SE, [float(H[b, 0])], 1e-2, x, y), rel=1e-9)


def _lower_b(f, b):
    lay = f.layout
    w = f.w(b).cpu().numpy()
    return np.tril(w[: lay.y_row + 1, : lay.y_row + 1])


def test_chain_batched_timeout_falls_back():
    """A forced timeout in a batched persistent launch marks every unfinished member -1 and the whole batch
    is re-run on the launch path in the same call."""
    x, y = o.make_inputs("C1", n=1500, seed=12)
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    H = torch.tensor([[0.08], [0.1], [0.12]], dtype=torch.float64, device=dev)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    before = engine.CHAIN_FALLBACKS
    engine.nat.tune("chain_force_timeout", 1)
    try:
        with engine.nat.thread_tune(chain=2, chain_max_batch=8):
            f = engine.AugmentedFactorization(1500, 1, 0, 3)
            f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
    finally:
        engine.nat.tune("chain_force_timeout", 0)
    got = f.nlml().cpu().numpy()
    assert engine.CHAIN_FALLBACKS == before + 1
    for b, l in enumerate((0.08, 0.1, 0.12)):
        assert got[b] == pytest.approx(o.nlml(SE, [l], 1e-2, x, y), rel=1e-9)


def test_run_is_asynchronous_and_verified_at_the_first_read():
    """run() does not synchronise (the persistent launch's timeout check waits for the first read of a result):
    several runs enqueue ahead of the device.  N = 8192 takes ~4.5 ms per run on the device, the enqueue well
    under a millisecond, so right after the third run the stream is still busy.  The first read then returns
    the oracle's -LML."""
    x, y = o.make_inputs("C1", n=8192, seed=3)
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    H = torch.tensor([[0.1]], dtype=torch.float64, device=dev)
    NZ = torch.tensor([1e-2], dtype=torch.float64, device=dev)
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    with engine.nat.thread_tune(chain=2):
        f = engine.AugmentedFactorization(8192, 1, 0, 1)
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
        before = engine.nat.chain_stats()["launches"]
        for _ in range(3):
            f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        busy = not torch.cuda.current_stream().query()
        assert engine.nat.chain_stats()["launches"] == before + 3
    assert busy, "run() synchronised with the device"
    assert f._pending is not None
    got = float(f.nlml().cpu()[0])
    assert f._pending is None
    assert got == pytest.approx(o.nlml(SE, [0.1], 1e-2, x, y), rel=1e-9)


# ------------------------------------------------------------------ identity-augmented (gradient / inverse) path
def _run_eye(n, chain, batch=1, seed=5, noise=1e-2):
    x, y = o.make_inputs("C1", n=n, seed=seed)
    dev = engine.device()
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    H = torch.linspace(0.08, 0.12, batch, dtype=torch.float64, device=dev).reshape(batch, 1).contiguous()
    NZ = torch.tensor([noise], dtype=torch.float64, device=dev)
    X = torch.tensor(x, dtype=torch.float64, device=dev).reshape(-1, 1).contiguous()
    Y = torch.tensor(y, dtype=torch.float64, device=dev).reshape(1, -1).contiguous()
    before = engine.nat.chain_stats()["launches"]
    with engine.nat.thread_tune(chain=2 if chain else 0, chain_max_batch=8):
        f = engine.InverseFactorization(n, 1, batch)
        f.W.zero_()
        f.run(kd, H, 1, NZ, 0, X, 0, Y, 0)
        torch.cuda.synchronize()
    assert (engine.nat.chain_stats()["launches"] > before) == bool(chain)
    return f, (x, y)


@pytest.mark.parametrize("n,batch", [(1, 1), (257, 1), (1000, 1), (2048, 1), (2048, 2), (4096, 1), (6144, 1),
                                     (8192, 1)])
def test_chain_eye_bitwise_vs_launch_path(n, batch):
    """The identity-augmented factorisation (the value + gradient call, include/gpk.h gpk_nlml_grad) as one
    persistent launch: its list leaves out the structurally zero tasks of E L^-T (gpk_chain_plan_ex), keeps the
    launch path's per-tile MFMA k-order, and reproduces the launch path bit for bit -- L, L^-T, -K^-1, -alpha, the
    -LML and the gradient."""
    fc, _ = _run_eye(n, 1, batch)
    fl, _ = _run_eye(n, 0, batch)
    for b in range(batch):
        a, c = _lower_b(fc, b), _lower_b(fl, b)
        diff = int(np.count_nonzero(a.view(np.uint64) != c.view(np.uint64)))
        assert diff == 0, "member %d: %d of %d lower-triangle words differ" % (b, diff, a.size)
    assert torch.equal(fc.out.cpu(), fl.out.cpu())
    assert torch.equal(fc.gradient().cpu(), fl.gradient().cpu())


def test_chain_eye_matches_the_oracle():
    from oracle import gp_autodiff as ad
    f, (x, y) = _run_eye(3000, 1, seed=9)
    nl, g, gn = ad.nlml_and_grad(SE, [0.08], 1e-2, x.reshape(-1, 1), y)
    assert float(f.nlml().cpu()[0]) == pytest.approx(nl, rel=1e-9)
    got = f.gradient()[0].cpu().numpy()
    exp = np.array([float(np.asarray(g[0]).reshape(-1)[0]), gn])
    assert np.max(np.abs(got - exp)) <= 1e-7 * max(1.0, np.max(np.abs(exp)))
    Kn = o.k_noised(SE, [0.08], 1e-2, x.reshape(-1, 1))
    Ki = np.linalg.inv(Kn)
    assert np.linalg.norm(f.k_inv(0).cpu().numpy() - Ki) / np.linalg.norm(Ki) < 1e-8


def test_chain_eye_timeout_falls_back():
    """A forced timeout in the identity-augmented persistent launch: the first read (the gradient) re-runs the
    value + gradient call on the launch path."""
    before = engine.CHAIN_FALLBACKS
    engine.nat.tune("chain_force_timeout", 1)
    try:
        f, (x, y) = _run_eye(1500, 1, seed=4)
    finally:
        engine.nat.tune("chain_force_timeout", 0)
    g = f.gradient()[0].cpu().numpy()
    assert engine.CHAIN_FALLBACKS == before + 1
    fl, _ = _run_eye(1500, 0, seed=4)
    assert np.array_equal(g, fl.gradient()[0].cpu().numpy())
    assert float(f.nlml().cpu()[0]) == float(fl.nlml().cpu()[0])


@pytest.mark.parametrize("n", [700, 4096, 8192])
def test_chain_sq_eye_and_timeout(n):
    """SQ tasks (chain_uq 2) in the identity-augmented list, bitwise against the launch path; and a forced timeout of
    an SQ launch recovers on the launch path."""
    with engine.nat.thread_tune(chain_uq=2):
        fc, _ = _run_eye(n, 1)
    fl, _ = _run_eye(n, 0)
    a, c = _lower_b(fc, 0), _lower_b(fl, 0)
    assert int(np.count_nonzero(a.view(np.uint64) != c.view(np.uint64))) == 0
    assert torch.equal(fc.gradient().cpu(), fl.gradient().cpu())
    if n == 700:
        engine.nat.tune("chain_force_timeout", 1)
        try:
            with engine.nat.thread_tune(chain_uq=2):
                f, (x, y) = _run(n, 0, 1)
        finally:
            engine.nat.tune("chain_force_timeout", 0)
        assert float(f.nlml().cpu()[0]) == pytest.approx(o.nlml(SE, [0.1], 1e-2, x, y), rel=1e-9)
