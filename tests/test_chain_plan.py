"""Host-side checks of the persistent single-member factorisation's task list (gpk_chain_plan; no GPU).

chain_kernel (gaussianprocessfundamentals_amd/csrc/gpk_potrf.hip) claims the tasks in list order and each task
waits on counters before it runs.  Here, for several augmented shapes and worker counts:
  * the waits are restated exactly as the kernel makes them, and an event simulation with random task
    durations checks that every wait is satisfied by a task claimed EARLIER (no deadlock whatever the
    residency) and that, at its start, every 32 x 128 cell a task reads or rewrites already holds the
    last version written by the earlier-claimed tasks (the waits cover every data dependency);
  * the tasks, run in list order on the augmented matrix in numpy, reproduce the blocked factorisation's
    results -- L, z = L^-1 y, the Schur-complement corner (-z^T z, -mu, Sigma) -- against numpy's
    Cholesky of K + noise I (the quantities of gpbasics/Statistics/CovarianceMatrix.py:247-265 and
    Metrics/LogLikelihood.py:30-65).
"""
import heapq

import numpy as np
import pytest

from gaussianprocessfundamentals_amd import _native as nat

NB, SL = 128, 32
D, S, U32, BLK = 0, 1, 2, 3


def _lib_or_skip():
    try:
        nat.load_library()
    except nat.NativeUnavailable as e:  # pragma: no cover - the build check builds it
        pytest.skip(str(e))


def shape(n, m):
    n_pad = -(-n // NB) * NB
    y_row = n_pad + m
    p = -(-(y_row + 1) // NB) * NB
    return n_pad, y_row, p


def decode(task):
    """(type, k, r, j, g): BLK tasks carry ty = 3 | (g - 1) << 2 for an update over panels k .. k + g - 1; a U32
    task with g > 1 is the quarter g - 2 (UQ) of slice r in diagonal block j; bit 6 (first(): identity-augmented
    lists) marks a task whose cells no earlier task updated; bits 8.. hold the member."""
    tyg, k, r, j = (int(v) for v in task)
    return tyg & 3, k, r, j, ((tyg >> 2) & 15) + 1


def first(task):
    return (int(task[0]) >> 6) & 1


def is_sq(task):
    """chain_uq 2: an S task with bit 7 -- the panel solve of slice r of diagonal block k + 1 followed by the slice's
    lower quarters of that block (publishes sdone after the solve, qdone = 1 at the end)."""
    return (int(task[0]) & 3) == S and (int(task[0]) >> 7) & 1 == 1


def cells(task, nsl, uq=False):
    """(reads, writes) of a task as sets of (slice, block column) cells plus ('inv', k) and, for the quarter
    updates (UQ), ('q', slice, block column, quarter)."""
    ty, k, r, j, g = decode(task)

    def sl(b):
        return [s for s in range(4 * b, 4 * b + 4) if s < nsl]

    if ty == D:
        c = {(s, k) for s in sl(k)}
        qc = {("q", s, k, q) for s in sl(k) for q in range(s - 4 * k + 1)} if (uq and k > 0) else set()
        return c | qc, c | {("inv", k)}
    if ty == S and is_sq(task):
        rl = r - 4 * (k + 1)
        rd = {(r, k), ("inv", k), (r, k + 1)} | {(s, k) for s in range(4 * (k + 1), r)}
        return rd, {(r, k)} | {("q", r, k + 1, q) for q in range(rl + 1)}
    if ty == S:   # (g > 1: the block row's slices r .. r + g - 1, chain_s128)
        return {(r + i, k) for i in range(g)} | {("inv", k)}, {(r + i, k) for i in range(g)}
    if ty == U32 and g > 1:
        q = g - 2
        return {(r, k), (4 * j + q, k), (r, j)}, {("q", r, j, q)}
    if ty == U32:
        return {(r, k), (r, j)} | {(s, k) for s in sl(j)}, {(r, j)}
    rd = {(s, q) for s in sl(r) + sl(j) for q in range(k, k + g)} | {(s, j) for s in sl(r)}
    return rd, {(s, j) for s in sl(r)}


def waits(task, nsl, uq=False):
    """The kernel's waits (chain_kernel, dependency section): (counter, index, value >= )."""
    ty, k, r, j, g = decode(task)
    kprev = 0 if first(task) else k   # (the count the previous update of the task's cells published)
    out = []
    if ty == D:
        if k > 0 and uq == 2:
            out += [("qdone", (k - 1, s), 1) for s in range(4 * k, 4 * k + 4) if s < nsl]
        elif k > 0 and uq:
            out += [("qdone", (k - 1, s), s - 4 * k + 1) for s in range(4 * k, 4 * k + 4) if s < nsl]
        elif k > 0:
            out += [("ucnt", (s, k), k) for s in range(4 * k, 4 * k + 4)]
    elif ty == S:
        out.append(("dflag", k, 1))
        if kprev > 0:
            out += [("ucnt", (r + i, k), kprev) for i in range(g)]
        if is_sq(task):
            if k > 0:
                out.append(("ucnt", (r, k + 1), k))
            out += [("sdone", (k, s), 1) for s in range(4 * (k + 1), r)]
    elif ty == U32:
        out.append(("sdone", (k, r), 1))
        if g > 1:
            out.append(("sdone", (k, 4 * j + g - 2), 1))
        else:
            out += [("sdone", (k, s), 1) for s in range(4 * j, 4 * j + 4) if s < nsl]
        if kprev > 0:
            out.append(("ucnt", (r, j), kprev))
    else:
        q = k + g - 1
        out += [("sdone", (q, s), 1) for s in range(4 * r, 4 * r + 4) if s < nsl]
        out += [("sdone", (q, s), 1) for s in range(4 * j, 4 * j + 4) if s < nsl]
        if kprev > 0:
            out += [("ucnt", (s, j), kprev) for s in range(4 * r, 4 * r + 4) if s < nsl]
    return out


def publishes(task, nsl):
    ty, k, r, j, g = decode(task)
    if ty == D:
        return [("dflag", k, 1)]
    if ty == S and is_sq(task):
        return [("sdone", (k, r), 1), ("qdone", (k, r), 1)]
    if ty == S:
        return [("sdone", (k, r + i), 1) for i in range(g)]
    if ty == U32 and g > 1:
        return [("qdone", (k, r), "+1")]
    if ty == U32:
        return [("ucnt", (r, j), k + 1)]
    return [("ucnt", (s, j), k + g) for s in range(4 * r, 4 * r + 4) if s < nsl]


def simulate(tasks, nsl, workers, rng):
    """Claim in list order; start = max(worker free, every wait's publish time); check cell versions."""
    uq = 2 if any(is_sq(t) for t in tasks) else any(decode(t)[0] == U32 and decode(t)[4] > 1 for t in tasks)
    pub = {}           # (counter, index) -> list of (value, time); counters added to: value = "+1"
    last_w = {}        # cell -> finish time of the last earlier-claimed writer
    readers = {}       # cell -> finish times of earlier-claimed readers since that writer
    free = [0.0] * workers
    dur = {D: 28.0, S: 7.0, U32: 7.0, BLK: 18.0}
    for t, task in enumerate(tasks):
        w = int(np.argmin(free))
        start = free[w]
        for cnt, idx, v in waits(task, nsl, uq):
            got = pub.get((cnt, idx), [])
            if got and got[0][0] == "+1":   # a counter of increments: the v-th finished add
                times = sorted(tm for _, tm in got)
                assert len(times) >= v, "task %d %s waits on %s%s >= %d, added to %d times earlier" % (
                    t, task, cnt, idx, v, len(times))
                start = max(start, times[v - 1])
                continue
            hits = [tm for (val, tm) in got if val >= v]
            assert hits, "task %d %s waits on %s%s >= %d, set by no earlier task" % (t, task, cnt, idx, v)
            start = max(start, min(hits))
        rd, wr = cells(task, nsl, uq)
        for c in rd | wr:  # read-after-write / write-after-write: the last writer is done
            assert start >= last_w.get(c, 0.0), "task %d %s starts before the last writer of %s" % (t, task, c)
        ty, g = decode(task)[0], decode(task)[4]
        finish = start + dur[ty] * g * rng.uniform(0.3, 3.0)
        for c in wr:  # write-after-read: earlier readers of the old version are done
            assert all(f <= finish for f in readers.get(c, [])), "task %d %s overwrites %s under a reader" % (
                t, task, c)
        for c in rd - wr:
            readers.setdefault(c, []).append(finish)
        for c in wr:
            last_w[c] = finish
            readers[c] = []
        for cnt, idx, v in publishes(task, nsl):
            pub.setdefault((cnt, idx), []).append((v, finish))
        free[w] = finish


def augmented(n, m, rng):
    n_pad, y_row, p = shape(n, m)
    x = np.sort(rng.uniform(0, 1, n + m))
    xt, xs = x[:n], x[n:]
    k = lambda a, b: np.exp(-0.5 * (a[:, None] - b[None, :]) ** 2 / 0.1 ** 2)  # noqa: E731
    noise = 1e-2
    y = np.sin(6 * xt) + 0.1 * rng.standard_normal(n)
    W = np.zeros((p, p))
    W[:n, :n] = k(xt, xt) + noise * np.eye(n)
    W[n:n_pad, n:n_pad] = np.eye(n_pad - n)
    if m:
        W[n_pad:n_pad + m, :n] = k(xs, xt)
        W[n_pad:n_pad + m, n_pad:n_pad + m] = k(xs, xs)
    W[y_row, :n] = y
    return np.tril(W), (xt, xs, y, noise, k)


def run_tasks(W, tasks, nblk):
    inv = {}
    for task in tasks:
        ty, k, r, j, g = decode(task)
        K = slice(NB * k, NB * k + NB)
        if ty == D:
            a = np.tril(W[K, K])
            L = np.linalg.cholesky(a + np.tril(a, -1).T)
            W[K, K] = L
            inv[k] = np.linalg.inv(L)
        elif ty == S:
            R = slice(SL * r, SL * r + SL * g)
            W[R, K] = W[R, K] @ inv[k].T
            if is_sq(task):
                for q in range(r - 4 * (k + 1) + 1):
                    Q = slice(NB * (k + 1) + SL * q, NB * (k + 1) + SL * q + SL)
                    W[R, Q] -= W[R, K] @ W[Q, K].T
        elif ty == U32 and g > 1:
            q = g - 2
            R, Q = slice(SL * r, SL * r + SL), slice(NB * j + SL * q, NB * j + SL * q + SL)
            W[R, Q] -= W[R, K] @ W[Q, K].T
        elif ty == U32:
            R, J = slice(SL * r, SL * r + SL), slice(NB * j, NB * j + NB)
            W[R, J] -= W[R, K] @ W[J, K].T
        else:
            I, J, KG = slice(NB * r, NB * r + NB), slice(NB * j, NB * j + NB), slice(NB * k, NB * (k + g))
            W[I, J] -= W[I, KG] @ W[J, KG].T
    return W


def plan(n_pad, y_row, grid, group, uq=1, eye=False, u128=0, s128=0):
    with nat.thread_tune(chain_group=group, chain_group_eye=group, chain_uq=uq, chain_u128=u128, chain_s128=s128):
        return nat.chain_plan(n_pad, y_row, grid, eye)


def applied_panels(tasks, nblk):
    """Every tile update (panel q, block row i, block column j) the list applies, each exactly once."""
    seen = []
    for task in tasks:
        ty, k, r, j, g = decode(task)
        if ty == BLK:
            seen += [(q, r, j) for q in range(k, k + g)]
    return seen


@pytest.mark.parametrize("n,m", [(1, 0), (128, 0), (300, 0), (700, 37), (1000, 200), (2048, 0), (3000, 0)])
@pytest.mark.parametrize("group,uq", [(1, 1), (4, 1), (8, 1), (4, 0), (4, 2), (1, 2)])
def test_chain_plan_waits_cover_every_dependency(n, m, group, uq):
    _lib_or_skip()
    n_pad, y_row, p = shape(n, m)
    nsl = y_row // SL + 1
    rng = np.random.default_rng(n + m)
    nblk, yb = n_pad // NB, y_row // NB
    for grid in (1, 3, 16, 256):
        tasks = plan(n_pad, y_row, grid, group, uq)
        kinds = np.bincount(tasks[:, 0] & 3, minlength=4)
        nq = int(np.sum(((tasks[:, 0] & 3) == U32) & (((tasks[:, 0] >> 2) & 15) > 0)))
        assert nq == (10 * (nblk - 1) if uq == 1 else 0)   # 1 + 2 + 3 + 4 quarters per next diagonal block
        assert sum(is_sq(t) for t in tasks) == (4 * (nblk - 1) if uq == 2 else 0)
        assert kinds[D] == nblk
        assert len({tuple(t) for t in tasks.tolist()}) == len(tasks)
        upd = applied_panels(tasks, nblk)
        exp = [(q, i, j) for q in range(nblk) for j in range(q + 2, yb + 1) for i in range(j, yb + 1)]
        assert sorted(upd) == sorted(exp)           # every (panel, tile) update exactly once
        if group > 1 and nblk >= 2 * group + 2:
            assert (tasks[(tasks[:, 0] & 3) == BLK, 0] >> 2).max() == group - 1   # deep updates are used
        for _ in range(3):
            simulate(tasks, nsl, grid, rng)


@pytest.mark.parametrize("n,m", [(200, 0), (600, 50), (1100, 0), (2100, 40)])
@pytest.mark.parametrize("group,uq", [(1, 0), (4, 1), (4, 2)])
def test_chain_plan_reproduces_the_blocked_factorisation(n, m, group, uq):
    _lib_or_skip()
    rng = np.random.default_rng(7)
    n_pad, y_row, p = shape(n, m)
    W0, (xt, xs, y, noise, k) = augmented(n, m, rng)
    tasks = plan(n_pad, y_row, 64, group, uq)
    W = run_tasks(W0.copy(), tasks, n_pad // NB)
    Kn = k(xt, xt) + noise * np.eye(n)
    L = np.linalg.cholesky(Kn)
    np.testing.assert_allclose(np.tril(W[:n, :n]), L, rtol=0, atol=1e-12)
    z = np.linalg.solve(L, y)
    np.testing.assert_allclose(W[y_row, :n], z, rtol=0, atol=1e-10)
    assert W[y_row, y_row] == pytest.approx(-z @ z, rel=1e-12)
    if m:
        alpha = np.linalg.solve(Kn, y)
        Ks = k(xs, xt)
        np.testing.assert_allclose(-W[y_row, n_pad:n_pad + m], Ks @ alpha, rtol=0, atol=1e-9)
        V = np.linalg.solve(L, Ks.T)
        sig = k(xs, xs) - V.T @ V
        np.testing.assert_allclose(np.diag(W[n_pad:n_pad + m, n_pad:n_pad + m]), np.diag(sig), rtol=0, atol=1e-9)


@pytest.mark.parametrize("n,m", [(300, 0), (1000, 37), (3000, 0), (8192, 0)])
def test_chain_plan_f32_is_the_slice_update_plan(n, m):
    """GPK_CHAIN_PLAN_F32 (chain_kernel<float>, which has no quarter-task bodies): whatever chain_uq says, one U32 per
    slice and no SQ task -- the plan chain_uq 0 gives at the f32 depth (8 panels unless chain_group is set) -- and
    it reproduces the blocked factorisation; with identity rows the flag is refused."""
    _lib_or_skip()
    n_pad, y_row, p = shape(n, m)
    nblk = n_pad // NB
    for uq in (0, 1, 2):
        with nat.thread_tune(chain_uq=uq, chain_u128=0, chain_s128=0):
            t32 = nat.chain_plan(n_pad, y_row, 64, f32=True)
        assert np.array_equal(t32, plan(n_pad, y_row, 64, 8, uq=0))
        assert not any(is_sq(t) for t in t32)
        assert int(np.sum(((t32[:, 0] & 3) == U32) & (((t32[:, 0] >> 2) & 15) > 0))) == 0
    if nblk >= 18:
        assert (t32[(t32[:, 0] & 3) == BLK, 0] >> 2).max() == 7
    with nat.thread_tune(chain_group=4, chain_u128=0, chain_s128=0):
        assert np.array_equal(nat.chain_plan(n_pad, y_row, 64, f32=True), plan(n_pad, y_row, 64, 4, uq=0))
    if n <= 3000:
        rng = np.random.default_rng(11)
        simulate(t32, y_row // SL + 1, 16, rng)
        W0, (xt, xs, y, noise, k) = augmented(n, m, rng)
        W = run_tasks(W0.copy(), t32, nblk)
        np.testing.assert_allclose(np.tril(W[:n, :n]), np.linalg.cholesky(k(xt, xt) + noise * np.eye(n)), rtol=0,
                                   atol=1e-12)
    with pytest.raises(nat.GpkError):
        nat.chain_plan(n_pad, n_pad + n, 64, eye=True, f32=True)


@pytest.mark.parametrize("n,m", [(300, 0), (1000, 200), (3000, 40)])
@pytest.mark.parametrize("group,near,uq,nla", [(8, 2, 1, 2), (8, 4, 0, 2), (4, 2, 1, 2), (16, 4, 2, 2), (8, 2, 1, 1),
                                                (4, 2, 0, 1)])
def test_chain_plan_near_subgroups(n, m, group, near, uq, nla):
    """chain_group_near: the tile updates of the columns too near the diagonal for the deferred group go in sub-groups
    of `near` panels under the same look-ahead rule -- every (panel, tile) update still exactly once, deeper tasks
    present, every wait covering its dependencies, and the blocked factorisation reproduced."""
    _lib_or_skip()
    n_pad, y_row, p = shape(n, m)
    nsl = y_row // SL + 1
    nblk, yb = n_pad // NB, y_row // NB
    rng = np.random.default_rng(n + near)
    with nat.thread_tune(chain_group_near=near, chain_near_la=nla):
        tasks = plan(n_pad, y_row, 16, group, uq)
    with nat.thread_tune(chain_group_near=1):
        base = plan(n_pad, y_row, 16, group, uq)
    upd = applied_panels(tasks, nblk)
    exp = [(q, i, j) for q in range(nblk) for j in range(q + 2, yb + 1) for i in range(j, yb + 1)]
    assert sorted(upd) == sorted(exp)
    g = ((tasks[:, 0] >> 2) & 15) + 1
    gb = ((base[:, 0] >> 2) & 15) + 1
    blk_t, blk_b = (tasks[:, 0] & 3) == BLK, (base[:, 0] & 3) == BLK
    assert int(np.sum(blk_t & (g == 1))) <= int(np.sum(blk_b & (gb == 1)))
    if nblk >= group + 4:
        assert int(np.sum(blk_t & (g == 1))) < int(np.sum(blk_b & (gb == 1)))
        assert int(np.sum(blk_t & (g == near))) > 0
    for _ in range(2):
        simulate(tasks, nsl, 16, rng)
    if n <= 1000:
        W0, (xt, xs, y, noise, k) = augmented(n, m, rng)
        W = run_tasks(W0.copy(), tasks, nblk)
        np.testing.assert_allclose(np.tril(W[:n, :n]), np.linalg.cholesky(k(xt, xt) + noise * np.eye(n)), rtol=0,
                                   atol=1e-12)


@pytest.mark.parametrize("n,m", [(300, 0), (1000, 200), (3000, 40)])
@pytest.mark.parametrize("uq", [0, 1, 2])
def test_chain_plan_u128_block_row_updates(n, m, uq):
    """chain_u128: below the next diagonal block the next panel's column is updated by one 128 x 128 tile task (BLK
    over one panel) per block row instead of four slice tasks -- every (panel, tile) update exactly once (the slice
    updates left only for the next diagonal block's slices), every wait covering its dependencies, and the blocked
    factorisation reproduced."""
    _lib_or_skip()
    n_pad, y_row, p = shape(n, m)
    nsl = y_row // SL + 1
    nblk, yb = n_pad // NB, y_row // NB
    rng = np.random.default_rng(n + uq)
    tasks = plan(n_pad, y_row, 16, 4, uq, u128=1)
    upd = applied_panels(tasks, nblk)
    exp = [(q, i, j) for q in range(nblk) for j in range(q + 2, yb + 1) for i in range(j, yb + 1)]
    exp += [(q, i, q + 1) for q in range(nblk) for i in range(q + 2, yb + 1)]
    assert sorted(upd) == sorted(exp)
    for t in tasks:
        ty, k, r, j, g = decode(t)
        if ty == U32:
            assert r < 4 * (k + 2)           # only the next diagonal block's slices
    for _ in range(2):
        simulate(tasks, nsl, 16, rng)
    if n <= 1000:
        W0, (xt, xs, y, noise, k) = augmented(n, m, rng)
        W = run_tasks(W0.copy(), tasks, nblk)
        np.testing.assert_allclose(np.tril(W[:n, :n]), np.linalg.cholesky(k(xt, xt) + noise * np.eye(n)), rtol=0,
                                   atol=1e-12)


@pytest.mark.parametrize("n,m", [(300, 0), (1000, 200), (3000, 40)])
@pytest.mark.parametrize("uq,u128", [(1, 1), (0, 0), (2, 1)])
def test_chain_plan_s128_block_row_solves(n, m, uq, u128):
    """chain_s128: below the next diagonal block a block row's slices take one panel-solve task (S with g = its slice
    count) -- every slice of every panel solved exactly once, every wait covering its dependencies, the blocked
    factorisation reproduced."""
    _lib_or_skip()
    n_pad, y_row, p = shape(n, m)
    nsl = y_row // SL + 1
    nblk = n_pad // NB
    rng = np.random.default_rng(n + uq)
    tasks = plan(n_pad, y_row, 16, 4, uq, u128=u128, s128=1)
    solved = []
    for t in tasks:
        ty, k, r, j, g = decode(t)
        if ty == S:
            solved += [(k, r + i) for i in range(g)]
            if g > 1:
                assert r % 4 == 0 and r >= 4 * (k + 2)
    exp = [(k, r) for k in range(nblk) for r in range(4 * (k + 1), nsl)]
    assert sorted(solved) == sorted(exp)
    if nblk >= 3:
        assert any(decode(t)[0] == S and decode(t)[4] > 1 for t in tasks)
    for _ in range(2):
        simulate(tasks, nsl, 16, rng)
    if n <= 1000:
        W0, (xt, xs, y, noise, k) = augmented(n, m, rng)
        W = run_tasks(W0.copy(), tasks, nblk)
        np.testing.assert_allclose(np.tril(W[:n, :n]), np.linalg.cholesky(k(xt, xt) + noise * np.eye(n)), rtol=0,
                                   atol=1e-12)


def test_chain_plan_u128_auto():
    """chain_u128 2 (auto, the default): slice updates for short chains on a full grid (fewer than 48 diagonal blocks and
    more than two workgroups per diagonal block), block-row updates otherwise."""
    _lib_or_skip()

    def has_row_updates(n, grid):
        n_pad, y_row, _ = shape(n, 0)
        with nat.thread_tune(chain_u128=2):
            t = nat.chain_plan(n_pad, y_row, grid)
        return any(decode(x)[0] == BLK and decode(x)[3] == decode(x)[1] + 1 for x in t)

    def has_row_solves(n, grid):
        n_pad, y_row, _ = shape(n, 0)
        with nat.thread_tune(chain_s128=2):
            t = nat.chain_plan(n_pad, y_row, grid)
        return any(decode(x)[0] == S and decode(x)[4] > 1 for x in t)

    assert has_row_solves(8192, 64) and has_row_solves(4096, 64)
    assert not has_row_solves(8192, 256) and not has_row_solves(4096, 256)
    with nat.thread_tune(chain_s128=2):
        te = nat.chain_plan(8192, 2 * 8192, 256, True)
        te4 = nat.chain_plan(4096, 2 * 4096, 256, True)
    assert any(decode(x)[0] == S and decode(x)[4] > 1 for x in te)
    assert not any(decode(x)[0] == S and decode(x)[4] > 1 for x in te4)
    assert not has_row_updates(4096, 256)
    assert has_row_updates(4096, 64)
    assert has_row_updates(8192, 256)
    assert not has_row_updates(2048, 256)


def test_chain_plan_eye_near_subgroups():
    _lib_or_skip()
    n = 1500
    n_pad = -(-n // NB) * NB
    y_row = n_pad + n
    rng = np.random.default_rng(5)
    for u128 in (0, 1):
        with nat.thread_tune(chain_group_near=2, chain_group_eye=8, chain_group=8, chain_u128=u128):
            tasks = nat.chain_plan(n_pad, y_row, 16, True)
        for _ in range(2):
            simulate(tasks, y_row // SL + 1, 16, rng)


def test_chain_plan_rejects_bad_shapes():
    _lib_or_skip()
    with pytest.raises(nat.GpkError):
        nat.chain_plan(100, 100, 8)
    with pytest.raises(nat.GpkError):
        nat.chain_plan(128, 100, 8)


def test_chain_plan_error_codes_name_each_entry_points_own_argument():
    """gpk.h: -i means the i-th argument of the called entry point.  gpk_chain_plan(n_pad, y_row, grid, tasks_out,
    cap, ntasks) and gpk_chain_plan_ex(n_pad, y_row, grid, flags, tasks_out, cap, ntasks) put cap / ntasks at
    positions 5 / 6 and 6 / 7."""
    import ctypes
    _lib_or_skip()
    L = nat.load_library()
    nt = ctypes.c_int64(0)
    buf = (ctypes.c_int32 * 4)()
    assert L.gpk_chain_plan(1024, 1024, 8, None, 0, None) == -6
    assert L.gpk_chain_plan_ex(1024, 1024, 8, 0, None, 0, None) == -7
    assert L.gpk_chain_plan(1024, 1024, 8, buf, 1, ctypes.byref(nt)) == -5     # cap below the task count
    assert L.gpk_chain_plan_ex(1024, 1024, 8, 0, buf, 1, ctypes.byref(nt)) == -6
    assert nt.value > 1
    assert L.gpk_chain_plan(1024, 1024, 0, None, 0, ctypes.byref(nt)) == -3
    assert L.gpk_chain_plan_ex(1024, 1024, 8, 1 << 20, None, 0, ctypes.byref(nt)) == -4
    assert L.gpk_chain_plan(1024, 1024, 8, None, 0, ctypes.byref(nt)) == 0


def test_chain_plan_corner_knobs_are_tune_knobs():
    """The identity-augmented planner's corner grouping (chain_group_corner, chain_corner_tail, chain_group_la) are
    gpk_tune knobs, read per call (and part of the device plan cache key): changing them changes the list that
    gpk_chain_plan_ex returns, and every list still applies each live update once."""
    _lib_or_skip()
    n = 3000
    n_pad = -(-n // NB) * NB
    y_row = n_pad + n
    nblk, yb = n_pad // NB, y_row // NB
    base = plan(n_pad, y_row, 64, 4, 1, eye=True)
    for knobs in ({"chain_group_corner": 4}, {"chain_corner_tail": 0}, {"chain_group_la": 3}):
        with nat.thread_tune(**knobs):
            alt = plan(n_pad, y_row, 64, 4, 1, eye=True)
        assert alt.shape != base.shape or not np.array_equal(alt, base), knobs
        upd = applied_panels(alt, nblk)
        assert len(upd) == len(set(upd))
        live = {(q, i, j) for q in range(nblk) for j in range(q + 2, yb + 1) for i in range(j, yb + 1)
                if eye_live(i, q, nblk, yb) and eye_live(j, q, nblk, yb)}
        assert live <= set(upd)
    assert np.array_equal(plan(n_pad, y_row, 64, 4, 1, eye=True), base)   # restored knobs, the same list


# ------------------------------------------------------------------ identity-augmented lists (gradient path)
def eye_live(i, q, nblk, yb):
    """Block i holds a nonzero row in panel q's columns: training blocks always, the y row's block always, extra
    block e = i - nblk from panel e on (row n_pad + t of E L^-T is zero left of column t)."""
    return i < nblk or i == yb or i - nblk <= q


def augmented_eye(n, rng):
    n_pad = -(-n // NB) * NB
    y_row = n_pad + n
    p = -(-(y_row + 1) // NB) * NB
    x = np.sort(rng.uniform(0, 1, n))
    Kn = np.exp(-0.5 * (x[:, None] - x[None, :]) ** 2 / 0.1 ** 2) + 1e-2 * np.eye(n)
    y = np.sin(6 * x) + 0.1 * rng.standard_normal(n)
    W = np.zeros((p, p))
    W[:n, :n] = Kn
    W[n:n_pad, n:n_pad] = np.eye(n_pad - n)
    W[n_pad:n_pad + n, :n] = np.eye(n)
    W[y_row, :n] = y
    return np.tril(W), Kn, y, n_pad, y_row


@pytest.mark.parametrize("n", [1, 100, 128, 300, 700, 1000, 1500])
@pytest.mark.parametrize("group,uq", [(1, 1), (4, 1), (8, 0), (4, 2)])
def test_chain_plan_eye_waits_cover_every_dependency(n, group, uq):
    """The identity-augmented list: every live (panel, tile) update exactly once, dead ones only as zero panels
    inside a group whose last panel is live, no panel solve of a still-zero slice, and the waits -- with the
    first-update bit -- cover every dependency under random durations."""
    _lib_or_skip()
    n_pad = -(-n // NB) * NB
    y_row = n_pad + n
    nsl = y_row // SL + 1
    nblk, yb = n_pad // NB, y_row // NB
    rng = np.random.default_rng(n)
    for grid in (1, 5, 64, 256):
        tasks = plan(n_pad, y_row, grid, group, uq, eye=True)
        assert len({tuple(t) for t in tasks.tolist()}) == len(tasks)
        assert np.bincount(tasks[:, 0] & 3, minlength=4)[D] == nblk
        for t in tasks:
            ty, k, r, j, g = decode(t)
            if ty == S:
                assert eye_live(r // 4, k, nblk, yb)
            if ty == BLK:
                assert eye_live(r, k + g - 1, nblk, yb) and eye_live(j, k + g - 1, nblk, yb)
        upd = applied_panels(tasks, nblk)
        assert len(upd) == len(set(upd))
        live = {(q, i, j) for q in range(nblk) for j in range(q + 2, yb + 1) for i in range(j, yb + 1)
                if eye_live(i, q, nblk, yb) and eye_live(j, q, nblk, yb)}
        assert live <= set(upd)
        for q, i, j in set(upd) - live:
            assert j >= q + 2 and i >= j
        for _ in range(2):
            simulate(tasks, nsl, grid, rng)


@pytest.mark.parametrize("n", [200, 300, 1100])
@pytest.mark.parametrize("group,uq,rows", [(1, 0, 0), (4, 1, 0), (4, 2, 0), (4, 1, 1)])
def test_chain_plan_eye_reproduces_the_inverse(n, group, uq, rows):
    """Run in list order on the identity-augmented matrix: L, the extra rows L^-T, the corner -K^-1 and its y row
    -alpha^T (the layout gpk_nlml_grad reads, include/gpk.h); rows: with block-row updates and panel solves."""
    _lib_or_skip()
    rng = np.random.default_rng(11)
    W0, Kn, y, n_pad, y_row = augmented_eye(n, rng)
    tasks = plan(n_pad, y_row, 64, group, uq, eye=True, u128=rows, s128=rows)
    if rows:
        for _ in range(2):
            simulate(tasks, y_row // SL + 1, 16, rng)
    W = run_tasks(W0.copy(), tasks, n_pad // NB)
    L = np.linalg.cholesky(Kn)
    np.testing.assert_allclose(np.tril(W[:n, :n]), L, rtol=0, atol=1e-12)
    Linv = np.linalg.inv(L)
    np.testing.assert_allclose(W[n_pad:n_pad + n, :n], Linv.T, rtol=0, atol=1e-9 * np.abs(Linv).max())
    Kinv = np.linalg.inv(Kn)
    got = np.tril(W[n_pad:n_pad + n, n_pad:n_pad + n])
    np.testing.assert_allclose(got, -np.tril(Kinv), rtol=0, atol=1e-9 * np.abs(Kinv).max())
    np.testing.assert_allclose(-W[y_row, n_pad:n_pad + n], Kinv @ y, rtol=0, atol=1e-8 * np.abs(Kinv @ y).max())


# ------------------------------------------------------------------ two task lists (gpk_tune "chain_xcd")
def split_lists(tasks):
    """chain_split_lists (gpk_abi.hip): the diagonal chain's tasks -- D, the panel solves of the next diagonal block's
    slices, its quarter updates (or per-slice updates) -- to list B, in order; the rest is list A."""
    la, lb = [], []
    for t in tasks:
        ty, k, r, j, g = decode(t)
        chain = ty == D or (ty == S and r // 4 == k + 1) or (ty == U32 and (g > 1 or (j == k + 1 and r // 4 == k + 1)))
        (lb if chain else la).append(t)
    return la, lb


def simulate_two_lists(tasks, nsl, wa, wb, rng):
    """Discrete-event run of chain_kernel's claim rule with two lists: wa workgroups claim list A first, wb list B
    first, a workgroup whose list is exhausted claims from the other; a claimed task starts once every counter it
    waits for is published.  Asserts progress (no state where claimed tasks wait on counters that no running task
    will publish and no free workgroup can claim) and, at every start, that each cell the task reads or writes holds
    the version the one-list (topological) order would give it."""
    uq = 2 if any(is_sq(t) for t in tasks) else any(decode(t)[0] == U32 and decode(t)[4] > 1 for t in tasks)
    order = {tuple(t): i for i, t in enumerate(tasks)}
    la, lb = split_lists(tasks)
    lists = [la, lb]
    nxt = [0, 0]
    writers, readers = {}, {}
    for i, t in enumerate(tasks):
        rd, wr = cells(t, nsl, uq)
        for c in wr:
            writers.setdefault(c, []).append(i)
        for c in rd - wr:
            readers.setdefault(c, []).append(i)
    pub = {}
    finished = set()
    dur = {D: 28.0, S: 7.0, U32: 7.0, BLK: 18.0}
    workers = [{"lst": 0, "sw": False, "task": None, "run": False, "done": False} for _ in range(wa)] + \
              [{"lst": 1, "sw": False, "task": None, "run": False, "done": False} for _ in range(wb)]
    running = []   # (finish time, worker index)
    now = 0.0

    def ready(task):
        for cnt, idx, v in waits(task, nsl, uq):
            got = pub.get((cnt, idx))
            if isinstance(v, int) and v == 0:
                continue
            if got is None or got < v:
                return False
        return True

    while True:
        for w in workers:
            while w["task"] is None and not w["done"]:
                l = w["lst"]
                if nxt[l] < len(lists[l]):
                    w["task"] = lists[l][nxt[l]]
                    nxt[l] += 1
                elif not w["sw"]:
                    w["sw"] = True
                    w["lst"] ^= 1
                else:
                    w["done"] = True
        for wi, w in enumerate(workers):
            if w["task"] is not None and not w["run"] and ready(w["task"]):
                x = order[tuple(w["task"])]
                rd, wr = cells(w["task"], nsl, uq)
                for c in rd | wr:   # every earlier writer finished, no later one
                    for i in writers.get(c, []):
                        assert (i in finished) == (i < x), "task %d %s: cell %s writer %d" % (x, w["task"], c, i)
                for c in wr:        # every earlier reader since ... finished (write-after-read)
                    for i in readers.get(c, []):
                        if i < x:
                            assert i in finished, "task %d %s overwrites %s under reader %d" % (x, w["task"], c, i)
                w["run"] = True
                ty, g = decode(w["task"])[0], decode(w["task"])[4]
                heapq.heappush(running, (now + dur[ty] * g * rng.uniform(0.3, 3.0), wi))
        if not running:
            stuck = [w["task"] for w in workers if w["task"] is not None]
            assert not stuck, "deadlock: %d claimed tasks wait, nothing runs (first %s)" % (len(stuck), stuck[0])
            assert nxt[0] == len(la) and nxt[1] == len(lb)
            return
        now, wi = heapq.heappop(running)
        w = workers[wi]
        x = order[tuple(w["task"])]
        finished.add(x)
        for cnt, idx, v in publishes(w["task"], nsl):
            if v == "+1":
                pub[(cnt, idx)] = pub.get((cnt, idx), 0) + 1
            else:
                pub[(cnt, idx)] = max(pub.get((cnt, idx), 0), v)
        w["task"], w["run"] = None, False


@pytest.mark.parametrize("n,m", [(300, 0), (1000, 200), (2048, 0), (3000, 40)])
@pytest.mark.parametrize("group,uq", [(4, 1), (8, 1), (1, 0), (4, 2)])
def test_chain_plan_two_lists_progress_and_order(n, m, group, uq):
    """gpk_tune("chain_xcd"): the diagonal chain's tasks as a second list claimed first by a few workgroups of one
    XCD.  Both lists are subsequences of the planner's topological order; with at least one workgroup per role every
    run completes and every task sees the one-list versions of its cells (random durations, several pool sizes)."""
    _lib_or_skip()
    n_pad, y_row, p = shape(n, m)
    nsl = y_row // SL + 1
    rng = np.random.default_rng(n + m + group)
    for grid in (64, 256):
        tasks = [tuple(int(v) for v in t) for t in plan(n_pad, y_row, grid, group, uq)]
        la, lb = split_lists(tasks)
        assert len(lb) >= n_pad // NB and all(decode(t)[0] != BLK for t in lb)
        for wa, wb in ((1, 1), (grid - 4, 4), (grid - 16, 16)):
            simulate_two_lists(tasks, nsl, wa, wb, rng)
