"""Ragged batches and the segmented models on the HIP path vs the CPU oracle (needs the MI355X).

SURVEY §8f.2 (blockwise / partitioned LML: a variable-size batched factorisation) and §8f.3
(BIC / MSE / cross-validation wrappers).  Tolerances as tests/test_gpu_parity.py: NLL rel <= 1e-9
at noise >= 1e-2; kernel matrices |dK| <= 1e-13 + 1e-12 |K|; factors / alphas / posteriors
max-abs <= 1e-9 (well-conditioned segments, noise 1e-2)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import gp_oracle as o
from tests.helpers import hyp_list, make_kernel
from tests.test_segmented_host import Interval

import gaussianprocessfundamentals_amd.global_parameters as gp
from gaussianprocessfundamentals_amd import _native as nat
from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd.DataHandling.DataInput import BlockwiseDataInput, DataInput
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk
from gaussianprocessfundamentals_amd.KernelBasics import Operators as ops
from gaussianprocessfundamentals_amd.KernelBasics import PartitioningModel as pm
from gaussianprocessfundamentals_amd.KernelBasics.PartitionOperator import PartitionOperator
from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction
from gaussianprocessfundamentals_amd.Metrics import CrossValidation as cv
from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type
from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType
from gaussianprocessfundamentals_amd.Metrics import MatrixHandlingTypes as mht
from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import (BlockwiseGaussianProcess, GaussianProcess,
                                                                        PartitionedGaussianProcess)

pytestmark = pytest.mark.gpu

SE = ("SE", {"ard": False})
PER = ("PER", {})
MAT52 = ("MAT52", {})
NOISE = 1e-2


def T(v):
    return torch.tensor(v, dtype=torch.float64)


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


def segment_data(n, seed, lo=0.0, hi=1.0, d=1):
    rng = np.random.default_rng(seed)
    x = np.sort(rng.uniform(lo, hi, n)).reshape(n, 1) if d == 1 else rng.uniform(lo, hi, (n, d))
    y = np.sin(4 * np.pi * x[:, 0]) + 0.1 * rng.standard_normal(n)
    return x, y


# ------------------------------------------------------------------------------ raw ragged engine
RAGGED_SIZES = [300, 1000, 129, 128, 1, 700, 257]


def ragged_members(trees_hyps, sizes, test_sizes=None, d=1):
    members, data = [], []
    for b, n in enumerate(sizes):
        tree, hyp = trees_hyps[b % len(trees_hyps)]
        x, y = segment_data(n, 100 + b, d=d)
        xs = segment_data(test_sizes[b], 200 + b, d=d)[0] if test_sizes and test_sizes[b] else None
        k = make_kernel(tree, d)
        kd = engine.kernel_descriptor(k, d)
        h = engine.pack_hyper_parameter(hyp_list(hyp), kd.n_hyp)
        dev = engine.device()
        members.append((kd, h, torch.tensor(x, device=dev), torch.tensor(y, device=dev),
                        torch.tensor(xs, device=dev) if xs is not None else None))
        data.append((tree, hyp, x, y, xs))
    return members, data


@pytest.mark.parametrize("trees_hyps", [
    [(SE, [0.1])],
    [(SE, [0.1]), (SE, [0.05]), (SE, [0.3])],                        # one program, per-member hyp
    [(SE, [0.1]), (PER, [0.8, 0.5]), (("ADD", [SE, MAT52]), [0.2, 0.4])],  # per-member programs
])
def test_ragged_nlml_factor_alpha_match_oracle(trees_hyps):
    members, data = ragged_members(trees_hyps, RAGGED_SIZES)
    f = engine.RaggedFactorization(RAGGED_SIZES, 1)
    f.run(members, T(NOISE))
    f.check_info()
    nl = f.nlml().cpu().numpy()
    assert np.array_equal(f.out.view(-1, 4)[:, 3].cpu().numpy(), np.array(RAGGED_SIZES, dtype=np.float64))
    alphas = f.alphas()
    for b, (tree, hyp, x, y, _) in enumerate(data):
        c = o.nlml_components(tree, hyp, NOISE, x, y)
        assert rel(float(nl[b]), c["nlml"]) < 1e-9, (b, float(nl[b]), c["nlml"])
        assert np.max(np.abs(f.cholesky(b).cpu().numpy() - c["L"])) < 1e-9
        assert np.max(np.abs(alphas[b].cpu().numpy() - c["alpha"].reshape(-1))) < 1e-8 * max(1, np.abs(c["alpha"]).max())


def test_ragged_posterior_with_test_rows():
    sizes, tsz = [400, 130, 900], [50, 0, 129]
    members, data = ragged_members([(SE, [0.1]), (MAT52, [0.3])], sizes, tsz)
    f = engine.RaggedFactorization(sizes, 1, tsz)
    f.run(members, T(NOISE))
    f.check_info()
    for b, (tree, hyp, x, y, xs) in enumerate(data):
        assert rel(float(f.nlml()[b]), o.nlml(tree, hyp, NOISE, x, y)) < 1e-9
        if xs is None:
            assert f.posterior_mu(b).numel() == 0
            continue
        mu, var = o.posterior(tree, hyp, NOISE, x, y, xs)
        assert np.max(np.abs(f.posterior_mu(b).cpu().numpy() - mu)) < 1e-8
        assert np.max(np.abs(f.corner(b).cpu().numpy() - var)) < 1e-8
        assert np.max(np.abs(f.posterior_var_diag(b).cpu().numpy() - np.diag(var))) < 1e-8


def test_ragged_equals_uniform_batch_and_reports_failures():
    """A ragged batch whose members all have the same size reproduces the uniform batched path
    bit for bit; a member that is not positive definite reports info > 0 (only that member)."""
    sizes = [256, 256, 256]
    members, data = ragged_members([(SE, [0.1])], sizes)
    f = engine.RaggedFactorization(sizes, 1)
    f.run(members, T(NOISE))
    g = engine.AugmentedFactorization(256, 1, 0, 3)
    X = torch.stack([m[2] for m in members]).contiguous()
    Y = torch.stack([m[3] for m in members]).contiguous()
    H = torch.stack([m[1] for m in members]).contiguous()
    g.run(members[0][0], H, H.shape[1], T(NOISE).reshape(1).to(X.device), 0, X, 256, Y, 256)
    assert torch.equal(f.nlml(), g.nlml())
    # member 1: PER with p = 1e-9 on duplicated points and zero noise -> not PD
    bad = list(members)
    x1 = torch.zeros_like(members[1][2])
    kd = engine.kernel_descriptor(make_kernel(SE, 1), 1)
    bad[1] = (kd, engine.pack_hyper_parameter(hyp_list([0.1]), 1), x1, members[1][3], None)
    f2 = engine.RaggedFactorization(sizes, 1)
    f2.run(bad, torch.tensor([NOISE, -1.0, NOISE], dtype=torch.float64))
    info = f2.info.cpu().numpy()
    assert info[0] == 0 and info[1] > 0 and info[2] == 0
    assert torch.isinf(f2.nlml()[1]) and torch.isfinite(f2.nlml()[0])


def test_ragged_abi_rejects_missing_sizes():
    lay = nat.plan(nat.GPK_F64, 2, 100, 0, 1)
    L = nat.lib()
    assert L.gpk_potrf_aug_ragged(ctypes.byref(lay), None, None, None, None, None, None) < 0
    assert L.gpk_finalize_ragged(ctypes.byref(lay), None, None, None, None, None, None, None) < 0


# ------------------------------------------------------------------------------ operators
@pytest.mark.parametrize("mode", ["INDICATOR", "SIGMOID", "APPROX_INDICATOR"])
def test_change_point_operator_matrix(mode):
    gp.p_cp_operator_type = getattr(gp.ChangePointOperatorType, mode)
    try:
        x, _ = segment_data(300, 1)
        xs, _ = segment_data(77, 2)
        k = ops.ChangePointOperator(1, [bk.SquaredExponentialKernel(1), bk.PeriodicKernel(1),
                                        bk.MaternKernel5_2(1)], [0.3, 0.65])
        hyp = [0.31, 0.62, 0.1, 0.7, 0.4, 0.25]
        K = k.get_tf_tensor(hyp_list(hyp), x, xs).cpu().numpy()
        ref = o.change_point_matrix([SE, PER, MAT52], [[0.1], [0.7, 0.4], [0.25]], [0.31, 0.62], x, xs, mode)
        assert np.max(np.abs(K - ref) - (1e-13 + 1e-12 * np.abs(ref))) <= 0
    finally:
        gp.p_cp_operator_type = gp.ChangePointOperatorType.INDICATOR


def test_partition_operator_block_matrix():
    model = pm.PartitioningModel(pm.PartitioningClass.SELF_SUFFICIENT, [])
    for lo, hi in [(0.0, 0.4), (0.4, 0.7), (0.7, 1.1)]:
        model.add_partitioning_criterion(Interval(lo, hi))
    k = PartitionOperator(1, [bk.SquaredExponentialKernel(1), bk.MaternKernel5_2(1), bk.PeriodicKernel(1)], model)
    rng = np.random.default_rng(3)
    x = rng.uniform(0, 1, (200, 1))
    K = k.get_tf_tensor(hyp_list([0.1, 0.3, 0.5, 0.6]), x, x).cpu().numpy()
    idx = model.get_data_record_indices_per_partition(x)
    blocks = [o.kernel_matrix(t, h, x[i], x[i]) for t, h, i in zip([SE, MAT52, PER], [[0.1], [0.3], [0.5, 0.6]], idx)]
    from scipy.linalg import block_diag
    ref = block_diag(*blocks)
    assert K.shape == ref.shape
    assert np.max(np.abs(K - ref) - (1e-13 + 1e-12 * np.abs(ref))) <= 0


# ------------------------------------------------------------------------------ segmented GPs
def blockwise_setup(n=1500, n_test=300, cps=(0.25, 0.6), seed=5):
    rng = np.random.default_rng(seed)
    x = np.sort(rng.uniform(0, 1, n)).reshape(-1, 1)
    y = np.where(x[:, 0] < 0.5, np.sin(8 * x[:, 0]), np.cos(3 * x[:, 0])) + 0.05 * rng.standard_normal(n)
    xt = np.sort(rng.uniform(0, 1, n_test)).reshape(-1, 1)
    yt = np.where(xt[:, 0] < 0.5, np.sin(8 * xt[:, 0]), np.cos(3 * xt[:, 0]))
    children = [bk.SquaredExponentialKernel(1), bk.MaternKernel5_2(1), bk.PeriodicKernel(1)]
    kernel = ops.ChangePointOperator(1, children, [T(c) for c in cps])
    di = BlockwiseDataInput(x, y.reshape(-1, 1), xt, yt.reshape(-1, 1), [T(c) for c in cps])
    di.set_mean_function(ZeroMeanFunction(1))
    g = BlockwiseGaussianProcess(kernel, ZeroMeanFunction(1))
    g.set_data_input(di)
    segs = []
    for i in range(len(cps) + 1):
        lo = cps[i - 1] if i else -np.inf
        hi = cps[i] if i < len(cps) else np.inf
        a, b = (x[:, 0] >= lo) & (x[:, 0] < hi), (xt[:, 0] >= lo) & (xt[:, 0] < hi)
        segs.append((x[a], y[a], xt[b], yt[b]))
    return g, segs


CHILD_TREES = [SE, MAT52, PER]
CHILD_HYPS = [[0.08], [0.3], [0.9, 0.45]]


def test_blockwise_log_likelihood_sums_segments():
    g, segs = blockwise_setup()
    flat = [0.08, 0.3, 0.9, 0.45]   # children only: the reference slices from offset 0 (quirk)
    m = get_metric_by_type(MetricType.blockwise_LL, g)
    got = float(m.get_metric(hyp_list(flat), T(NOISE)))
    exp = o.blockwise_nlml([(t, h, s[0], s[1]) for t, h, s in zip(CHILD_TREES, CHILD_HYPS, segs)], NOISE)
    assert rel(got, exp) < 1e-9, (got, exp)
    # quirk: a full change-point list [cp1, cp2, children...] is sliced from 0 as well
    full = [0.25, 0.6] + flat
    got_q = float(m.get_metric(hyp_list(full), T(NOISE)))
    exp_q = o.blockwise_nlml([(SE, [0.25], segs[0][0], segs[0][1]), (MAT52, [0.6], segs[1][0], segs[1][1]),
                              (PER, [0.08, 0.3], segs[2][0], segs[2][1])], NOISE)
    assert rel(got_q, exp_q) < 1e-9
    bic = float(get_metric_by_type(MetricType.blockwise_BIC, g).get_metric(hyp_list(flat), T(NOISE)))
    assert rel(bic, o.bic(exp, 6, 1500)) < 1e-9
    mse = float(get_metric_by_type(MetricType.blockwise_MSE, g).get_metric(hyp_list(flat), T(NOISE)))
    exp_mu = np.concatenate([o.posterior(t, h, NOISE, s[0], s[1], s[2])[0] for t, h, s in zip(CHILD_TREES, CHILD_HYPS, segs)])
    exp_mse = float(np.mean((exp_mu - np.concatenate([s[3] for s in segs])) ** 2))
    assert rel(mse, exp_mse) < 1e-8


def test_segmented_covariance_matrix_getters():
    from scipy.linalg import block_diag
    g, segs = blockwise_setup(n=700, n_test=90)
    cm = g.covariance_matrix
    hyp = hyp_list([0.25, 0.6, 0.08, 0.3, 0.9, 0.45])   # SegmentedCovarianceMatrix skips the change points
    nz = T(NOISE)
    Kn = [o.k_noised(t, h, NOISE, s[0]) for t, h, s in zip(CHILD_TREES, CHILD_HYPS, segs)]
    Ls = [o.cholesky_lower(k) for k in Kn]
    tol = 1e-9
    assert np.max(np.abs(cm.get_K_noised(hyp, nz).cpu().numpy() - block_diag(*Kn))) < 1e-12
    assert np.max(np.abs(cm.get_L_K(hyp, nz).cpu().numpy() - block_diag(*Ls))) < tol
    alpha = np.concatenate([o.l_alpha(L, s[1].reshape(-1, 1)).reshape(-1) for L, s in zip(Ls, segs)])
    got_a = cm.get_L_alpha(hyp, nz).cpu().numpy().reshape(-1)
    assert np.max(np.abs(got_a - alpha)) < 1e-8 * max(1.0, np.abs(alpha).max())
    assert np.max(np.abs(cm.get_K_inv(hyp, nz).cpu().numpy() - block_diag(*[np.linalg.inv(k) for k in Kn]))) < 1e-6
    assert np.max(np.abs(cm.get_L_inv_K(hyp, nz).cpu().numpy() - block_diag(*[np.linalg.inv(L) for L in Ls]))) < 1e-6
    Kss = [o.kernel_matrix(t, h, s[2], s[2]) for t, h, s in zip(CHILD_TREES, CHILD_HYPS, segs)]
    assert np.max(np.abs(cm.get_K_ss(hyp).cpu().numpy() - block_diag(*Kss))) < 1e-12
    Lss = [o.cholesky_lower(k + NOISE * np.eye(k.shape[0])) for k in Kss]
    assert np.max(np.abs(cm.get_L_K_ss(hyp, nz).cpu().numpy() - block_diag(*Lss))) < tol
    # posterior of the segmented GP: mu concatenated, covariance block-diagonal
    post = [o.posterior(t, h, NOISE, s[0], s[1], s[2]) for t, h, s in zip(CHILD_TREES, CHILD_HYPS, segs)]
    mu = g.aux.get_posterior_mu(hyp, nz).cpu().numpy()
    assert np.max(np.abs(mu - np.concatenate([p[0] for p in post]))) < 1e-8
    var = g.aux.get_posterior_var(hyp, nz).cpu().numpy()
    assert np.max(np.abs(var - block_diag(*[p[1] for p in post]))) < 1e-8
    full, mean_mu, post_mu = g.predict(hyp, noise=nz)
    assert np.max(np.abs(post_mu.cpu().numpy() - np.concatenate([p[0] for p in post]))) < 1e-8
    # inv(L) K_s: block-diagonal of the segments' L_i^-1 K_s,i (Auxiliary.py:57-66 over the segments)
    Vs = [np.linalg.solve(L, o.kernel_matrix(t, h, s[0], s[2])) for L, t, h, s in zip(Ls, CHILD_TREES, CHILD_HYPS, segs)]
    g.aux.reset()
    V = g.aux.get_inverse_cholesky_k_times_k_s(hyp, nz).cpu().numpy()
    assert V.shape == (sum(v.shape[0] for v in Vs), sum(v.shape[1] for v in Vs))
    assert np.max(np.abs(V - block_diag(*Vs))) < 1e-8


def test_partitioned_gp_predict_and_empty_training_segment():
    model = pm.PartitioningModel(pm.PartitioningClass.SELF_SUFFICIENT, [])
    for lo, hi in [(0.0, 0.5), (0.5, 0.8), (0.8, 1.1)]:
        model.add_partitioning_criterion(Interval(lo, hi))
    rng = np.random.default_rng(9)
    x = rng.uniform(0, 0.8, (400, 1))                # nothing in the last partition's training set
    y = np.sin(5 * x[:, 0])
    xt = rng.uniform(0, 1, (60, 1))
    base = DataInput(x, y.reshape(-1, 1), xt, np.sin(5 * xt))
    pdi = model.partition_data_input(base)
    pdi.set_mean_function(ZeroMeanFunction(1))
    kernel = PartitionOperator(1, [bk.SquaredExponentialKernel(1), bk.SquaredExponentialKernel(1),
                                   bk.SquaredExponentialKernel(1)], model)
    g = PartitionedGaussianProcess(kernel, ZeroMeanFunction(1))
    g.set_data_input(pdi)
    hyp = hyp_list([0.1, 0.2, 0.3])
    _, _, post_mu = g.predict(hyp, noise=T(NOISE))
    tr = model.get_data_record_indices_per_partition(x)
    te = model.get_data_record_indices_per_partition(xt)
    exp = []
    for i, l in enumerate([0.1, 0.2, 0.3]):
        if len(tr[i]) == 0:
            exp.append(np.zeros(len(te[i])))
        else:
            exp.append(o.posterior(SE, [l], NOISE, x[tr[i]], y[tr[i]], xt[te[i]])[0])
    assert np.max(np.abs(post_mu.cpu().numpy() - np.concatenate(exp))) < 1e-8
    ll = float(get_metric_by_type(MetricType.blockwise_LL, g).get_metric(hyp, T(NOISE)))
    exp_ll = o.blockwise_nlml([(SE, [l], x[tr[i]], y[tr[i]]) for i, l in enumerate([0.1, 0.2, 0.3])], NOISE)
    assert rel(ll, exp_ll) < 1e-9


# ------------------------------------------------------------------------------ BIC / MSE / CV
def holistic(n=600, n_test=120, seed=4):
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, 1, (n, 1))
    y = np.sin(6 * x[:, 0]) + 0.1 * rng.standard_normal(n)
    xt = rng.uniform(0, 1, (n_test, 1))
    yt = np.sin(6 * xt[:, 0])
    di = DataInput(x, y.reshape(-1, 1), xt, yt.reshape(-1, 1))
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(make_kernel(SE, 1), ZeroMeanFunction(1))
    g.set_data_input(di)
    return g, x, y, xt, yt


def test_bic_and_mse_match_oracle():
    g, x, y, xt, yt = holistic()
    nl = o.nlml(SE, [0.15], NOISE, x, y)
    bic = get_metric_by_type(MetricType.BIC, g).get_metric(hyp_list([0.15]), T(NOISE))
    assert tuple(bic.shape) == (1, 1)
    assert rel(float(bic), o.bic(nl, 1, 600)) < 1e-9
    mse = get_metric_by_type(MetricType.MSE, g).get_metric(hyp_list([0.15]), T(NOISE))
    assert rel(float(mse), o.mse(SE, [0.15], NOISE, x, y, xt, yt)) < 1e-8


@pytest.mark.parametrize("metric", [MetricType.LL, MetricType.MSE, MetricType.BIC])
def test_cross_validation_matches_oracle_folds(metric):
    g, x, y, _, _ = holistic(n=503)
    g.kernel.set_last_hyper_parameter(hyp_list([0.15]))
    g.kernel.set_noise(T(NOISE))
    c = cv.CrossValidation(g, g.data_input, mht.MatrixApproximations.NONE,
                           mht.NumericalMatrixHandlingType.CHOLESKY_BASED, metric_type=metric)
    np.random.seed(11)
    got = c.cross_validation(0.2)
    np.random.seed(11)
    vals = []
    for tr, te in o.cv_folds(503, 0.2):
        if metric is MetricType.LL:
            vals.append(o.nlml(SE, [0.15], NOISE, x[tr], y[tr]))
        elif metric is MetricType.BIC:
            vals.append(o.bic(o.nlml(SE, [0.15], NOISE, x[tr], y[tr]), 1, len(tr)))
        else:
            vals.append(o.mse(SE, [0.15], NOISE, x[tr], y[tr], x[te], y[te]))
    assert rel(got, float(np.mean(vals))) < 1e-9


@pytest.mark.parametrize("approx,handling", [
    (mht.MatrixApproximations.NONE, mht.NumericalMatrixHandlingType.STRICT_INVERSE),
    (mht.MatrixApproximations.SKI, mht.NumericalMatrixHandlingType.CHOLESKY_BASED),
    (mht.MatrixApproximations.SKI, mht.NumericalMatrixHandlingType.STRICT_INVERSE)])
def test_blockwise_log_likelihood_per_segment_strategies(approx, handling):
    """Other strategies run one LogLikelihood per segment, as the reference always does
    (M/LogLikelihood.py:86-104): STRICT_INVERSE and SKI + CHOLESKY (= exact) give the exact sum;
    SKI + STRICT the sum of the per-segment SKI likelihoods (m = 10 % of each segment)."""
    g, segs = blockwise_setup(n=900, n_test=60)
    flat = [0.08, 0.3, 0.9, 0.45]
    m = get_metric_by_type(MetricType.blockwise_LL, g, approx, handling)
    got = float(m.get_metric(hyp_list(flat), T(NOISE)))
    if approx is mht.MatrixApproximations.SKI and handling is mht.NumericalMatrixHandlingType.STRICT_INVERSE:
        exp = sum(o.ski_nlml(t, h, NOISE, s[0], s[1], int(len(s[0]) * 0.1), handling="STRICT_INVERSE")
                  for t, h, s in zip(CHILD_TREES, CHILD_HYPS, segs))
    else:
        exp = o.blockwise_nlml([(t, h, s[0], s[1]) for t, h, s in zip(CHILD_TREES, CHILD_HYPS, segs)], NOISE)
    assert rel(got, exp) < 1e-9, (got, exp)


def test_cp_encapsulated_kernel_matches_oracle():
    # one child through get_cp_encapsulated_kernel (Operators.py:410-440): K * prev * ind ind'^T and
    # the complement mask; chaining both children reproduces the operator's matrix
    x = np.sort(np.random.default_rng(3).uniform(0, 1, 70)).reshape(-1, 1)
    a, b = bk.SquaredExponentialKernel(1), bk.MaternKernel5_2(1)
    cpo = ops.ChangePointOperator(1, [a, b], [0.4])
    K0, prev = cpo.get_cp_encapsulated_kernel(a, x, x, [0.2], 1.0, 0.4)
    K1, none = cpo.get_cp_encapsulated_kernel(b, x, x, [0.3], prev, None)
    ref = o.change_point_matrix([("SE", {}), ("MAT52", {})], [[0.2], [0.3]], [0.4], x, x)
    assert float(torch.max(torch.abs((K0 + K1).cpu() - torch.as_tensor(ref)))) <= 1e-13
    assert float(none) == 0.0
    full = cpo.get_tf_tensor([0.4, 0.2, 0.3], x, x)
    assert float(torch.max(torch.abs(full - (K0 + K1)))) <= 1e-14


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_ragged_paths_under_every_in_group_schedule(mode):
    """Ragged batches (per-member sizes, zero-row skipping) and test rows under the left-looking,
    right-looking and two-level in-group schedules: the same oracle bars as above."""
    old = nat.tune("ingroup", mode)
    try:
        test_ragged_nlml_factor_alpha_match_oracle([(SE, [0.1]), (PER, [0.8, 0.5]), (("ADD", [SE, MAT52]), [0.2, 0.4])])
        test_ragged_posterior_with_test_rows()
    finally:
        nat.tune("ingroup", old)
