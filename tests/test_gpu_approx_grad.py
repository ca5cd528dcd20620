"""Gradients through the approximations on the device (SURVEY §8f.1 x §8f.4): d(-LML)/d(hyperparameters,
noise, inducing inputs) under BASIC_NYSTROEM / SKC_LOWER_BOUND and SKI (STRICT / PSEUDO), as the reference's
VariationalSgdFitter takes them with tf.GradientTape over ``hyper_parameter + [indices]``
(gpbasics/Optimizer/Fitter.py:76-87, :124-132, :155-156).

Oracle: oracle/gp_autodiff.py (nystroem_nlml_and_grad / ski_nlml_and_grad: torch reverse mode of the restated
op sequence, pinned by finite differences in tests/test_grad_oracle.py).  Building blocks first:
gpk_kernel_vjp against torch autograd of the kernel program, gpk_pinv_backward_scale against autograd
through an SVD pseudo-inverse.  Tolerances (fp64): kernel VJP |g - g_ref| <= 1e-11 max|g_ref|; pinv
backward 1e-9 relative (condition <= 1e6); metric gradients 1e-7 max|g_ref| (well-conditioned K_mm) and
1e-5 for the SKC lower bound (its 1 / (2 jitter) = 5e7 factor amplifies the rounding of trace terms)."""
import numpy as np
import pytest
import torch

from oracle import gp_autodiff as ad
from oracle import gp_oracle as o
from tests.helpers import make_kernel, set_flags
from tests.test_grad_oracle import GRAD_CASES

from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd.DataHandling.DataInput import DataInput
from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction
from gaussianprocessfundamentals_amd.Metrics import MatrixHandlingTypes as mht
from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type
from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType
from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import GaussianProcess
import gaussianprocessfundamentals_amd.global_parameters as gpar

pytestmark = pytest.mark.gpu

A = mht.MatrixApproximations
H = mht.NumericalMatrixHandlingType
F64 = torch.float64


def _close(got, exp, tol):
    got, exp = np.asarray(got, dtype=np.float64), np.asarray(exp, dtype=np.float64)
    scale = max(1e-300, float(np.max(np.abs(exp))))
    assert float(np.max(np.abs(got - exp))) <= tol * scale, (got, exp)


# ------------------------------------------------------------------------------------ building blocks
@pytest.mark.parametrize("case", range(len(GRAD_CASES)))
def test_kernel_vjp_matches_autograd(case):
    tree, hyp, d, scaled, expanded = GRAD_CASES[case]
    set_flags(scaled=scaled, expanded=expanded)
    rng = np.random.default_rng(40 + case)
    x, z = rng.uniform(0, 1, (70, d)), rng.uniform(0, 1, (45, d))
    z[3] = x[5]                                        # a coincident pair: distance terms differentiate to 0
    G = rng.standard_normal((70, 45))
    params = [torch.tensor(np.asarray(h, dtype=np.float64), requires_grad=True) for h in hyp]
    Zt = torch.tensor(z, requires_grad=True)
    K = ad.kernel_matrix_t(tree, params, torch.tensor(x), Zt, scaled)
    gref = torch.autograd.grad(torch.sum(torch.tensor(G) * K), params + [Zt], retain_graph=True)
    kern = make_kernel(tree, d)
    gh, gz = engine.kernel_vjp(kern, [torch.tensor(h, dtype=F64) for h in hyp], x, z,
                               G=torch.tensor(G, device=engine.device()), want_z=True)
    _close(gh.cpu().numpy(), np.concatenate([g.numpy().reshape(-1) for g in gref[:-1]]), 1e-11)
    _close(gz.cpu().numpy(), gref[-1].numpy(), 1e-11)
    # rank-1 weights u v^T
    u, v = rng.standard_normal(70), rng.standard_normal(45)
    gh1, gz1 = engine.kernel_vjp(kern, [torch.tensor(h, dtype=F64) for h in hyp], x, z,
                                 gu=torch.tensor(u, device=engine.device()), gv=torch.tensor(v, device=engine.device()),
                                 want_z=True)
    gref1 = torch.autograd.grad(torch.sum(torch.tensor(np.outer(u, v)) * K), params + [Zt])
    _close(gh1.cpu().numpy(), np.concatenate([g.numpy().reshape(-1) for g in gref1[:-1]]), 1e-11)
    _close(gz1.cpu().numpy(), gref1[-1].numpy(), 1e-11)


@pytest.mark.parametrize("truncate", [False, True])
def test_pinv_backward_matches_autograd(truncate):
    rng = np.random.default_rng(5)
    m = 60
    Q, _ = np.linalg.qr(rng.standard_normal((m, m)))
    lam = np.geomspace(1.0, 1e-5, m)
    if truncate:
        lam[-15:] = 1e-17 * rng.uniform(0.5, 2.0, 15)    # below tf.linalg.pinv's cutoff 10 m eps
    Am = (Q * lam) @ Q.T
    Am = 0.5 * (Am + Am.T)
    Pbar = rng.standard_normal((m, m))
    if not truncate:
        At = torch.tensor(Am, requires_grad=True)
        ref = torch.autograd.grad(torch.sum(torch.tensor(Pbar) * ad.tf_pinv(At)), At)[0].numpy()
        ref = 0.5 * (ref + ref.T)                        # the adjoint of a symmetric input
    else:
        # truncated spectrum: torch's SVD backward divides by the zero gaps between the dropped singular
        # values (NaN; TensorFlow regularises that reciprocal).  Reference: the Daleckii-Krein derivative of
        # the fixed-rank pseudo-inverse from numpy's eigh (the formula the untruncated case pins above)
        lam_r, Vr = np.linalg.eigh(Am)
        keep = np.abs(lam_r) > 10 * m * np.finfo(np.float64).eps * np.abs(lam_r).max()
        f = np.where(keep, 1.0 / np.where(keep, lam_r, 1.0), 0.0)
        dl = lam_r[:, None] - lam_r[None, :]
        with np.errstate(divide="ignore", invalid="ignore"):
            F = np.where(keep[:, None] & keep[None, :], -np.outer(f, f),
                         np.where(keep[:, None] | keep[None, :], (f[:, None] - f[None, :]) / dl, 0.0))
        T = Vr.T @ Pbar @ Vr
        ref = Vr @ (F * 0.5 * (T + T.T)) @ Vr.T
    Ad = torch.tensor(Am, device=engine.device())
    lam_d, V, _ = engine.syevj(Ad)
    _, _, mu = engine.pinv_factor(lam_d, V, 0, return_mu=True)
    got = engine.pinv_backward(lam_d, V, mu, torch.tensor(Pbar, device=engine.device())).cpu().numpy()
    _close(got, ref, 1e-9)


# ------------------------------------------------------------------------------------ metric gradients
def _gp(tree, n=256, seed=3):
    x, y = o.make_inputs("C1", n=n, seed=seed)
    di = DataInput(x, y.reshape(-1, 1), x[:5], y[:5].reshape(-1, 1))
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(make_kernel(tree, 1), ZeroMeanFunction(1))
    g.set_data_input(di)
    return g, x, y


NYS_CASES = [
    # handling, lower bound, tree, hyp, scaled
    (H.CHOLESKY_BASED, False, ("SE", {}), [0.03], False),
    (H.CHOLESKY_BASED, True, ("SE", {}), [0.03, 1.3], True),
    (H.STRICT_INVERSE, False, ("MAT52", {}), [0.05], False),
    (H.PSEUDO_INVERSE, False, ("ADD", [("SE", {}), ("PER", {})]), [0.03, 0.5, 1.7], False),
    (H.STRICT_INVERSE, True, ("MAT32", {}), [0.04], False),
]


@pytest.mark.parametrize("case", range(len(NYS_CASES)))
def test_nystroem_gradient_matches_oracle(case):
    handling, lower, tree, hyp, scaled = NYS_CASES[case]
    set_flags(scaled=scaled)
    g, x, y = _gp(tree)
    m = 25
    z = np.sort(np.random.default_rng(case).uniform(0, 1, (m, 1)), axis=0)
    noise = 0.05
    jitter = float(gpar.p_cov_matrix_jitter)
    met = get_metric_by_type(MetricType.LL, g, A.SKC_LOWER_BOUND if lower else A.BASIC_NYSTROEM, handling,
                             subset_size=m)
    h = [torch.tensor(v, dtype=F64, requires_grad=True) for v in hyp]
    nz = torch.tensor(noise, dtype=F64, requires_grad=True)
    zt = torch.tensor(z, dtype=F64, requires_grad=True)
    out = met.get_metric(h, nz, zt)
    out.sum().backward()
    nl, gh, gn, gz = ad.nystroem_nlml_and_grad(tree, hyp, noise, x, y, z, handling.name, lower, jitter, scaled)
    assert abs(float(out) - nl) <= 1e-9 * abs(nl)
    tol = 1e-5 if lower else 1e-7
    _close([float(t.grad) for t in h] + [float(nz.grad)], [float(v) for v in gh] + [gn], tol)
    _close(zt.grad.numpy(), gz, tol)


def test_nystroem_cached_determinant_is_a_constant_for_the_tape():
    """The fitter's pattern (Fitter.py:120 then :124-132): the pre-fit call caches the Nystroem
    log-determinant outside the tape, so inside it only the exact data fit depends on the hyperparameters
    and nothing on the inducing inputs (BASIC_NYSTROEM + CHOLESKY_BASED) -- tape.gradient gives None there."""
    g, x, y = _gp(("SE", {}))
    m = 25
    z = np.sort(np.random.default_rng(1).uniform(0, 1, (m, 1)), axis=0)
    met = get_metric_by_type(MetricType.LL, g, A.BASIC_NYSTROEM, H.CHOLESKY_BASED, subset_size=m)
    met.get_metric([torch.tensor(0.03, dtype=F64)], torch.tensor(0.05, dtype=F64), torch.tensor(z))
    h = [torch.tensor(0.03, dtype=F64, requires_grad=True)]
    nz = torch.tensor(0.05, dtype=F64, requires_grad=True)
    zt = torch.tensor(z, dtype=F64, requires_grad=True)
    met.get_metric(h, nz, zt).sum().backward()
    _, gh, gn, gz = ad.nystroem_nlml_and_grad(("SE", {}), [0.03], 0.05, x, y, z, det_fresh=False)
    assert gz is None and zt.grad is None
    _close([float(h[0].grad), float(nz.grad)], [float(gh[0]), gn], 1e-7)


@pytest.mark.parametrize("handling", [H.STRICT_INVERSE, H.PSEUDO_INVERSE])
def test_ski_gradient_matches_oracle(handling):
    g, x, y = _gp(("SE", {}), n=200, seed=4)
    m = 40
    met = get_metric_by_type(MetricType.LL, g, A.SKI, handling, subset_size=m)
    h = [torch.tensor(0.08, dtype=F64, requires_grad=True)]
    nz = torch.tensor(0.05, dtype=F64, requires_grad=True)
    out = met.get_metric(h, nz)
    out.sum().backward()
    nl, gh, gn = ad.ski_nlml_and_grad(("SE", {}), [0.08], 0.05, x, y, m, handling.name)
    assert abs(float(out) - nl) <= 1e-9 * abs(nl)
    _close([float(h[0].grad), float(nz.grad)], [float(gh[0]), gn], 1e-7)


@pytest.mark.parametrize("approx", [A.BASIC_NYSTROEM, A.SKC_LOWER_BOUND, A.SKI])
def test_approximation_lcg_gradient_matches_oracle(approx):
    """LINEAR_CONJUGATE_GRADIENT on the approximate matrix (M/Metrics.py:141-147 with :95-105): the tape
    gradient through the executed CG iterations (linear_cg_backward) mapped through the Nystroem / SKI
    structure, against oracle/gp_autodiff (torch's tape of the same loop).  Noise 0.4 keeps the CG iterate
    insensitive to the device GEMV's rounding: value rel 1e-9, gradients 1e-6 max|g|."""
    g, x, y = _gp(("SE", {}), n=256, seed=6)
    m = 24
    noise = 0.4
    h = [torch.tensor(0.05, dtype=F64, requires_grad=True)]
    nz = torch.tensor(noise, dtype=F64, requires_grad=True)
    if approx is A.SKI:
        met = get_metric_by_type(MetricType.LL, g, A.SKI, H.LINEAR_CONJUGATE_GRADIENT, subset_size=m)
        out = met.get_metric(h, nz)
        out.sum().backward()
        nl, gh, gn = ad.ski_nlml_and_grad(("SE", {}), [0.05], noise, x, y, m, "LINEAR_CONJUGATE_GRADIENT")
    else:
        lower = approx is A.SKC_LOWER_BOUND
        # well-separated inducing inputs: two nearly coincident ones make K_mm's pinv split their adjoint
        # between them at the level of its conditioning (their sum stays exact)
        z = np.linspace(0.02, 0.98, m).reshape(-1, 1) + 0.003 * np.sin(np.arange(m)).reshape(-1, 1)
        zt = torch.tensor(z, dtype=F64, requires_grad=True)
        met = get_metric_by_type(MetricType.LL, g, approx, H.LINEAR_CONJUGATE_GRADIENT, subset_size=m)
        out = met.get_metric(h, nz, zt)
        out.sum().backward()
        nl, gh, gn, gz = ad.nystroem_nlml_and_grad(("SE", {}), [0.05], noise, x, y, z, "LINEAR_CONJUGATE_GRADIENT",
                                                   lower, float(gpar.p_cov_matrix_jitter))
        _close(zt.grad.numpy(), gz, 1e-5 if lower else 1e-6)
    assert abs(float(out) - nl) <= 1e-9 * abs(nl)
    _close([float(h[0].grad), float(nz.grad)], [float(gh[0]), gn], 1e-5 if approx is A.SKC_LOWER_BOUND else 1e-6)


def test_skc_upper_bound_gradient_matches_oracle():
    """SKC_UPPER_BOUND (M/SkcLogLikelihood.py:53-69) differentiated as the fitter's tape does: alpha from
    the VariationalSGD step is a constant; the first call computes K and the Nystroem determinant (both
    differentiated), a second call reuses the metric's caches (constants: no gradient at all)."""
    g, x, y = _gp(("SE", {}), n=200, seed=7)
    m = 20
    z = np.sort(np.random.default_rng(4).uniform(0, 1, (m, 1)), axis=0)
    met = get_metric_by_type(MetricType.LL, g, A.SKC_UPPER_BOUND, subset_size=m)
    h = [torch.tensor(0.06, dtype=F64, requires_grad=True)]
    nz = torch.tensor(0.05, dtype=F64, requires_grad=True)
    zt = torch.tensor(z, dtype=F64, requires_grad=True)
    out = met.get_metric(h, nz, zt)
    out.sum().backward()
    val, gh, gn, gz = ad.skc_upper_nlml_and_grad(("SE", {}), [0.06], 0.05, x, y, z)
    assert abs(float(out) - val) <= 1e-9 * abs(val)
    _close([float(h[0].grad), float(nz.grad)], [float(gh[0]), gn], 1e-7)
    _close(zt.grad.numpy(), gz, 1e-6)
    h2 = [torch.tensor(0.07, dtype=F64, requires_grad=True)]
    nz2 = torch.tensor(0.05, dtype=F64, requires_grad=True)
    met.get_metric(h2, nz2, torch.tensor(z, dtype=F64)).sum().backward()
    assert float(h2[0].grad) == 0.0 and float(nz2.grad) == 0.0
