"""The drop-in as a reference user would use it (SURVEY §3B wiring): a fresh interpreter calls
``global_parameters.init`` and ``install_gpbasics_alias()``, then runs the INTEGRATION.md snippet with unmodified
``from gpbasics.…`` imports -- DataInput -> GaussianProcess -> get_metric_by_type(LL) -> get_metric, predict and
aux.get_posterior_sd -- and the values are checked against the oracle here.  Also get_posterior_sd's semantics
(S/Auxiliary.py:95-103, quirk Q8): the elementwise sqrt of the FULL posterior covariance, NaN where an entry is
negative (tf.sqrt of a negative float).  Tolerances: -LML rel <= 1e-9, mu / covariance abs <= 1e-8."""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest
import torch

from oracle import gp_oracle as o
from tests.test_gpu_parity import build_gp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SNIPPET = textwrap.dedent('''
    import json, sys
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    import gaussianprocessfundamentals_amd as gpa
    import gaussianprocessfundamentals_amd.global_parameters as global_param
    global_param.init(tf_parallel=0)          # the same call gpbasics requires first (GP:38-39)
    gpa.install_gpbasics_alias()              # unmodified `import gpbasics.…` now resolves here

    from gpbasics.KernelBasics.BaseKernels import SquaredExponentialKernel
    from gpbasics.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction
    from gpbasics.DataHandling.DataInput import DataInput
    from gpbasics.Statistics.GaussianProcess import GaussianProcess
    from gpbasics.Metrics.Auxiliary import get_metric_by_type
    from gpbasics.Metrics.Metrics import MetricType
    import gpbasics.global_parameters as gpb_params

    d = np.load(DATA)
    x_train, y_train, x_test, y_test = d["x"], d["y"].reshape(-1, 1), d["xs"], d["ys"].reshape(-1, 1)
    hyper_parameter = [torch.tensor(0.1, dtype=torch.float64)]
    noise = torch.tensor(1e-2, dtype=torch.float64)

    gp = GaussianProcess(SquaredExponentialKernel(1), ZeroMeanFunction(1))
    di = DataInput(x_train, y_train, x_test, y_test)
    di.set_mean_function(ZeroMeanFunction(1))
    gp.set_data_input(di)
    ll = get_metric_by_type(MetricType.LL, gp)
    nlml = ll.get_metric(hyper_parameter, noise)           # [1,1] tensor holding -LML (M/LogLikelihood.py:30-65)
    mean, _, mu = gp.predict(hyper_parameter, noise=noise)  # S/GaussianProcess.py:42-85
    sd = gp.aux.get_posterior_sd(hyper_parameter, noise)
    import gaussianprocessfundamentals_amd._native as nat
    print(json.dumps({"nlml_shape": list(nlml.shape), "nlml": float(nlml.reshape(-1)[0]),
                      "mu": mu.cpu().tolist(), "sd": sd.cpu().tolist(),
                      "alias_is_package": sys.modules["gpbasics"] is gpa,
                      "same_params_module": gpb_params is global_param,
                      "native": nat.load_library()._name}))
''')


def test_install_gpbasics_alias_and_integration_snippet(tmp_path):
    x, y = o.make_inputs("C1", n=400, seed=11)
    xs = np.linspace(-0.1, 1.1, 37).reshape(-1, 1)
    ys = np.sin(4 * np.pi * xs[:, 0])
    data = tmp_path / "data.npz"
    np.savez(data, x=x, y=y, xs=xs, ys=ys)
    script = tmp_path / "user.py"
    script.write_text("ROOT = %r\nDATA = %r\n" % (ROOT, str(data)) + SNIPPET)
    cp = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=100, cwd=str(tmp_path))
    assert cp.returncode == 0, cp.stderr[-4000:]
    r = json.loads([l for l in cp.stdout.splitlines() if l.startswith("{")][-1])
    assert r["alias_is_package"] and r["same_params_module"] and r["native"].endswith("libgpk.so")
    assert r["nlml_shape"] == [1, 1]
    exp = o.nlml(("SE", {}), [0.1], 1e-2, x, y)
    assert abs(r["nlml"] - exp) <= 1e-9 * abs(exp)
    mu_ref, cov_ref = o.posterior(("SE", {}), [0.1], 1e-2, x, y, xs)
    np.testing.assert_allclose(r["mu"], mu_ref, rtol=0, atol=1e-8)
    sd = np.array(r["sd"], dtype=np.float64)
    with np.errstate(invalid="ignore"):
        sd_ref = np.sqrt(cov_ref)
    # the same entries are NaN (negative covariances; which near-zero ones round negative is a rounding
    # question, so only the clearly negative ones are required to agree)
    clear = np.abs(cov_ref) > 1e-10
    assert np.array_equal(np.isnan(sd[clear]), np.isnan(sd_ref[clear]))
    ok = clear & ~np.isnan(sd_ref)
    np.testing.assert_allclose(sd[ok] ** 2, cov_ref[ok], rtol=0, atol=1e-8)


def test_posterior_sd_is_the_elementwise_sqrt_of_the_full_covariance():
    """S/Auxiliary.py:95-103: tf.sqrt(variance) of the [M, M] covariance -- a matrix, NaN at negative
    covariances, its diagonal the pointwise predictive standard deviation."""
    x, y = o.make_inputs("C1", n=300, seed=2)
    xs = np.linspace(0.0, 1.0, 25).reshape(-1, 1)
    g = build_gp(("SE", {}), x, y, xs, np.zeros(25))
    hyp, noise = [torch.tensor(0.2, dtype=torch.float64)], torch.tensor(1e-2, dtype=torch.float64)
    var = g.aux.get_posterior_var(hyp, noise).cpu().numpy()
    sd = g.aux.get_posterior_sd(hyp, noise).cpu().numpy()
    assert sd.shape == (25, 25)
    _, cov_ref = o.posterior(("SE", {}), [0.2], 1e-2, x, y, xs)
    np.testing.assert_allclose(var, cov_ref, rtol=0, atol=1e-8)
    neg = var < 0
    assert neg.any(), "the test needs negative posterior covariances"
    assert np.isnan(sd[neg]).all() and not np.isnan(sd[~neg]).any()
    np.testing.assert_allclose(sd[~neg], np.sqrt(var[~neg]), rtol=1e-15, atol=0)
    np.testing.assert_allclose(np.diag(sd), np.sqrt(np.diag(cov_ref)), rtol=0, atol=1e-7)


@pytest.mark.parametrize("n", [200, 1500])
def test_consecutive_get_metric_results_stay_independent(n):
    """get_metric returns a view of the evaluation's read-out buffer (no copy): every evaluation writes a fresh
    one, so a result held across later evaluations -- launch path (n = 200) or persistent launch (n = 1500),
    with and without the gradient -- keeps its value and equals the oracle's."""
    from gaussianprocessfundamentals_amd.Metrics.Auxiliary import get_metric_by_type
    from gaussianprocessfundamentals_amd.Metrics.Metrics import MetricType
    rng = np.random.default_rng(5)
    x = np.sort(rng.uniform(0, 1, n)).reshape(n, 1)
    y = np.sin(6 * x[:, 0]) + 0.1 * rng.standard_normal(n)
    g = build_gp(("SE", {}), x, y)
    m = get_metric_by_type(MetricType.LL, g)
    noise = torch.tensor(1e-2, dtype=torch.float64)
    ls = [0.05, 0.1, 0.2]
    held = [m.get_metric([torch.tensor(l, dtype=torch.float64)], noise) for l in ls]
    held_g = [m.get_metric_and_gradient([torch.tensor(l, dtype=torch.float64)], noise)[0] for l in ls]
    for l, v, vg in zip(ls, held, held_g):
        ref = o.nlml(("SE", {}), [l], 1e-2, x, y)
        assert abs(float(v) - ref) <= 1e-9 * abs(ref)
        assert abs(float(vg) - ref) <= 1e-9 * abs(ref)
