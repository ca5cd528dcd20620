"""Prior / posterior function draws (gpbasics/Statistics/GaussianProcess.py:87-110) on the device
against the oracle with the same standard-normal draw (regenerated from the torch generator's seed;
torch's RNG is only the source of the draw, as tf.random.normal is in the reference).
Tolerances: max-abs <= 1e-10 (prior) and 1e-9 (posterior: the Cholesky of Sigma + 1e-8 I amplifies
the ~1e-13 difference between the Schur-complement and the explicit-inverse Sigma; cond(Sigma) = 7.7
on these 12 test points)."""
import numpy as np
import pytest
import torch

from oracle import gp_oracle as o

import gaussianprocessfundamentals_amd.global_parameters as gp
from gaussianprocessfundamentals_amd.DataHandling.DataInput import DataInput
from gaussianprocessfundamentals_amd.KernelBasics.BaseKernels import SquaredExponentialKernel
from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction
from gaussianprocessfundamentals_amd.Statistics.GaussianProcess import GaussianProcess

pytestmark = pytest.mark.gpu


def make_gp(n=300, m=12):
    x, y = o.make_inputs("C1", n=n)
    xt = np.linspace(0.0, 1.0, m).reshape(m, 1)
    yt = np.sin(4.0 * np.pi * xt)
    di = DataInput(x, y.reshape(-1, 1), xt, yt)
    di.set_mean_function(ZeroMeanFunction(1))
    g = GaussianProcess(SquaredExponentialKernel(1), ZeroMeanFunction(1))
    g.set_data_input(di)
    return g, x, y, xt


def draw(seed, m, n):
    gen = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randn((m, n), dtype=torch.float64, device="cuda", generator=gen).cpu().numpy()


@pytest.mark.parametrize("n_draws", [1, 7])
def test_posterior_functions_match_oracle(n_draws):
    g, x, y, xt = make_gp()
    gen = torch.Generator(device="cuda").manual_seed(11)
    f = g.get_n_posterior_functions(n_draws, [0.1], 1e-2, generator=gen)
    assert tuple(f.shape) == (xt.shape[0], n_draws)
    jit = float(torch.as_tensor(gp.p_cov_matrix_jitter))
    ref = o.n_posterior_functions(("SE", {}), [0.1], 1e-2, x, y, xt, draw(11, xt.shape[0], n_draws), jit)
    assert float(np.max(np.abs(f.cpu().numpy() - ref))) <= 1e-9


def test_prior_functions_match_oracle():
    g, x, y, xt = make_gp()
    gen = torch.Generator(device="cuda").manual_seed(5)
    f = g.get_n_prior_functions(4, [0.1], 1e-2, generator=gen)
    assert tuple(f.shape) == (xt.shape[0], 4)
    ref = o.n_prior_functions(("SE", {}), [0.1], 1e-2, xt, y, draw(5, xt.shape[0], 4))
    assert float(np.max(np.abs(f.cpu().numpy() - ref))) <= 1e-10


def test_posterior_draws_centre_on_the_mean():
    # many draws: their sample mean approaches mu (Monte-Carlo error ~ sd / sqrt(draws))
    g, x, y, xt = make_gp()
    f = g.get_n_posterior_functions(4000, [0.1], 1e-2).cpu().numpy()
    mu, var = o.posterior(("SE", {}), [0.1], 1e-2, x, y, xt)
    sd = np.sqrt(np.clip(np.diag(var), 0.0, None) + float(torch.as_tensor(gp.p_cov_matrix_jitter)))
    assert np.all(np.abs(f.mean(axis=1) - mu) <= 6.0 * sd / np.sqrt(4000) + 1e-12)
