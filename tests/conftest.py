import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402

import gaussianprocessfundamentals_amd.global_parameters as gp  # noqa: E402

gp.init(0)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(autouse=True)
def _reset_globals():
    """Tests may flip global flags; restore the defaults after each test."""
    yield
    gp.p_scaled_base_kernel = False
    gp.p_se_expanded_norm = False
    gp.p_dtype = torch.float64


# Modules that test the launch path's own schedules (fused panel solve, diagonal-kernel versions, K-build
# variants, group / look-ahead / fused-K-build knobs, gradient schedules) against each other, often bit for
# bit: the persistent factorisation (on by default for single f64 evaluations) would stand in for both
# sides, so they run with it off.  tests/test_gpu_parity.py runs its golden-fixture and size tests through
# BOTH paths (fixture `factor_path`), tests/test_gpu_chain.py compares the two paths with each other.
_LAUNCH_PATH_MODULES = {"test_gpu_fused_panel", "test_gpu_diag_versions", "test_gpu_kbuild", "test_gpu_grad"}


@pytest.fixture(autouse=True)
def _launch_path_only(request):
    mod = request.module.__name__.rsplit(".", 1)[-1]
    if mod not in _LAUNCH_PATH_MODULES or not torch.cuda.is_available():
        yield
        return
    from gaussianprocessfundamentals_amd import _native as nat
    old = nat.tune("chain", 0)
    try:
        yield
    finally:
        nat.tune("chain", old)


@pytest.fixture(params=["launch", "chain"])
def factor_path(request):
    """Single f64 factorisations through the launch-per-panel path (gpk_tune chain 0) or the persistent
    launch (chain 2: always, even if another stream still has work in flight).  Yields the path name;
    the chain variant asserts on exit that the persistent launch really ran."""
    from gaussianprocessfundamentals_amd import _native as nat
    mode = 0 if request.param == "launch" else 2
    before = nat.chain_stats()["launches"]
    with nat.thread_tune(chain=mode):
        yield request.param
    launched = nat.chain_stats()["launches"] - before
    if request.param == "chain":
        assert launched > 0, "the persistent factorisation did not run"
    else:
        assert launched == 0
