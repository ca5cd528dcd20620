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
# sides, so they run with it off; tests/test_gpu_chain.py compares it with the launch path and the oracle.
_LAUNCH_PATH_MODULES = {"test_gpu_fused_panel", "test_gpu_diag_versions", "test_gpu_kbuild", "test_gpu_parity",
                        "test_gpu_grad"}


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
