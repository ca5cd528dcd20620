"""Host-side logic of the drop-in: tree flattening, hyperparameter plumbing, data inputs,
metric dispatch and sharding (CPU only, no compute calls)."""
import math

import numpy as np
import pytest
import torch

import gaussianprocessfundamentals_amd.global_parameters as gp
from gaussianprocessfundamentals_amd import _native as nat
from gaussianprocessfundamentals_amd import engine
from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk
from gaussianprocessfundamentals_amd.KernelBasics import Operators as ops
from gaussianprocessfundamentals_amd.DataHandling.DataInput import DataInput, AbstractDataInput
from gaussianprocessfundamentals_amd.Metrics import MatrixHandlingTypes as mht
from gaussianprocessfundamentals_amd.sweep import shard_range
from tests.helpers import set_flags


def flat(kernel, dim=1):
    kd = engine.kernel_descriptor(kernel, dim)
    return [(kd.nodes[i].op, kd.nodes[i].hyp_offset, kd.nodes[i].ard_slot, kd.nodes[i].flags)
            for i in range(kd.n_nodes)], kd.n_hyp


def test_flatten_left_fold_and_dfs_offsets():
    se, per, m32 = bk.SquaredExponentialKernel(1), bk.PeriodicKernel(1), bk.MaternKernel3_2(1)
    k = ops.MultiplicationOperator(1, [ops.AdditionOperator(1, [se, m32]), per])
    nodes, nh = flat(k)
    assert nodes == [(nat.OP_SE, 0, -1, 0), (nat.OP_MAT32, 1, -1, 0), (nat.OP_ADD, 0, -1, 0),
                     (nat.OP_PER, 2, -1, 0), (nat.OP_MUL, 0, -1, 0)]
    assert nh == 4 == k.get_number_of_hyper_parameter()
    add3 = ops.AdditionOperator(1, [bk.SquaredExponentialKernel(1) for _ in range(3)])
    nodes, nh = flat(add3)
    assert [n[0] for n in nodes] == [nat.OP_SE, nat.OP_SE, nat.OP_ADD, nat.OP_SE, nat.OP_ADD]


def test_flatten_scaled_ard_expanded_standard_flags():
    set_flags(scaled=True, expanded=True)
    k = ops.AdditionOperator(4, [bk.SquaredExponentialKernel(4, ard=True), bk.PeriodicKernel(4, standard=True),
                                 bk.MaternKernel5_2(4, ard=True, standard=True)])
    nodes, nh = flat(k, 4)
    assert nodes[0] == (nat.OP_SE, 0, 0, nat.NODE_SCALED | nat.NODE_ARD | nat.NODE_SE_EXPANDED)
    assert nodes[1] == (nat.OP_PER, 5, -1, nat.NODE_SCALED | nat.NODE_STANDARD)
    assert nodes[3] == (nat.OP_MAT52, 8, 1, nat.NODE_SCALED | nat.NODE_ARD | nat.NODE_STANDARD)
    assert nh == 5 + 3 + 5
    assert k.get_number_of_hyper_parameter() == 2 + 3 + 2
    with pytest.raises(ValueError):
        bk.PeriodicKernel(2, ard=True)


def test_pack_hyper_parameter_dfs_order():
    gp.p_device = "cpu"
    try:
        v = engine.pack_hyper_parameter([torch.tensor(0.5), torch.tensor([1.0, 2.0]), 3.0])
        assert v.tolist() == [0.5, 1.0, 2.0, 3.0]
        with pytest.raises(ValueError):
            engine.pack_hyper_parameter([1.0, 2.0], n_expected=3)
    finally:
        gp.p_device = "cuda"


def test_pack_hyper_parameter_and_noise_one_buffer():
    """Host hyperparameters + host noise: one buffer, two views (one copy to the device); a noise that needs its
    gradient keeps its own path (None: the caller's noise_vector)."""
    gp.p_device = "cpu"
    try:
        h, nz = engine.pack_hyper_parameter_and_noise([torch.tensor(0.5), [1.0, 2.0]], torch.tensor(0.01, dtype=torch.float64), 3)
        assert h.tolist() == [0.5, 1.0, 2.0] and nz.tolist() == [0.01]
        assert h.untyped_storage().data_ptr() == nz.untyped_storage().data_ptr()
        h, nz = engine.pack_hyper_parameter_and_noise([0.5], 0.25, 1)
        assert h.tolist() == [0.5] and nz.tolist() == [0.25]
        h, nz = engine.pack_hyper_parameter_and_noise([0.5], torch.tensor(0.1, requires_grad=True), 1)
        assert h.tolist() == [0.5] and nz is None
        with pytest.raises(ValueError):
            engine.pack_hyper_parameter_and_noise([1.0, 2.0], 0.1, 3)
    finally:
        gp.p_device = "cuda"


def test_reference_hyperparameter_plumbing():
    set_flags(scaled=True)
    se = bk.SquaredExponentialKernel(1)
    per = bk.PeriodicKernel(1)
    k = ops.AdditionOperator(1, [se, per])
    assert k.get_hyper_parameter_names(0) == ["SE_0_l", "SE_0_sg", "PER_1_l", "PER_1_p", "PER_1_sg"]
    d = k.get_default_hyper_parameter([[0.0, 2.0]], 100)
    assert [float(h) for h in d] == pytest.approx([0.2, 0.1, 0.2, 0.2, 0.1])
    b = se.get_hyper_parameter_bounds([[0.0, 1.0]], 100)
    assert float(b[0][0]) == pytest.approx(0.05) and float(b[0][1]) == pytest.approx(1 / 3)
    assert float(b[1][0]) == pytest.approx(1e-6) and math.isinf(float(b[1][1]))
    k.set_last_hyper_parameter([torch.tensor(-0.3), torch.tensor(1.0), torch.tensor(-0.4), torch.tensor(-2.0), torch.tensor(0.5)])
    assert [float(h) for h in k.get_last_hyper_parameter()] == pytest.approx([0.3, 1.0, 0.4, 2.0, 0.5])
    assert k.get_string_representation() == "(SE + PER)"
    assert k.get_hyper_parameter_dimensionalities() == [[], [], [], [], []]
    assert bk.SquaredExponentialKernel(3, ard=True).get_hyper_parameter_dimensionalities() == [[3], []]
    c = k.deepcopy()
    assert c.get_string_representation() == "(SE + PER)" and c is not k


def test_simplified_version_distributes():
    se, per, m = bk.SquaredExponentialKernel(1), bk.PeriodicKernel(1), bk.MaternKernel5_2(1)
    k = ops.MultiplicationOperator(1, [ops.AdditionOperator(1, [se, per]), m])
    s = k.get_simplified_version()
    assert s.get_string_representation() == "((MAT52 x SE) + (MAT52 x PER))"


def test_noise_must_be_rank0():
    se = bk.SquaredExponentialKernel(1)
    se.set_noise(torch.tensor(0.1))
    with pytest.raises(Exception):
        se.set_noise(torch.tensor([0.1, 0.2]))


def test_data_input_split_and_shapes():
    gp.p_device = "cpu"
    try:
        x = np.linspace(0, 1, 50).reshape(-1, 1)
        y = np.sin(x)
        di = DataInput(x, y)
        assert di.n_train == 40 and di.n_test == 10
        assert di.data_x_train.dtype == torch.float64
        assert torch.all(di.data_x_train[1:] >= di.data_x_train[:-1])
        di2 = DataInput(x, y, test_ratio=0)
        assert di2.n_train == 50 and di2.n_test == 50
        assert di.get_x_range()[0][0] >= 0.0
        folds = AbstractDataInput.get_k_fold_data_inputs(torch.as_tensor(x), torch.as_tensor(y), 5)
        assert sum(f.n_test for f in folds) == 50
        with pytest.raises(AssertionError):
            DataInput(x, np.zeros((50, 2)))
    finally:
        gp.p_device = "cuda"


def test_metric_approximation_binding():
    """Metric.__init__ (gpbasics/Metrics/Metrics.py:45-107): approximations set n_inducting_train and
    swap get_covariance_matrix / get_log_determinant; a subset as large as the data disables them."""
    from gaussianprocessfundamentals_amd.Metrics.Metrics import Metric, MetricType

    class Dummy:
        n_train = 10
        n_test = 5

    class Cov:
        kernel = None

        def set_data_input(self, di):
            self.di = di

    A, H = mht.MatrixApproximations, mht.NumericalMatrixHandlingType
    m = Metric(Dummy(), Cov(), MetricType.LL, A.BASIC_NYSTROEM, H.CHOLESKY_BASED, subset_size=4)
    assert m.data_input.n_inducting_train == 4 and m.data_input.n_inducting_test == 2.0
    assert m.get_covariance_matrix.__func__ is Metric.get_nystroem_matrix
    assert m.get_log_determinant.__func__ is Metric.get_log_determinant_nystroem
    assert m.get_alpha.__func__ is Metric.get_alpha_cholesky and m._approximate()
    m = Metric(Dummy(), Cov(), MetricType.LL, A.SKC_UPPER_BOUND, H.LINEAR_CONJUGATE_GRADIENT, subset_size=4)
    assert m.get_covariance_matrix.__func__ is Metric.get_default_covariance_matrix and not m._approximate()
    assert m.get_log_determinant.__func__ is Metric.get_log_determinant_nystroem
    m = Metric(Dummy(), Cov(), MetricType.LL, A.SKI, H.STRICT_INVERSE, subset_size=4)
    assert m.get_covariance_matrix.__func__ is Metric.get_ski_matrix
    assert m.get_log_determinant.__func__ is Metric.get_log_determinant_slodget
    m = Metric(Dummy(), Cov(), MetricType.LL, A.SKI, H.CHOLESKY_BASED)         # subset = int(10 * 0.1)
    assert m.subset_size == 1 and m.data_input.n_inducting_train == 1
    m = Metric(Dummy(), Cov(), MetricType.LL, A.SKI, H.CHOLESKY_BASED, subset_size=10)
    assert m.local_approx is A.NONE and not m._approximate()


def test_variational_sgd_step_matches_oracle():
    from oracle import gp_oracle as o
    from gaussianprocessfundamentals_amd.Metrics.SkcLogLikelihood import variational_sgd_step
    g = np.array([0.0, 1.0, -3.0, 5e3, 6.5e3, -7e3, 1e5]).reshape(-1, 1)
    a = np.ones_like(g)
    got = variational_sgd_step(torch.as_tensor(a), torch.as_tensor(g)).numpy()
    assert np.array_equal(got, o.vsgd_step(a, g))
    assert got[0, 0] == 1.0 and got[1, 0] == 1.0 - 1e-6


@pytest.mark.parametrize("n,world", [(128, 1), (128, 2), (128, 8), (10, 3), (3, 8), (0, 4)])
def test_shard_range_partitions(n, world):
    parts = [shard_range(n, r, world) for r in range(world)]
    assert parts[0][0] == 0 and parts[-1][1] == n
    for (a, b), (c, d) in zip(parts, parts[1:]):
        assert b == c
    sizes = [b - a for a, b in parts]
    assert max(sizes) - min(sizes) <= 1


def test_ensure_init_exits_when_not_initialised():
    gp.initiated = False
    try:
        with pytest.raises(SystemExit) as e:
            gp.ensure_init()
        assert e.value.code == -100
    finally:
        gp.initiated = True


def test_is_equidistant_and_individual_detrending():
    import numpy as np
    import torch
    from gaussianprocessfundamentals_amd.DataHandling import DataInput as dim
    from gaussianprocessfundamentals_amd.DataHandling.BatchDataInput import BatchDataInput, is_equidistant as eq_b
    from gaussianprocessfundamentals_amd.MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction
    grid = np.linspace(0.0, 1.0, 50).reshape(-1, 1)
    assert dim.is_equidistant(grid)
    jitter = grid.copy()
    jitter[10, 0] += 1e-3  # > 1 / (100 * 50) off the mean spacing
    assert not dim.is_equidistant(jitter)
    di = dim.DataInput(grid, np.sin(grid), grid[:5], np.cos(grid[:5]))
    assert di.is_equidistant_input_x()
    di.set_mean_function(ZeroMeanFunction(1))
    y = di.get_detrended_y_test_individual(grid[:3], np.ones((3, 1)))
    assert y.dtype == torch.float64 and torch.equal(y.cpu(), torch.ones(3, 1, dtype=torch.float64))
    # batched form: B = 1 broadcasts; a non-uniform member fails
    xb = np.stack([grid])
    assert bool(eq_b(xb).all())
    assert not bool(eq_b(np.stack([jitter])).all())
    bdi = BatchDataInput(xb, np.sin(xb), xb, np.sin(xb))
    assert bool(bdi.is_equidistant_input_x().all())
    with pytest.raises(Exception, match="Not implemented for BatchDataInput"):
        bdi.get_subset(10, None)


def test_change_point_mask_functions_match_oracle():
    import numpy as np
    import torch
    from oracle import gp_oracle as o
    from gaussianprocessfundamentals_amd.KernelBasics.Operators import ChangePointOperator as CP
    x = np.linspace(0.0, 1.0, 41).reshape(-1, 1)
    xt = torch.as_tensor(x)
    for cp in (0.3, 0.5125):
        assert np.array_equal(CP.indicator_function_tf_less(xt, cp).numpy().reshape(-1), o.cp_indicator(x, cp))
        assert np.allclose(CP.sigmoid(xt, cp).numpy().reshape(-1), o.cp_indicator(x, cp, "SIGMOID"), atol=1e-15)
        assert np.allclose(CP.approx_indicator(xt, cp).numpy().reshape(-1), o.cp_indicator(x, cp, "APPROX_INDICATOR"),
                           atol=1e-15)
        assert CP.indicator_function_tf_less(xt, cp).shape == (41, 1)
        assert np.array_equal(CP.indicator_function_relu_sign(xt, cp).numpy(), (x > cp).astype(np.float64))


def test_default_hyper_parameter_fixed_and_distribution():
    import torch
    from gaussianprocessfundamentals_amd.KernelBasics import BaseKernels as bk
    kern = bk.PeriodicKernel(1)
    fixed = kern.get_default_hyper_parameter_fixed([[0.0, 2.0]], 100)
    assert [float(h) for h in fixed] == [float(h) for h in kern.get_default_hyper_parameter([[0.0, 2.0]], 100)]
    assert abs(float(fixed[0]) - 0.2) < 1e-15
    torch.manual_seed(0)
    rnd = kern.get_default_hyper_parameter_distribution([[0.0, 2.0]], 100)
    assert len(rnd) == len(fixed) and all(float(h) >= 0 for h in rnd)
