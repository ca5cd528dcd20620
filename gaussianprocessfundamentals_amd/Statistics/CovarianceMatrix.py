"""Covariance-matrix plugin (gpbasics/Statistics/CovarianceMatrix.py:15-286) on the MI355X engine.

``HolisticCovarianceMatrix`` keeps the reference's contract: it owns and memoises every matrix it
hands out until :meth:`reset` / :meth:`set_data_input` (CovarianceMatrix.py:37-62); callers reset
when hyperparameters change.  Underneath, the factorisation is ONE augmented Cholesky in libgpk
(include/gpk.h): L, z = L^-1 y, the log-determinant and the data-fit term come out of the same
launches, and alpha = L^-T z is a device triangular solve.  Nothing is computed on the host.

Errors: "No Data Input given" (CovarianceMatrix.py:195); a noise that is not rank-0 raises
(:198-206); a matrix that is not positive definite raises ``CholeskyError`` when the factor is
requested (TensorFlow raises InvalidArgumentError at :250).
"""
from __future__ import annotations

from enum import Enum
from typing import List, Optional

import torch

from .. import engine
from .. import global_parameters as global_param

global_param.ensure_init()


class CovarianceMatrixType(Enum):
    HOLISTIC = 0
    SEGMENTED = 1
    GLOBALIZED_SEGMENTED = 2


def _is_scalar(noise) -> bool:
    return noise is not None and torch.as_tensor(noise).shape == torch.Size([])


def _noise_float(noise) -> float:
    """The noise as a Python float without a float32 detour (torch.as_tensor(0.01) is float32)."""
    t = noise if isinstance(noise, torch.Tensor) else torch.as_tensor(noise, dtype=torch.float64)
    return float(t)


def noise_vector(noise) -> torch.Tensor:
    """Rank-0 noise as a 1-element fp64 device vector (no host round trip for device tensors)."""
    if not isinstance(noise, torch.Tensor) or (noise.device.type == "cpu" and not noise.requires_grad):
        return engine.host_f64_to_device([float(noise)])
    return noise.detach().to(device=engine.device(), dtype=torch.float64).reshape(1)


class CovarianceMatrix:
    _CACHES = ("K", "noised_K", "K_ss", "noised_K_ss", "L_K_ss", "L_K", "L_inv_K", "K_inv", "K_s", "L_alpha")

    def __init__(self, matrix_type: CovarianceMatrixType, kernel):
        self.kernel = kernel
        self.data_input = None
        self.type = matrix_type
        for c in self._CACHES:
            setattr(self, c, None)

    def reset(self):
        """Drop every memoised matrix (CovarianceMatrix.py:37-53)."""
        for c in self._CACHES:
            setattr(self, c, None)

    def set_data_input(self, data_input):
        self.data_input = data_input
        self.reset()

    def is_segmented(self) -> bool:
        return self.type == CovarianceMatrixType.SEGMENTED


class HolisticCovarianceMatrix(CovarianceMatrix):
    """The usual, unapproximated covariance matrix of a GP (CovarianceMatrix.py:178-286)."""

    def __init__(self, kernel):
        super().__init__(CovarianceMatrixType.HOLISTIC, kernel)
        self._fact: Optional[engine.AugmentedFactorization] = None   # y only (the LML)
        self._fact_key = None
        self._inv_fact: Optional[engine.AugmentedFactorization] = None  # identity rows (inverses)

    def reset(self):
        super().reset()
        self._fact_key = None
        self._inv_fact = None

    # -- helpers --------------------------------------------------------------------------------
    def _require_data(self):
        if self.data_input is None:
            raise Exception("No Data Input given")

    def _xy(self):
        di = self.data_input
        y = di.get_detrended_y_train()
        return di.data_x_train, y

    def _shape(self, x):
        if x.dim() == 3:
            return int(x.shape[0]), int(x.shape[1]), int(x.shape[2])
        return 1, int(x.shape[0]), int(x.shape[1])

    def _run(self, fact, hyper_parameter, noise, E=None):
        x, y = self._xy()
        batch, n, d = self._shape(x)
        kd = engine.kernel_descriptor(self.kernel, d)
        hyp, nz = engine.pack_hyper_parameter_and_noise(hyper_parameter, noise, kd.n_hyp)
        x = x.contiguous()
        yv = y.reshape(batch, n).to(torch.float64).contiguous()
        fact.run(kd, hyp, 0, nz if nz is not None else noise_vector(noise), 0, x, n * d if batch > 1 else 0, yv,
                 n if batch > 1 else 0, E=E, e_bstride=0)
        self.kernel._record_hyper_parameter(list(hyper_parameter))
        return fact

    def factorization(self, hyper_parameter: List, noise) -> engine.AugmentedFactorization:
        """The augmented factorisation carrying y (memoised until reset)."""
        self._require_data()
        if not _is_scalar(noise):
            raise Exception("No Data Input given or Noise unspecified")
        if self._fact_key is None:
            x, _ = self._xy()
            batch, n, d = self._shape(x)
            shape = (batch, n, d, global_param.p_dtype)
            if self._fact is None or self._fact.shape_key != shape:
                f = engine.AugmentedFactorization(n, d, 0, batch, global_param.p_dtype)
                f.shape_key = shape
                self._fact = f
            self._run(self._fact, hyper_parameter, noise)
            self._fact_key = True
        return self._fact

    # -- reference surface ------------------------------------------------------------------------
    def get_K(self, hyper_parameter: List) -> torch.Tensor:
        self._require_data()
        if self.K is None:
            x = self.data_input.data_x_train
            if x.dim() == 3:
                self.K = torch.stack([self.kernel.get_tf_tensor(hyper_parameter, xb, xb) for xb in x])
            else:
                self.K = self.kernel.get_tf_tensor(hyper_parameter, x, x)
        return self.K

    def get_K_noised(self, hyper_parameter: List, noise) -> torch.Tensor:
        if _is_scalar(noise) and self.data_input is not None:
            if self.noised_K is None:
                x = self.data_input.data_x_train
                nv = _noise_float(noise)
                if x.dim() == 3:
                    self.noised_K = torch.stack([engine.kernel_matrix(self.kernel, hyper_parameter, xb, xb, nv) for xb in x])
                else:
                    self.noised_K = engine.kernel_matrix(self.kernel, hyper_parameter, x, x, nv)
            return self.noised_K
        raise Exception("No Data Input given or Noise unspecified")

    def get_L_K(self, hyper_parameter: List, noise) -> torch.Tensor:
        """Lower Cholesky factor of K + noise I (CovarianceMatrix.py:247-254)."""
        self._require_data()
        if self.L_K is None:
            f = self.factorization(hyper_parameter, noise)
            f.check_info()
            if f.batch == 1 and self.data_input.data_x_train.dim() == 2:
                self.L_K = f.cholesky(0).to(torch.float64)
            else:
                self.L_K = torch.stack([f.cholesky(b).to(torch.float64) for b in range(f.batch)])
        return self.L_K

    def get_L_alpha(self, hyper_parameter: List, noise) -> torch.Tensor:
        """alpha = L^-T (L^-1 y) as [N, 1] (CovarianceMatrix.py:256-265)."""
        self._require_data()
        if self.L_alpha is None:
            f = self.factorization(hyper_parameter, noise)
            f.check_info()
            if f.batch == 1 and self.data_input.data_x_train.dim() == 2:
                self.L_alpha = f.alpha(0).reshape(-1, 1)
            else:
                self.L_alpha = f.alphas().reshape(f.batch, -1, 1)  # one batched solve for every member
        return self.L_alpha

    def _inverse_factorization(self, hyper_parameter, noise):
        """Augment with identity rows: extra rows -> L^-T, corner -> -K^-1 (one factorisation)."""
        self._require_data()
        if self._inv_fact is None:
            self._inv_fact = self.inverse_factorization(hyper_parameter, noise, gradient=False)
            self._inv_fact.check_info()
        return self._inv_fact

    def inverse_factorization(self, hyper_parameter, noise, gradient: bool = True, y_scale: float = 1.0):
        """One factorisation with identity extra rows (engine.InverseFactorization): -LML, K^-1,
        L^-1, alpha and (gradient=True) d(-LML)/d(hyperparameters, noise) for every member of a
        DataInput (batch 1) or BatchDataInput (one member per batch entry).  y_scale multiplies the
        targets (the batch aggregate's gradient weights the data fit by 1 / B).  Not memoised."""
        self._require_data()
        if not _is_scalar(noise):
            raise Exception("No Data Input given or Noise unspecified")
        x, y = self._xy()
        batch, n, d = self._shape(x)
        kd = engine.kernel_descriptor(self.kernel, d)
        hyp, nz = engine.pack_hyper_parameter_and_noise(hyper_parameter, noise, kd.n_hyp)
        f = engine.InverseFactorization(n, d, batch, global_param.p_dtype)
        yv = y.reshape(batch, n).to(torch.float64)
        yv = (yv * y_scale if y_scale != 1.0 else yv).contiguous()
        f.run(kd, hyp, 0, nz if nz is not None else noise_vector(noise), 0, x.contiguous(),
              n * d if batch > 1 else 0, yv, n if batch > 1 else 0, gradient=gradient)
        self.kernel._record_hyper_parameter(list(hyper_parameter))
        return f

    def get_L_inv_K(self, hyper_parameter: List, noise) -> torch.Tensor:
        """inv(L) (CovarianceMatrix.py:267-275), without an explicit inverse: the identity rows of
        the augmented matrix come out as L^-T."""
        if self.L_inv_K is None:
            f = self._inverse_factorization(hyper_parameter, noise)
            if self.data_input.data_x_train.dim() == 3:   # BatchDataInput: [B, N, N]
                self.L_inv_K = torch.stack([f.l_inv(b).to(torch.float64) for b in range(f.batch)])
            else:
                self.L_inv_K = f.l_inv(0).to(torch.float64).contiguous()
        return self.L_inv_K

    def get_K_inv(self, hyper_parameter: List, noise) -> torch.Tensor:
        """inv(K + noise I) (CovarianceMatrix.py:208-216) from the Schur complement corner."""
        if self.K_inv is None:
            f = self._inverse_factorization(hyper_parameter, noise)
            if self.data_input.data_x_train.dim() == 3:   # BatchDataInput: [B, N, N]
                self.K_inv = torch.stack([f.k_inv(b).to(torch.float64) for b in range(f.batch)])
            else:
                self.K_inv = f.k_inv(0).to(torch.float64)
        return self.K_inv

    def get_K_s(self, hyper_parameter: List) -> torch.Tensor:
        """k(X_train, X_test) [N, M] (CovarianceMatrix.py:277-286)."""
        self._require_data()
        if self.K_s is None:
            di = self.data_input
            self.K_s = self.kernel.get_tf_tensor(hyper_parameter, di.data_x_train, di.data_x_test)
        return self.K_s

    def get_K_ss(self, hyper_parameter: List) -> torch.Tensor:
        """k(X_test, X_test) without noise (CovarianceMatrix.py:218-225)."""
        self._require_data()
        if self.K_ss is None:
            xt = self.data_input.data_x_test
            self.K_ss = self.kernel.get_tf_tensor(hyper_parameter, xt, xt)
        return self.K_ss

    def get_K_ss_noised(self, hyper_parameter: List, noise) -> torch.Tensor:
        if _is_scalar(noise) and self.data_input is not None:
            if self.noised_K_ss is None:
                xt = self.data_input.data_x_test
                self.noised_K_ss = engine.kernel_matrix(self.kernel, hyper_parameter, xt, xt, _noise_float(noise))
            return self.noised_K_ss
        raise Exception("No Data Input given or noise unspecified")

    def get_L_K_ss(self, hyper_parameter: List, noise) -> torch.Tensor:
        """Cholesky of K_ss + noise I (CovarianceMatrix.py:238-245)."""
        self._require_data()
        if self.L_K_ss is None:
            xt = self.data_input.data_x_test
            m, d = int(xt.shape[0]), int(xt.shape[1])
            f = engine.AugmentedFactorization(m, d, 0, 1, global_param.p_dtype)
            kd = engine.kernel_descriptor(self.kernel, d)
            hyp = engine.pack_hyper_parameter(hyper_parameter, kd.n_hyp)
            zeros = torch.zeros(1, m, dtype=torch.float64, device=engine.device())
            f.run(kd, hyp, 0, noise_vector(noise), 0, xt.contiguous(), 0, zeros, 0)
            f.check_info()
            self.L_K_ss = f.cholesky(0).to(torch.float64)
        return self.L_K_ss


# ============================================================================ segmented (blockwise)
def factor_segments(kernels, hyper_parameters, data_inputs, noise, with_test: bool = False):
    """ONE ragged device factorisation (engine.RaggedFactorization) of the independent segments
    (kernel_i, hyp_i, data_input_i); segments without training points are left out.  Returns
    (factorisation or None, index of the segment behind each batch member).

    The reference factors the segments one after another, one TensorFlow Cholesky each
    (SegmentedCovarianceMatrix.get_L_K_blocks / get_L_alpha_blocks, CovarianceMatrix.py:445-484;
    BlockwiseLogLikelihood.get_metric, gpbasics/Metrics/LogLikelihood.py:76-104)."""
    if not _is_scalar(noise):
        raise Exception("Invalid Noise given")
    members, index = [], []
    dims = {int(di.data_x_train.shape[1]) for di in data_inputs}
    if len(dims) != 1:
        raise ValueError("segments must share the input dimensionality")
    d = dims.pop()
    for i, (kern, hyp, di) in enumerate(zip(kernels, hyper_parameters, data_inputs)):
        if di.n_train == 0:
            continue
        kd = engine.kernel_descriptor(kern, d)
        h = engine.pack_hyper_parameter(hyp, kd.n_hyp)
        y = di.get_detrended_y_train().reshape(-1).to(torch.float64)
        xs = di.data_x_test.contiguous() if with_test and di.n_test > 0 else None
        members.append((kd, h, di.data_x_train.contiguous(), y, xs))
        index.append(i)
        kern._record_hyper_parameter(list(hyp))
    if not members:
        return None, index
    sizes = [int(m[2].shape[0]) for m in members]
    tsz = [int(m[4].shape[0]) if m[4] is not None else 0 for m in members] if with_test else None
    f = engine.RaggedFactorization(sizes, d, tsz, global_param.p_dtype)
    f.run(members, noise_vector(noise))
    return f, index


class SegmentedCovarianceMatrix(CovarianceMatrix):
    """Block-diagonal covariance of a change-point / partition operator whose segments are
    independent local models (CovarianceMatrix.py:289-565).  Every ``get_*_blocks`` returns one
    entry per child (None for an empty segment) and the plain getters the block-diagonal matrix
    (rows regrouped segment by segment, as LinearOperatorBlockDiag.to_dense does).  All segments are
    factored together by one ragged device batch (:func:`factor_segments`)."""

    def __init__(self, kernel):
        super().__init__(CovarianceMatrixType.SEGMENTED, kernel)
        self._seg = None

    def reset(self):
        super().reset()
        self._seg = None

    def set_data_input(self, data_input):
        assert len(data_input.data_inputs) == len(self.kernel.child_nodes), \
            "Invalid data input. Data input does not match segments prescribed by given kernel"
        super().set_data_input(data_input)

    def _require_data(self):
        if self.data_input is None:
            raise Exception("No Data Input given")

    def _slices(self, hyper_parameter):
        """Per child: its hyperparameters, after the change points of a ChangePointOperator
        (CovarianceMatrix.py:318-335)."""
        idx = len(self.kernel.change_point_positions) if hasattr(self.kernel, "change_point_positions") else 0
        out = []
        for cn in self.kernel.child_nodes:
            nh = cn.get_number_of_hyper_parameter()
            out.append(list(hyper_parameter[idx:idx + nh]))
            idx += nh
        return out

    @staticmethod
    def _block_diag(blocks):
        present = [b for b in blocks if b is not None]
        return torch.block_diag(*present) if present else \
            torch.zeros((0, 0), dtype=torch.float64, device=engine.device())

    def segment_factorization(self, hyper_parameter, noise):
        """The ragged factorisation of all segments (memoised until reset)."""
        self._require_data()
        if self._seg is None:
            self._seg = factor_segments(self.kernel.child_nodes, self._slices(hyper_parameter),
                                        self.data_input.data_inputs, noise)
        return self._seg

    def _per_segment(self, values_by_member, index):
        out = [None] * len(self.kernel.child_nodes)
        for j, i in enumerate(index):
            out[i] = values_by_member[j]
        return out

    # -- kernel matrices ------------------------------------------------------------------------
    def get_K_blocks(self, hyper_parameter) -> List:
        self._require_data()
        out = []
        for cn, hyp, di in zip(self.kernel.child_nodes, self._slices(hyper_parameter), self.data_input.data_inputs):
            out.append(cn.get_tf_tensor(hyp, di.data_x_train, di.data_x_train) if di.n_train > 0 else None)
        return out

    def get_K(self, hyper_parameter: List) -> torch.Tensor:
        self._require_data()
        if self.K is None:
            self.K = self._block_diag(self.get_K_blocks(hyper_parameter))
        return self.K

    def get_K_noised_blocks(self, hyper_parameter, noise) -> List:
        if not _is_scalar(noise):
            raise Exception("Invalid Noise given")
        self._require_data()
        nv = _noise_float(noise)
        out = []
        for cn, hyp, di in zip(self.kernel.child_nodes, self._slices(hyper_parameter), self.data_input.data_inputs):
            out.append(engine.kernel_matrix(cn, hyp, di.data_x_train, di.data_x_train, nv) if di.n_train > 0 else None)
        return out

    def get_K_noised(self, hyper_parameter: List, noise) -> torch.Tensor:
        self._require_data()
        if self.noised_K is None:
            self.noised_K = self._block_diag(self.get_K_noised_blocks(hyper_parameter, noise))
        return self.noised_K

    def get_K_ss_blocks(self, hyper_parameter) -> List:
        self._require_data()
        out = []
        for cn, hyp, di in zip(self.kernel.child_nodes, self._slices(hyper_parameter), self.data_input.data_inputs):
            out.append(cn.get_tf_tensor(hyp, di.data_x_test, di.data_x_test) if di.n_test > 0 else None)
        return out

    def get_K_ss(self, hyper_parameter: List) -> torch.Tensor:
        self._require_data()
        if self.K_ss is None:
            self.K_ss = self._block_diag(self.get_K_ss_blocks(hyper_parameter))
        return self.K_ss

    def get_K_ss_noised_blocks(self, hyper_parameter, noise) -> List:
        if not _is_scalar(noise):
            raise Exception("Invalid noise provided")
        self._require_data()
        nv = _noise_float(noise)
        out = []
        for cn, hyp, di in zip(self.kernel.child_nodes, self._slices(hyper_parameter), self.data_input.data_inputs):
            out.append(engine.kernel_matrix(cn, hyp, di.data_x_test, di.data_x_test, nv) if di.n_test > 0 else None)
        return out

    def get_K_ss_noised(self, hyper_parameter: List, noise) -> torch.Tensor:
        self._require_data()
        if self.noised_K_ss is None:
            self.noised_K_ss = self._block_diag(self.get_K_ss_noised_blocks(hyper_parameter, noise))
        return self.noised_K_ss

    def get_L_K_ss_blocks(self, hyper_parameter, noise) -> List:
        """Cholesky of every K_ss + noise I block: one ragged factorisation of the test segments."""
        self._require_data()
        from ..DataHandling.DataInput import DataInput
        from ..MeanFunctionBasics.BaseMeanFunctions import ZeroMeanFunction
        tests = []
        for di in self.data_input.data_inputs:
            xt = di.data_x_test
            dtest = DataInput(xt, torch.zeros((xt.shape[0], 1), dtype=torch.float64, device=xt.device), xt,
                              torch.zeros((xt.shape[0], 1), dtype=torch.float64, device=xt.device))
            dtest.mean_function = ZeroMeanFunction(int(xt.shape[1]))
            tests.append(dtest)
        f, index = factor_segments(self.kernel.child_nodes, self._slices(hyper_parameter), tests, noise)
        if f is None:
            return [None] * len(tests)
        f.check_info()
        return self._per_segment([f.cholesky(j).to(torch.float64) for j in range(f.batch)], index)

    def get_L_K_ss(self, hyper_parameter: List, noise) -> torch.Tensor:
        if self.L_K_ss is None:
            self.L_K_ss = self._block_diag(self.get_L_K_ss_blocks(hyper_parameter, noise))
        return self.L_K_ss

    # -- factorisation ----------------------------------------------------------------------------
    def get_L_K_blocks(self, hyper_parameter, noise) -> List:
        f, index = self.segment_factorization(hyper_parameter, noise)
        if f is None:
            return [None] * len(self.kernel.child_nodes)
        f.check_info()
        return self._per_segment([f.cholesky(j).to(torch.float64) for j in range(f.batch)], index)

    def get_L_K(self, hyper_parameter: List, noise) -> torch.Tensor:
        if self.L_K is None:
            self.L_K = self._block_diag(self.get_L_K_blocks(hyper_parameter, noise))
        return self.L_K

    def get_L_alpha_blocks(self, hyper_parameter, noise) -> List:
        """alpha of every segment, [n_i, 1] (CovarianceMatrix.py:469-484): one batched backward solve."""
        f, index = self.segment_factorization(hyper_parameter, noise)
        if f is None:
            return [None] * len(self.kernel.child_nodes)
        f.check_info()
        return self._per_segment([a.reshape(-1, 1) for a in f.alphas()], index)

    def get_L_alpha(self, hyper_parameter: List, noise) -> torch.Tensor:
        if self.L_alpha is None:
            blocks = [b for b in self.get_L_alpha_blocks(hyper_parameter, noise) if b is not None]
            self.L_alpha = torch.cat(blocks, dim=0)
        return self.L_alpha

    def _inverse_blocks(self, hyper_parameter, noise, which):
        out = []
        for cn, hyp, di in zip(self.kernel.child_nodes, self._slices(hyper_parameter), self.data_input.data_inputs):
            if di.n_train == 0:
                out.append(None)
                continue
            h = HolisticCovarianceMatrix(cn)
            h.set_data_input(di)
            out.append(h.get_L_inv_K(hyp, noise) if which == "L" else h.get_K_inv(hyp, noise))
        return out

    def get_L_inv_K_blocks(self, hyper_parameter, noise) -> List:
        """inv(L) per segment (CovarianceMatrix.py:497-509), from identity-augmented factorisations."""
        self._require_data()
        return self._inverse_blocks(hyper_parameter, noise, "L")

    def get_L_inv_K(self, hyper_parameter: List, noise) -> torch.Tensor:
        if self.L_inv_K is None:
            self.L_inv_K = self._block_diag(self.get_L_inv_K_blocks(hyper_parameter, noise))
        return self.L_inv_K

    def get_K_inv_blocks(self, hyper_parameter, noise) -> List:
        """inv(K_i + noise I) per segment (CovarianceMatrix.py:522-534)."""
        self._require_data()
        return self._inverse_blocks(hyper_parameter, noise, "K")

    def get_K_inv(self, hyper_parameter: List, noise) -> torch.Tensor:
        if self.K_inv is None:
            self.K_inv = self._block_diag(self.get_K_inv_blocks(hyper_parameter, noise))
        return self.K_inv

    def get_K_s(self, hyper_parameter: List) -> torch.Tensor:
        """kernel(X_train, X_test) of the whole operator (CovarianceMatrix.py:555-565)."""
        self._require_data()
        if self.K_s is None:
            di = self.data_input
            self.K_s = self.kernel.get_tf_tensor(hyper_parameter, di.data_x_train, di.data_x_test)
        return self.K_s
