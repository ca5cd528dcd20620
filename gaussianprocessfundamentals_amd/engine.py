"""Device engine: the glue between the gpbasics-style Python objects and libgpk.

* :func:`kernel_descriptor` flattens a kernel tree (KernelBasics) into the postfix program the
  HIP kernels evaluate (include/gpk.h, ``gpk_kdesc``).
* :func:`pack_hyper_parameter` concatenates a hyperparameter list in DFS order, the layout of
  ``Component.serialize_hyper_parameter`` (gpbasics/Auxiliary/BasicGPComponent.py:16-23).
* :class:`AugmentedFactorization` owns the device buffers of one factorisation of the augmented
  matrix (training block + optional extra rows + the y row) and reads results out of it.

All arithmetic runs in libgpk on the GPU; torch only allocates and views device memory.
"""
from __future__ import annotations

import ctypes
import logging
import os
from typing import List, Optional, Sequence

import torch

from . import _native as nat
from . import global_parameters as gp

# A single f64 factorisation may run as ONE persistent launch (gpk_tune "chain", include/gpk.h).  Its
# inter-workgroup waits are bounded; a wait that times out (the device shared with another process past
# chain_timeout_ms, a preempted workgroup) leaves info = -1 and the factorisation incomplete.  With
# CHAIN_VERIFY (default) a run that took the persistent launch is verified lazily: run() itself never
# synchronises (calls enqueue ahead of the device), and the FIRST read of its results -- info, out, W and every
# read-out accessor -- reads info back (one 4-byte device-to-host copy, which waits for that run) and, on -1,
# assembles and factors again on the launch path, on the run's own stream, before returning; CHAIN_FALLBACKS
# counts those re-runs.  (The re-run reads the operands passed to run(): they must not be overwritten in
# between.)  The reference's tf.linalg.cholesky never fails spuriously
# (gpbasics/Statistics/CovarianceMatrix.py:250), so neither may this.
CHAIN_VERIFY = True
CHAIN_FALLBACKS = 0


class CholeskyError(RuntimeError):
    """Cholesky of K + noise*I failed (not positive definite).  The reference propagates
    TensorFlow's InvalidArgumentError from tf.linalg.cholesky
    (gpbasics/Statistics/CovarianceMatrix.py:250)."""

    def __init__(self, info):
        super().__init__("Cholesky decomposition was not successful: leading minor of order %s is "
                         "not positive definite" % (info,))
        self.info = info


def device() -> torch.device:
    d = torch.device(gp.p_device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def as_device_f64(x) -> torch.Tensor:
    """fp64 device copy/view of array-like x (the reference casts every input to p_dtype=fp64,
    gpbasics/DataHandling/DataInput.py:198-206)."""
    if isinstance(x, torch.Tensor):
        t = x.detach()
    else:
        t = torch.as_tensor(x)
    return t.to(device=device(), dtype=torch.float64).contiguous()


# ----------------------------------------------------------------------------- kernel programs
def kernel_descriptor(kernel, dim: Optional[int] = None) -> nat.GpkKdesc:
    """Flatten ``kernel`` (a Kernel tree) to the postfix program of include/gpk.h."""
    dim = int(dim if dim is not None else kernel.get_dimensionality())
    nodes: List[tuple] = []
    slots: List[int] = []
    n_hyp = kernel._emit(nodes, 0, slots, dim)
    if len(nodes) > nat.MAX_NODES:
        raise ValueError("kernel tree too large for the device program (%d > %d nodes)"
                         % (len(nodes), nat.MAX_NODES))
    if len(slots) > nat.MAX_ARD:
        raise ValueError("at most %d ARD base kernels per tree" % nat.MAX_ARD)
    if n_hyp > nat.MAX_HYP:
        raise ValueError("too many hyperparameters (%d > %d)" % (n_hyp, nat.MAX_HYP))
    if dim < 1 or dim > nat.MAX_DIM:
        raise ValueError("input dimensionality must be in [1, %d]" % nat.MAX_DIM)
    kd = nat.GpkKdesc()
    kd.n_nodes = len(nodes)
    kd.n_hyp = n_hyp
    kd.dim = dim
    kd.n_ard = len(slots)
    for i, (op, off, slot, flags) in enumerate(nodes):
        kd.nodes[i].op = op
        kd.nodes[i].hyp_offset = off
        kd.nodes[i].ard_slot = slot
        kd.nodes[i].flags = flags
    return kd


# small host values (hyperparameters, noise) reach the device through one asynchronous copy from pinned memory
# (torch's caching host allocator keeps the block until the copy is done) instead of a synchronous pageable copy
# per tensor; GPK_PINNED_H2D=0 restores the plain copy (A/B)
PINNED_H2D = os.environ.get("GPK_PINNED_H2D", "1") != "0"


def host_f64_to_device(values) -> torch.Tensor:
    """fp64 device vector of a short list of host floats (asynchronous, stream-ordered on the current stream)."""
    t = torch.tensor(values, dtype=torch.float64)
    dev = device()
    if PINNED_H2D and dev.type == "cuda":
        return t.pin_memory().to(dev, non_blocking=True)
    return t.to(dev)


def _host_values(hyper_parameter: Sequence) -> Optional[List[float]]:
    """The flat host floats of a hyperparameter list, or None if an entry lives on the device."""
    for h in hyper_parameter:
        if isinstance(h, torch.Tensor) and h.device.type != "cpu":
            return None
    vals: List[float] = []
    for h in hyper_parameter:
        if isinstance(h, torch.Tensor):
            vals.extend(float(v) for v in h.detach().reshape(-1).tolist())
        else:
            try:
                vals.extend(float(v) for v in h)
            except TypeError:
                vals.append(float(h))
    return vals


def pack_hyper_parameter_and_noise(hyper_parameter: Sequence, noise, n_expected: int):
    """(hyperparameter vector, 1-element noise vector) on the device; when both are host values, through ONE
    asynchronous copy (one buffer, two views) instead of one per operand.  noise None: the caller's own."""
    host_noise = not isinstance(noise, torch.Tensor) or (noise.device.type == "cpu" and not noise.requires_grad)
    vals = _host_values(hyper_parameter) if host_noise and not (
        isinstance(hyper_parameter, torch.Tensor) and hyper_parameter.dim() == 1) else None
    if vals is None:
        return pack_hyper_parameter(hyper_parameter, n_expected), None
    if len(vals) != n_expected:
        raise ValueError("hyperparameter vector has %d values, kernel expects %d" % (len(vals), n_expected))
    t = host_f64_to_device(vals + [float(noise)])
    return t[:n_expected], t[n_expected:]


def pack_hyper_parameter(hyper_parameter: Sequence, n_expected: Optional[int] = None) -> torch.Tensor:
    """Flat fp64 device vector of a hyperparameter list (each entry reshaped to [-1], concatenated;
    BasicGPComponent.serialize_hyper_parameter, gpbasics/Auxiliary/BasicGPComponent.py:16-23)."""
    dev = device()
    if isinstance(hyper_parameter, torch.Tensor) and hyper_parameter.dim() == 1:
        flat = hyper_parameter.to(device=dev, dtype=torch.float64)
    else:
        parts = []
        host_vals = _host_values(hyper_parameter)
        if host_vals is not None:
            flat = host_f64_to_device(host_vals)
        else:
            for h in hyper_parameter:
                parts.append(torch.as_tensor(h).to(device=dev, dtype=torch.float64).reshape(-1))
            flat = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.float64, device=dev)
    if n_expected is not None and flat.numel() != n_expected:
        raise ValueError("hyperparameter vector has %d values, kernel expects %d"
                         % (flat.numel(), n_expected))
    return flat.contiguous()


def kernel_matrix(kernel, hyper_parameter, x, x_, diag_add: float = 0.0, lower: bool = False,
                  out_dtype=None) -> torch.Tensor:
    """k(x, x_) as an [n, m] device tensor via gpk_kernel_matrix (K/Kernel.py:51-52)."""
    L = nat.lib()
    x = as_device_f64(x)
    x_ = as_device_f64(x_)
    if x.dim() != 2 or x_.dim() != 2 or x.shape[1] != x_.shape[1]:
        raise ValueError("kernel inputs must be [n, D] and [m, D]")
    kd = kernel_descriptor(kernel, x.shape[1])
    hyp = pack_hyper_parameter(hyper_parameter, kd.n_hyp)
    dt = out_dtype or torch.float64
    n, m = x.shape[0], x_.shape[0]
    K = torch.empty((n, m), dtype=dt, device=x.device)
    if n == 0 or m == 0:
        return K
    nat.check(L.gpk_kernel_matrix(ctypes.byref(kd), nat.ptr(hyp), nat.dtype_code(dt), 1 if lower else 0,
                                  nat.ptr(x), n, nat.ptr(x_), m, x.shape[1], float(diag_add),
                                  nat.ptr(K), m, nat.stream_handle(x.device)), "gpk_kernel_matrix")
    return K


# ----------------------------------------------------------------------------- factorisation
def _check_operand(name: str, t: torch.Tensor, bstride: int, per_member: int, batch: int,
                   dev: torch.device) -> None:
    if t is None:
        raise ValueError("%s is required" % name)
    if t.dtype != torch.float64 or not t.is_contiguous() or t.device != dev:
        raise ValueError("%s must be a contiguous float64 tensor on %s (got %s, %s, contiguous=%s)"
                         % (name, dev, t.dtype, t.device, t.is_contiguous()))
    need = (batch - 1) * int(bstride) + int(per_member) if batch > 0 else 0
    if int(bstride) < 0 or t.numel() < need:
        raise ValueError("%s holds %d elements, the layout reads %d (batch %d, stride %d, %d per member)"
                         % (name, t.numel(), need, batch, bstride, per_member))


class AugmentedFactorization:
    """One factorisation of the augmented matrix W (include/gpk.h) for ``batch`` problems.

    After :meth:`run`, W's first n_pad columns hold L, the y row holds z = L^-1 y, the extra rows
    hold V^T = Ks^T L^-T and the corner holds the Schur complement (posterior covariance,
    -posterior mean, -z^T z).
    """

    def __init__(self, n: int, d: int, m: int = 0, batch: int = 1, dtype=None):
        self.L = nat.lib()
        self.dtype = dtype or gp.p_dtype
        self.code = nat.dtype_code(self.dtype)
        self.n, self.d, self.m, self.batch = int(n), int(d), int(m), int(batch)
        self.layout = nat.plan(self.code, self.batch, self.n, self.m, self.d)
        lay = self.layout
        dev = device()
        es = 8 if self.code == nat.GPK_F64 else 4
        self._pending = None   # (rerun, stream) of a persistent run not yet verified (see CHAIN_VERIFY)
        self._W = torch.empty(lay.w_bytes // es, dtype=self.dtype, device=dev)
        self._Winv = torch.empty(max(1, lay.inv_bytes // es), dtype=self.dtype, device=dev)
        self._info = torch.zeros(self.batch, dtype=torch.int32, device=dev)
        self._out = torch.empty(self.batch * 4, dtype=torch.float64, device=dev)
        self._mu = torch.empty(max(1, self.batch * self.m), dtype=torch.float64, device=dev)
        self._var = torch.empty(max(1, self.batch * self.m), dtype=torch.float64, device=dev)
        self.kd = None
        self.done = False
        self.shape_key = None

    # -- result buffers: every read settles a pending persistent run first ---------------------
    @property
    def W(self) -> torch.Tensor:
        self._settle()
        return self._W

    @property
    def Winv(self) -> torch.Tensor:
        self._settle()
        return self._Winv

    @property
    def info(self) -> torch.Tensor:
        self._settle()
        return self._info

    @property
    def out(self) -> torch.Tensor:
        self._settle()
        return self._out

    @property
    def mu(self) -> torch.Tensor:
        self._settle()
        return self._mu

    @property
    def var(self) -> torch.Tensor:
        self._settle()
        return self._var

    # -- launches ---------------------------------------------------------------------------
    def _defer_verify(self, rerun) -> None:
        """After a run: if libgpk took the persistent launch for it, remember how to re-run it; the first read
        of a result verifies it (:meth:`_settle`).  No synchronisation here."""
        self._pending = None
        if CHAIN_VERIFY and nat.last_factorisation_was_chain():
            self._pending = (rerun, torch.cuda.current_stream(self._W.device))

    def _settle(self) -> None:
        """Verify a pending persistent run: if a wait timed out (info = -1), run it again on the launch path on
        the run's own stream and count the fallback.  Synchronises with that run."""
        global CHAIN_FALLBACKS
        pend = self._pending
        if pend is None:
            return
        self._pending = None
        rerun, stream = pend
        with torch.cuda.stream(stream):
            if not bool((self._info == -1).any()):   # (waits for the run)
                return
            CHAIN_FALLBACKS += 1
            logging.warning("persistent factorisation timed out (gpk_tune chain_timeout_ms): re-running it on the "
                            "launch path (%d fallbacks so far)", CHAIN_FALLBACKS)
            with nat.thread_tune(chain=0):
                rerun()

    def run(self, kd: nat.GpkKdesc, hyp: torch.Tensor, hyp_stride: int, noise: torch.Tensor,
            noise_stride: int, X: torch.Tensor, x_bstride: int, y: torch.Tensor, y_bstride: int,
            Xs: Optional[torch.Tensor] = None, xs_bstride: int = 0,
            E: Optional[torch.Tensor] = None, e_bstride: int = 0):
        """Enqueue the factorisation (asynchronous: a persistent run is verified at the first read, see
        CHAIN_VERIFY)."""
        args = (kd, hyp, hyp_stride, noise, noise_stride, X, x_bstride, y, y_bstride, Xs, xs_bstride, E, e_bstride)
        self._pending = None   # (the previous run's results are overwritten unread)
        self._run_once(*args)
        self._defer_verify(lambda: self._run_once(*args))
        return self

    def _fresh_out(self) -> None:
        """A new read-out buffer per evaluation (the caching allocator's, no device work): views of an earlier
        evaluation's -LML stay valid without a copy (LogLikelihood.get_metric returns one)."""
        self._out = torch.empty(self.batch * 4, dtype=torch.float64, device=self._W.device)

    def _run_once(self, kd, hyp, hyp_stride, noise, noise_stride, X, x_bstride, y, y_bstride, Xs, xs_bstride,
                  E, e_bstride):
        lay = self.layout
        B, n, m, d = self.batch, self.n, self.m, self.d
        self._alphas = None
        self._fresh_out()
        # the device reads these extents blindly: check them here (an undersized operand would
        # be read out of bounds, not reported)
        _check_operand("hyper_parameter", hyp, hyp_stride, kd.n_hyp, B, self.W.device)
        _check_operand("noise", noise, noise_stride, 1, B, self.W.device)
        _check_operand("X", X, x_bstride, n * d, B, self.W.device)
        _check_operand("y", y, y_bstride, n, B, self.W.device)
        if m:
            if E is not None:
                _check_operand("E", E, e_bstride, m * n, B, self.W.device)
            elif Xs is not None:
                _check_operand("X_test", Xs, xs_bstride, m * d, B, self.W.device)
            else:
                raise ValueError("m = %d extra rows need X_test or E" % m)
        s = nat.stream_handle(self.W.device)
        L = self.L
        if m == 0:
            # gpk_nlml: K build (fused into the first trailing update for single-node kernels) +
            # factorisation + read-out; zeroes info itself
            nat.check(L.gpk_nlml(ctypes.byref(kd), ctypes.byref(lay), nat.ptr(hyp), hyp_stride, nat.ptr(noise),
                                 noise_stride, nat.ptr(X), x_bstride, nat.ptr(y), y_bstride, nat.ptr(self.W),
                                 nat.ptr(self.Winv), nat.ptr(self.info), nat.ptr(self.out), s), "gpk_nlml")
            self.kd = kd
            self.done = True
            return self
        self.info.zero_()
        nat.check(L.gpk_assemble(ctypes.byref(kd), ctypes.byref(lay), nat.ptr(hyp), hyp_stride,
                                 nat.ptr(noise), noise_stride, nat.ptr(X), x_bstride,
                                 nat.ptr(Xs), xs_bstride, nat.ptr(E), e_bstride,
                                 nat.ptr(y), y_bstride, nat.ptr(self.W), s), "gpk_assemble")
        nat.check(L.gpk_potrf_aug(ctypes.byref(lay), nat.ptr(self.W), nat.ptr(self.Winv),
                                  nat.ptr(self.info), s), "gpk_potrf_aug")
        nat.check(L.gpk_finalize(ctypes.byref(lay), nat.ptr(self.W), nat.ptr(self.info),
                                 nat.ptr(self.out), nat.ptr(self.mu) if self.m else None,
                                 nat.ptr(self.var) if self.m else None, s), "gpk_finalize")
        self.kd = kd
        self.done = True
        return self

    # -- read-out (device views, no host synchronisation) -----------------------------------
    def w(self, b: int = 0) -> torch.Tensor:
        lay = self.layout
        return self.W[b * lay.w_batch_stride:(b + 1) * lay.w_batch_stride].view(lay.p, lay.ld)

    def nlml(self) -> torch.Tensor:
        return self.out.view(self.batch, 4)[:, 0]

    def unsettled_results(self):
        """(-LML, info) device views WITHOUT settling a pending persistent run (no host synchronisation): for callers
        that pipeline runs and only forward the values on the device -- a wait that timed out shows as info = -1
        there, and the run is not re-done.  Everyone else reads nlml() / info."""
        return self._out.view(self.batch, 4)[:, 0], self._info

    def fit(self) -> torch.Tensor:
        return self.out.view(self.batch, 4)[:, 1]

    def logdet(self) -> torch.Tensor:
        return self.out.view(self.batch, 4)[:, 2]

    def cholesky(self, b: int = 0) -> torch.Tensor:
        """L (lower, [n, n], p_dtype)."""
        return torch.tril(self.w(b)[:self.n, :self.n])

    def z(self, b: int = 0) -> torch.Tensor:
        lay = self.layout
        return self.w(b)[lay.y_row, :self.n]

    def extra_rows(self, b: int = 0) -> torch.Tensor:
        """Rows n_pad .. n_pad+m-1 restricted to the first n columns: V^T = Ks^T L^-T (or E L^-T)."""
        lay = self.layout
        return self.w(b)[lay.n_pad:lay.n_pad + self.m, :self.n]

    def corner(self, b: int = 0) -> torch.Tensor:
        """Symmetrised m x m Schur complement: Kss - V^T V (or -E K^-1 E^T)."""
        lay = self.layout
        c = self.w(b)[lay.n_pad:lay.n_pad + self.m, lay.n_pad:lay.n_pad + self.m]
        lo = torch.tril(c)
        return lo + torch.tril(c, -1).transpose(0, 1)

    def posterior_mu(self, b: int = 0) -> torch.Tensor:
        return self.mu[b * self.m:(b + 1) * self.m]

    def posterior_var_diag(self, b: int = 0) -> torch.Tensor:
        return self.var[b * self.m:(b + 1) * self.m]

    def alphas(self) -> torch.Tensor:
        """[batch, n]: alpha_b = L_b^-T z_b = (K_b + noise I)^-1 y_b for every member from ONE batched
        backward solve (gpk_trsv), computed once per run and kept until the next one."""
        if getattr(self, "_alphas", None) is None:
            lay = self.layout
            x = torch.zeros((self.batch, lay.n_pad), dtype=torch.float64, device=self.W.device)
            x[:, :self.n] = self.W.view(self.batch, lay.p, lay.ld)[:, lay.y_row, :self.n]
            nat.check(self.L.gpk_trsv(ctypes.byref(lay), 1, nat.ptr(self.W), nat.ptr(self.Winv),
                                      nat.ptr(x), nat.stream_handle(self.W.device)), "gpk_trsv")
            self._alphas = x[:, :self.n]
        return self._alphas

    def alpha(self, b: int = 0) -> torch.Tensor:
        """alpha = L^-T z = (K + noise I)^-1 y of member b (see :meth:`alphas`)."""
        return self.alphas()[b]

    def check_info(self):
        """Raise CholeskyError if any batch member failed (synchronises)."""
        info = self.info.cpu()
        bad = torch.nonzero(info).flatten()
        if bad.numel():
            if int(info[bad[0]]) < 0:
                # (run() re-runs a timed-out persistent launch on the launch path, so this is reached only
                # with CHAIN_VERIFY off: an infrastructure failure, never "not positive definite")
                raise RuntimeError("device factorisation aborted: a wait of the persistent factorisation timed "
                                   "out (gpk_tune chain_timeout_ms)")
            raise CholeskyError(int(info[bad[0]]))


class InverseFactorization(AugmentedFactorization):
    """Factorisation of the augmented matrix with identity extra rows (m = n), optionally followed
    by the -LML gradient (``gpk_nlml_grad``).

    After :meth:`run` the extra rows hold L^-T, the corner -K^-1 and the corner's y row -alpha^T
    (include/gpk.h); tiles of structurally zero identity rows are skipped, so the factorisation
    costs n^3 flops -- the work of potrf + trtri + lauum, i.e. of the reference's explicit
    tf.linalg.inv(L) / inv(K) (gpbasics/Statistics/CovarianceMatrix.py:267-275).
    ``gradient()[b]`` = d(-LML)/d(hyperparameters in DFS order) followed by d(-LML)/d(noise).
    """

    def __init__(self, n: int, d: int, batch: int = 1, dtype=None):
        super().__init__(n, d, n, batch, dtype)
        self.grad = None
        self.work = None

    def run(self, kd: nat.GpkKdesc, hyp: torch.Tensor, hyp_stride: int, noise: torch.Tensor,
            noise_stride: int, X: torch.Tensor, x_bstride: int, y: torch.Tensor, y_bstride: int,
            gradient: bool = True, **unused):
        """Enqueue the identity-augmented factorisation (+ gradient); single evaluations take the persistent
        launch like the value path and are verified at the first read (CHAIN_VERIFY)."""
        args = (kd, hyp, hyp_stride, noise, noise_stride, X, x_bstride, y, y_bstride, gradient)
        self._pending = None
        self._run_inverse(*args)
        self._defer_verify(lambda: self._run_inverse(*args))
        return self

    def _run_inverse(self, kd, hyp, hyp_stride, noise, noise_stride, X, x_bstride, y, y_bstride, gradient):
        lay = self.layout
        B, n, d = self.batch, self.n, self.d
        dev = self.W.device
        self._alphas = None
        self._fresh_out()
        _check_operand("hyper_parameter", hyp, hyp_stride, kd.n_hyp, B, dev)
        _check_operand("noise", noise, noise_stride, 1, B, dev)
        _check_operand("X", X, x_bstride, n * d, B, dev)
        _check_operand("y", y, y_bstride, n, B, dev)
        L = self.L
        grad_ptr = work_ptr = None
        work_bytes = 0
        if gradient:
            work_bytes = int(L.gpk_grad_workspace_bytes(ctypes.byref(kd), ctypes.byref(lay)))
            if self.work is None or self.work.numel() * 8 < work_bytes:
                self.work = torch.empty(max(1, work_bytes // 8), dtype=torch.float64, device=dev)
            self.grad = torch.empty((B, kd.n_hyp + 1), dtype=torch.float64, device=dev)
            grad_ptr, work_ptr = nat.ptr(self.grad), nat.ptr(self.work)
        else:
            self.grad = None
        nat.check(L.gpk_nlml_grad(ctypes.byref(kd), ctypes.byref(lay), nat.ptr(hyp), hyp_stride,
                                  nat.ptr(noise), noise_stride, nat.ptr(X), x_bstride, nat.ptr(y), y_bstride,
                                  nat.ptr(self.W), nat.ptr(self.Winv), nat.ptr(self.info), nat.ptr(self.out),
                                  grad_ptr, work_ptr, work_bytes, nat.stream_handle(dev)), "gpk_nlml_grad")
        self.kd = kd
        self.done = True
        return self

    def gradient(self) -> torch.Tensor:
        """[batch, n_hyp + 1] fp64: d(-LML)/d hyp (DFS order), then d(-LML)/d noise."""
        self._settle()
        if self.grad is None:
            raise RuntimeError("run(..., gradient=True) first")
        return self.grad

    def k_inv(self, b: int = 0) -> torch.Tensor:
        """(K + noise I)^-1, symmetrised from the corner's lower triangle."""
        return -self.corner(b)

    def l_inv(self, b: int = 0) -> torch.Tensor:
        """L^-1 (lower): the transpose of the extra rows, which hold L^-T."""
        return torch.triu(self.extra_rows(b)).transpose(0, 1)

    def alpha(self, b: int = 0) -> torch.Tensor:
        lay = self.layout
        return -self.w(b)[lay.y_row, lay.n_pad:lay.n_pad + self.n].to(torch.float64)


def _offset_ptr(t: torch.Tensor, elements: int):
    """ctypes pointer to element ``elements`` of t (for per-member launches)."""
    return ctypes.c_void_p(t.data_ptr() + int(elements) * t.element_size())


class RaggedFactorization(AugmentedFactorization):
    """One factorisation of independent problems of DIFFERENT sizes (gpk_*_ragged).

    Member b has ``sizes[b]`` training points and ``test_sizes[b]`` test points; the layout is
    planned for the largest member and every smaller member's block is completed with identity
    rows (training) or zero rows (test), which the device skips tile by tile.  This replaces the
    reference's one-segment-at-a-time loops over constituent GPs (SegmentedCovarianceMatrix
    get_*_blocks, gpbasics/Statistics/CovarianceMatrix.py:289-565; BlockwiseLogLikelihood,
    gpbasics/Metrics/LogLikelihood.py:68-104) by one set of batched launches: the panel chain is
    paid once for all segments instead of once per segment.

    Members may carry different kernel trees (the children of a change-point or partition
    operator): members sharing one device program are assembled by one launch, the others by a
    launch each; the factorisation and read-out are always one set of launches.
    """

    def __init__(self, sizes: Sequence[int], d: int, test_sizes: Optional[Sequence[int]] = None, dtype=None):
        sizes = [int(s) for s in sizes]
        if not sizes or min(sizes) < 1:
            raise ValueError("every member of a ragged batch needs at least one training point")
        tsz = [int(s) for s in test_sizes] if test_sizes is not None else [0] * len(sizes)
        if len(tsz) != len(sizes) or min(tsz) < 0:
            raise ValueError("test_sizes must hold one count >= 0 per member")
        super().__init__(max(sizes), d, max(tsz), len(sizes), dtype)
        self.sizes, self.test_sizes = sizes, tsz
        dev = self.W.device
        self.n_dev = torch.tensor(sizes, dtype=torch.int64, device=dev)
        self.m_dev = torch.tensor(tsz, dtype=torch.int64, device=dev)

    def run(self, members: Sequence, noise) -> "RaggedFactorization":
        """members[b] = (kdesc, hyp [n_hyp] fp64, X_b [n_b, d], y_b [n_b], Xs_b [m_b, d] or None);
        noise: rank-0 or one value per member."""
        self._pending = None
        B, n, m, d = self.batch, self.n, self.m, self.d
        self._alphas = None
        if len(members) != B:
            raise ValueError("expected %d members, got %d" % (B, len(members)))
        dev = self.W.device
        X = torch.zeros((B, n, d), dtype=torch.float64, device=dev)
        y = torch.zeros((B, n), dtype=torch.float64, device=dev)
        Xs = torch.zeros((B, max(m, 1), d), dtype=torch.float64, device=dev)
        hyp = torch.zeros((B, nat.MAX_HYP), dtype=torch.float64, device=dev)
        kds = []
        for b, (kd, h, xb, yb, xsb) in enumerate(members):
            nb, mb = self.sizes[b], self.test_sizes[b]
            if tuple(xb.shape) != (nb, d) or yb.numel() != nb:
                raise ValueError("member %d: X must be [%d, %d] and y hold %d values" % (b, nb, d, nb))
            if h.numel() != kd.n_hyp:
                raise ValueError("member %d: %d hyperparameters, kernel expects %d" % (b, h.numel(), kd.n_hyp))
            X[b, :nb] = xb
            y[b, :nb] = yb.reshape(-1)
            if mb:
                if xsb is None or tuple(xsb.shape) != (mb, d):
                    raise ValueError("member %d: X_test must be [%d, %d]" % (b, mb, d))
                Xs[b, :mb] = xsb
            hyp[b, :kd.n_hyp] = h
            kds.append(kd)
        nz = noise if isinstance(noise, torch.Tensor) else torch.as_tensor(noise, dtype=torch.float64)
        nz = nz.detach().to(device=dev, dtype=torch.float64).reshape(-1)
        nz = (nz.expand(B) if nz.numel() == 1 else nz).contiguous()
        if nz.numel() != B:
            raise ValueError("noise must be rank-0 or hold one value per member")
        L, s = self.L, nat.stream_handle(dev)
        lay = self.layout
        self.info.zero_()
        mptr = nat.ptr(self.m_dev) if m else None
        xs_ptr = nat.ptr(Xs) if m else None
        if all(bytes(k) == bytes(kds[0]) for k in kds):
            nat.check(L.gpk_assemble_ragged(ctypes.byref(kds[0]), ctypes.byref(lay), nat.ptr(hyp), nat.MAX_HYP,
                                            nat.ptr(nz), 1, nat.ptr(X), n * d, xs_ptr, max(m, 1) * d,
                                            nat.ptr(y), n, nat.ptr(self.n_dev), mptr, nat.ptr(self.W), s),
                      "gpk_assemble_ragged")
        else:
            one = nat.plan(self.code, 1, n, m, d)   # same p / ld as the batched layout
            for b, kd in enumerate(kds):
                nat.check(L.gpk_assemble_ragged(
                    ctypes.byref(kd), ctypes.byref(one), _offset_ptr(hyp, b * nat.MAX_HYP), 0,
                    _offset_ptr(nz, b), 0, _offset_ptr(X, b * n * d), 0,
                    _offset_ptr(Xs, b * max(m, 1) * d) if m else None, 0, _offset_ptr(y, b * n), 0,
                    _offset_ptr(self.n_dev, b), _offset_ptr(self.m_dev, b) if m else None,
                    _offset_ptr(self.W, b * lay.w_batch_stride), s), "gpk_assemble_ragged")
        nat.check(L.gpk_potrf_aug_ragged(ctypes.byref(lay), nat.ptr(self.W), nat.ptr(self.Winv),
                                         nat.ptr(self.info), nat.ptr(self.n_dev), mptr, s), "gpk_potrf_aug_ragged")
        nat.check(L.gpk_finalize_ragged(ctypes.byref(lay), nat.ptr(self.W), nat.ptr(self.info),
                                        nat.ptr(self.n_dev), nat.ptr(self.out),
                                        nat.ptr(self.mu) if m else None, nat.ptr(self.var) if m else None, s),
                  "gpk_finalize_ragged")
        self._keep = (X, y, Xs, hyp, nz)  # operands stay alive until the stream has consumed them
        self.kd = kds
        self.done = True
        return self

    # -- per-member read-out ------------------------------------------------------------------
    def cholesky(self, b: int = 0) -> torch.Tensor:
        nb = self.sizes[b]
        return torch.tril(self.w(b)[:nb, :nb])

    def z(self, b: int = 0) -> torch.Tensor:
        return self.w(b)[self.layout.y_row, :self.sizes[b]]

    def extra_rows(self, b: int = 0) -> torch.Tensor:
        lay = self.layout
        return self.w(b)[lay.n_pad:lay.n_pad + self.test_sizes[b], :self.sizes[b]]

    def corner(self, b: int = 0) -> torch.Tensor:
        lay, mb = self.layout, self.test_sizes[b]
        c = self.w(b)[lay.n_pad:lay.n_pad + mb, lay.n_pad:lay.n_pad + mb]
        return torch.tril(c) + torch.tril(c, -1).transpose(0, 1)

    def posterior_mu(self, b: int = 0) -> torch.Tensor:
        return self.mu[b * self.m:b * self.m + self.test_sizes[b]]

    def posterior_var_diag(self, b: int = 0) -> torch.Tensor:
        return self.var[b * self.m:b * self.m + self.test_sizes[b]]

    def alphas(self) -> List[torch.Tensor]:
        """alpha_b = L_b^-T z_b for every member: one batched backward solve (gpk_trsv; a member's
        padding rows carry z = 0), computed once per run."""
        if getattr(self, "_alphas", None) is None:
            lay = self.layout
            x = torch.zeros((self.batch, lay.n_pad), dtype=torch.float64, device=self.W.device)
            x[:, :self.n] = self.W.view(self.batch, lay.p, lay.ld)[:, lay.y_row, :self.n]
            nat.check(self.L.gpk_trsv(ctypes.byref(lay), 1, nat.ptr(self.W), nat.ptr(self.Winv),
                                      nat.ptr(x), nat.stream_handle(self.W.device)), "gpk_trsv")
            self._alphas = [x[b, :self.sizes[b]] for b in range(self.batch)]
        return self._alphas

    def alpha(self, b: int = 0) -> torch.Tensor:
        return self.alphas()[b]


def gemv(A: torch.Tensor, x: torch.Tensor, y: Optional[torch.Tensor] = None, alpha: float = 1.0,
         beta: float = 0.0) -> torch.Tensor:
    """y <- alpha A x + beta y on the device (gpk_gemv; A row-major fp64 [n, m], x [m] or [m, 1]).
    Returns y with x's trailing shape ([n] or [n, 1])."""
    if A.dim() != 2 or A.dtype != torch.float64 or A.stride(1) != 1:
        raise ValueError("A must be a row-major float64 matrix")
    n, m = int(A.shape[0]), int(A.shape[1])
    xv = x.reshape(-1)
    if xv.numel() != m or xv.dtype != torch.float64:
        raise ValueError("x must hold %d float64 values" % m)
    xv = xv.contiguous()
    out_shape = (n, 1) if x.dim() == 2 else (n,)
    if y is None:
        y = torch.empty(out_shape, dtype=torch.float64, device=A.device)
        beta = 0.0
    elif y.numel() != n or not y.is_contiguous():
        raise ValueError("y must be a contiguous tensor of %d values" % n)
    nat.check(nat.lib().gpk_gemv(nat.ptr(A), n, m, int(A.stride(0)), nat.ptr(xv), nat.ptr(y), float(alpha),
                                 float(beta), nat.stream_handle(A.device)), "gpk_gemv")
    return y


# ----------------------------------------------------------------------------- approximation paths
# Dense device building blocks of the Nystroem / SKC / SKI matrices (include/gpk.h
# "approximation paths").  Matrices are row-major fp64 device tensors, [n, m] or batched [B, n, m].
def _mat_args(t: torch.Tensor, name: str):
    if t.dtype != torch.float64 or t.device != device():
        raise ValueError("%s must be a float64 tensor on %s" % (name, device()))
    if t.dim() == 2:
        t = t.unsqueeze(0)
    if t.dim() != 3 or t.stride(2) != 1:
        raise ValueError("%s must be a row-major [n, m] or [B, n, m] matrix" % name)
    return t, int(t.stride(1)), int(t.stride(0)) if t.shape[0] > 1 else 0


def dgemm(A: torch.Tensor, B: torch.Tensor, trans_a: bool = False, trans_b: bool = False, alpha: float = 1.0,
          beta: float = 0.0, C: Optional[torch.Tensor] = None) -> torch.Tensor:
    """C <- alpha op(A) op(B) + beta C on f64 MFMA (gpk_dgemm); the tf.matmul / tf.tensordot products
    of gpbasics/Statistics/Nystroem_K.py and Metrics/StructuredKernelInterpolation.py."""
    squeeze = A.dim() == 2 and B.dim() == 2 and (C is None or C.dim() == 2)
    A3, lda, abs_ = _mat_args(A, "A")
    B3, ldb, bbs = _mat_args(B, "B")
    batch = max(A3.shape[0], B3.shape[0])
    if A3.shape[0] not in (1, batch) or B3.shape[0] not in (1, batch):
        raise ValueError("batch sizes of A and B differ")
    M = A3.shape[2] if trans_a else A3.shape[1]
    K = A3.shape[1] if trans_a else A3.shape[2]
    Kb = B3.shape[2] if trans_b else B3.shape[1]
    N = B3.shape[1] if trans_b else B3.shape[2]
    if K != Kb:
        raise ValueError("inner dimensions differ: %d vs %d" % (K, Kb))
    if C is None:
        C3 = torch.empty((batch, M, N), dtype=torch.float64, device=A.device)
        beta = 0.0
    else:
        C3 = C.unsqueeze(0) if C.dim() == 2 else C
        if tuple(C3.shape) != (batch, M, N) or not C3.is_contiguous():
            raise ValueError("C must be a contiguous [%d, %d, %d] tensor" % (batch, M, N))
    nat.check(nat.lib().gpk_dgemm(int(trans_a), int(trans_b), M, N, K, float(alpha), nat.ptr(A3), lda, abs_,
                                  nat.ptr(B3), ldb, bbs, float(beta), nat.ptr(C3), N, M * N, batch,
                                  nat.stream_handle(A.device)), "gpk_dgemm")
    return C3[0] if squeeze else C3


def syevj(A: torch.Tensor, max_sweeps: int = 60):
    """Eigendecomposition of a symmetric [m, m] (or [B, m, m]) device matrix by two-sided Jacobi
    (gpk_syevj): returns (lam [.., m], V [.., m, m] with the eigenvectors in its columns, sweeps)."""
    A3, lda, abs_ = _mat_args(A, "A")
    batch, m = A3.shape[0], A3.shape[1]
    if A3.shape[2] != m:
        raise ValueError("A must be square")
    L = nat.lib()
    V = torch.empty((batch, m, m), dtype=torch.float64, device=A.device)
    lam = torch.empty((batch, m), dtype=torch.float64, device=A.device)
    wb = int(L.gpk_syevj_workspace_bytes(m, batch))
    work = torch.empty(max(1, (wb + 7) // 8), dtype=torch.float64, device=A.device)
    sweeps = ctypes.c_int32(0)
    nat.check(L.gpk_syevj(m, batch, nat.ptr(A3), lda, abs_, nat.ptr(V), nat.ptr(lam), nat.ptr(work), wb,
                          int(max_sweeps), ctypes.byref(sweeps), nat.stream_handle(A.device)), "gpk_syevj")
    if A.dim() == 2:
        return lam[0], V[0], int(sweeps.value)
    return lam, V, int(sweeps.value)


def syevd(A: torch.Tensor):
    """Eigendecomposition of a symmetric [m, m] (or [B, m, m]) device matrix by the tridiagonal route
    (gpk_syevd: blocked Householder tridiagonalisation, divide and conquer on the tridiagonal matrix,
    compact-WY back-transformation): returns (lam, V with the eigenvectors in its columns), eigenvalues in no
    particular order (any m up to gpk_syevd's cap, 46340)."""
    A3, lda, abs_ = _mat_args(A, "A")
    batch, m = A3.shape[0], A3.shape[1]
    if A3.shape[2] != m:
        raise ValueError("A must be square")
    L = nat.lib()
    V = torch.empty((batch, m, m), dtype=torch.float64, device=A.device)
    lam = torch.empty((batch, m), dtype=torch.float64, device=A.device)
    wb = int(L.gpk_syevd_workspace_bytes(m))
    work = torch.empty(max(1, (wb + 7) // 8), dtype=torch.float64, device=A.device)
    nat.check(L.gpk_syevd(m, batch, nat.ptr(A3), lda, abs_, nat.ptr(V), nat.ptr(lam), nat.ptr(work), wb,
                          nat.stream_handle(A.device)), "gpk_syevd")
    if A.dim() == 2:
        return lam[0], V[0]
    return lam, V


def eigh(A: torch.Tensor):
    """The product's symmetric eigensolver: syevd (tridiagonal route); returns (lam, V, 0) like syevj."""
    lam, V = syevd(A)
    return lam, V, 0


def pinv_factor(lam: torch.Tensor, V: torch.Tensor, mode: int, rcond: float = -1.0, return_mu: bool = False):
    """U = V diag(mu) with tf.linalg.pinv's cutoff (gpk_pinv_factor): mode 0 mu = 1/lam (pinv = U V^T),
    mode 1 mu = lam^-1/2 (pinv = U U^T), mode 2 mu = |lam|^-1/2 (pinv = U diag(sign lam) U^T).  Returns (U, rank
    [B] int32 device tensor) (+ mu)."""
    squeeze = V.dim() == 2
    V3 = V.unsqueeze(0) if squeeze else V
    lam2 = lam.unsqueeze(0) if lam.dim() == 1 else lam
    batch, m = V3.shape[0], V3.shape[1]
    U = torch.empty_like(V3)
    mu = torch.empty((batch, m), dtype=torch.float64, device=V.device)
    rank = torch.empty(batch, dtype=torch.int32, device=V.device)
    nat.check(nat.lib().gpk_pinv_factor(m, batch, nat.ptr(V3.contiguous()), nat.ptr(lam2.contiguous()),
                                        float(rcond), int(mode), nat.ptr(mu), nat.ptr(U), nat.ptr(rank),
                                        nat.stream_handle(V.device)), "gpk_pinv_factor")
    if return_mu:
        return (U[0] if squeeze else U), rank, (mu[0] if squeeze else mu)
    return (U[0] if squeeze else U), rank


def pinv_sym(A: torch.Tensor, rcond: float = -1.0) -> torch.Tensor:
    """tf.linalg.pinv of a symmetric matrix (gpbasics/Statistics/Nystroem_K.py:53): the eigendecomposition
    (:func:`eigh`, gpk_syevd), the reference's cutoff 10 m eps max|lam|, then V diag(1/lam) V^T on MFMA."""
    lam, V, _ = eigh(A)
    U, _ = pinv_factor(lam, V, 0, rcond)
    return dgemm(U, V, trans_b=True)


def pinv_backward(lam: torch.Tensor, V: torch.Tensor, mu: torch.Tensor, Pbar: Optional[torch.Tensor] = None,
                  T: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Adjoint of a symmetric A from the adjoint Pbar of pinv(A) (tf.linalg.pinv's reverse mode,
    gpbasics/Statistics/Nystroem_K.py:53): V (F o sym(V^T Pbar V)) V^T with the Daleckii-Krein quotients of
    f = 1/lam over the kept eigenvalues (gpk_pinv_backward_scale); lam, V from :func:`eigh`, mu the mode-0
    factors of :func:`pinv_factor`.  T: the adjoint already in the eigenbasis (V^T Pbar V) instead."""
    m = int(V.shape[-1])
    if T is None:
        T = dgemm(dgemm(V, Pbar.contiguous(), trans_a=True), V)
    T = T.contiguous().clone()
    nat.check(nat.lib().gpk_pinv_backward_scale(m, 1, nat.ptr(lam.contiguous()), nat.ptr(mu.contiguous()),
                                                nat.ptr(T), nat.stream_handle(V.device)), "gpk_pinv_backward_scale")
    return dgemm(dgemm(V, T), V, trans_b=True)


def kernel_vjp(kernel, hyper_parameter, X, Z, G: Optional[torch.Tensor] = None, gu: Optional[torch.Tensor] = None,
               gv: Optional[torch.Tensor] = None, want_z: bool = False):
    """Reverse mode of K = kernel(X, Z) (gpk_kernel_vjp) for the adjoint G [n, m] of K, or the rank-1
    adjoint gu gv^T: returns (flat hyperparameter adjoint [n_hyp], adjoint of Z [m, d] or None)."""
    L = nat.lib()
    X = as_device_f64(X)
    Z = as_device_f64(Z)
    n, d = int(X.shape[0]), int(X.shape[1])
    m = int(Z.shape[0])
    kd = kernel_descriptor(kernel, d)
    hyp = pack_hyper_parameter(hyper_parameter, kd.n_hyp)
    gh = torch.zeros(max(1, kd.n_hyp), dtype=torch.float64, device=X.device)
    gz = torch.zeros((m, d), dtype=torch.float64, device=X.device) if want_z else None
    if n == 0 or m == 0:
        return gh[:kd.n_hyp], gz
    if G is not None:
        G = G.to(dtype=torch.float64)
        if G.dim() != 2 or tuple(G.shape) != (n, m) or G.stride(1) != 1:
            raise ValueError("G must be a row-major [%d, %d] matrix" % (n, m))
        ldg = int(G.stride(0))
    else:
        gu = gu.reshape(-1).to(dtype=torch.float64).contiguous()
        gv = gv.reshape(-1).to(dtype=torch.float64).contiguous()
        if gu.numel() != n or gv.numel() != m:
            raise ValueError("rank-1 weights must hold %d and %d values" % (n, m))
        ldg = m
    wb = int(L.gpk_kernel_vjp_workspace_bytes(ctypes.byref(kd), n, m, d, int(want_z)))
    work = torch.empty(max(1, (wb + 7) // 8), dtype=torch.float64, device=X.device)
    nat.check(L.gpk_kernel_vjp(ctypes.byref(kd), nat.ptr(hyp), nat.ptr(X), n, nat.ptr(Z), m, d,
                               nat.ptr(G) if G is not None else None, ldg,
                               nat.ptr(gu) if G is None else None, nat.ptr(gv) if G is None else None,
                               nat.ptr(gh), nat.ptr(gz) if want_z else None, nat.ptr(work), wb,
                               nat.stream_handle(X.device)), "gpk_kernel_vjp")
    return gh[:kd.n_hyp], gz


def ski_weights(X: torch.Tensor, Z: torch.Tensor) -> torch.Tensor:
    """SKI interpolation weights [n, m] (gpk_ski_weights; StructuredKernelInterpolation.py:31-49)."""
    X = as_device_f64(X)
    Z = as_device_f64(Z)
    n, d = X.shape
    m = Z.shape[0]
    Wm = torch.empty((n, m), dtype=torch.float64, device=X.device)
    work = torch.empty(2 * n + 1, dtype=torch.float64, device=X.device)
    nat.check(nat.lib().gpk_ski_weights(nat.ptr(X), n, nat.ptr(Z), m, d, nat.ptr(Wm), nat.ptr(work),
                                        nat.stream_handle(X.device)), "gpk_ski_weights")
    return Wm


def add_diagonal(A: torch.Tensor, value: float) -> torch.Tensor:
    """A += value * I in place (gpk_add_diagonal)."""
    A3, lda, abs_ = _mat_args(A, "A")
    n = min(A3.shape[1], A3.shape[2])
    nat.check(nat.lib().gpk_add_diagonal(nat.ptr(A3), n, lda, abs_, A3.shape[0], float(value),
                                         nat.stream_handle(A.device)), "gpk_add_diagonal")
    return A


class DenseFactorization(AugmentedFactorization):
    """Augmented factorisation of a caller-supplied dense SPD matrix A + noise I (gpk_assemble_dense):
    the approximate covariance matrices of the metrics (Nystroem, SKI) go through the same blocked
    Cholesky as K.  ``inverse=True`` carries identity extra rows, so the corner holds -(A + noise I)^-1
    (read out by :meth:`k_inv`); ``m`` > 0 with explicit rows E gives -E A^-1 E^T in the corner."""

    def __init__(self, n: int, m: int = 0, batch: int = 1, inverse: bool = False):
        self.inverse = bool(inverse)
        super().__init__(n, 1, n if inverse else m, batch, torch.float64)

    def run(self, A: torch.Tensor, noise, y: Optional[torch.Tensor] = None, E: Optional[torch.Tensor] = None):
        self._pending = None
        self._run_once(A, noise, y, E)
        self._defer_verify(lambda: self._run_once(A, noise, y, E))
        return self

    def _run_once(self, A, noise, y, E):
        A3, lda, abs_ = _mat_args(A, "A")
        B, n = self.batch, self.n
        if A3.shape[1] < n or A3.shape[2] < n or A3.shape[0] not in (1, B):
            raise ValueError("A must hold [%d, %d] per member" % (n, n))
        dev = self.W.device
        noise_t = torch.as_tensor(noise, dtype=torch.float64).to(dev).reshape(-1).contiguous()
        if noise_t.numel() not in (1, B):
            raise ValueError("noise must be a scalar or one value per member")
        ns = 1 if noise_t.numel() == B and B > 1 else 0
        if y is None:
            y = torch.zeros(n, dtype=torch.float64, device=dev)
        y = y.to(device=dev, dtype=torch.float64).contiguous()
        ybs = n if y.numel() == B * n and B > 1 else 0
        _check_operand("y", y, ybs, n, B, dev)
        ebs = 0
        if self.m and not self.inverse:
            if E is None:
                raise ValueError("m = %d extra rows need E" % self.m)
            E = E.to(device=dev, dtype=torch.float64).contiguous()
            ebs = self.m * n if E.numel() == B * self.m * n and B > 1 else 0
            _check_operand("E", E, ebs, self.m * n, B, dev)
        s = nat.stream_handle(dev)
        L = self.L
        lay = self.layout
        self.info.zero_()
        self._alphas = None
        nat.check(L.gpk_assemble_dense(ctypes.byref(lay), nat.ptr(A3), lda, abs_, nat.ptr(noise_t), ns,
                                       nat.ptr(E) if E is not None else None, ebs, int(self.inverse),
                                       nat.ptr(y), ybs, nat.ptr(self.W), s), "gpk_assemble_dense")
        nat.check(L.gpk_potrf_aug_ex(ctypes.byref(lay), nat.ptr(self.W), nat.ptr(self.Winv), nat.ptr(self.info),
                                     nat.AUG_EXTRA_IDENTITY if self.inverse else 0, s), "gpk_potrf_aug_ex")
        nat.check(L.gpk_finalize(ctypes.byref(lay), nat.ptr(self.W), nat.ptr(self.info), nat.ptr(self.out),
                                 nat.ptr(self.mu) if self.m else None, nat.ptr(self.var) if self.m else None, s),
                  "gpk_finalize")
        self.done = True
        return self

    def k_inv(self, b: int = 0) -> torch.Tensor:
        if not self.inverse:
            raise RuntimeError("DenseFactorization(..., inverse=True) carries the inverse")
        return -self.corner(b)
