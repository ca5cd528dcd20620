"""ctypes binding of libgpk.so (the C ABI declared in include/gpk.h).

There is deliberately no CPU fallback: when the HIP extension cannot be loaded, or no GPU is
visible, every product entry point raises :class:`NativeUnavailable`.
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_size_t, c_void_p

import torch  # noqa: F401  (must be loaded first: libgpk binds to torch's HIP runtime by soname)

from . import _build

GPK_ABI_VERSION = 6
GPK_F64, GPK_F32 = 0, 1
OP_PER, OP_SE, OP_MAT32, OP_MAT52, OP_ADD, OP_MUL = 104, 105, 107, 108, 201, 202
NODE_SCALED, NODE_ARD, NODE_SE_EXPANDED, NODE_STANDARD = 1, 2, 4, 8
MAX_NODES, MAX_DIM, MAX_ARD, MAX_HYP = 16, 16, 2, 64
NUM_CLASSES = 7
TIMING_CLASSES = ("assemble", "diag", "trsm", "update", "finalize", "trsv", "grad")
AUG_EXTRA_IDENTITY = 1

# every function include/gpk.h declares (checked by tests/test_abi.py against the header)
EXPORTS = (
    "gpk_abi_version", "gpk_last_error", "gpk_plan", "gpk_assemble", "gpk_potrf_aug",
    "gpk_finalize", "gpk_nlml", "gpk_kernel_matrix", "gpk_trsv", "gpk_timing_enable",
    "gpk_timing_read", "gpk_timing_reset", "gpk_tune", "gpk_potrf_aug_ex", "gpk_assemble_inverse",
    "gpk_grad_workspace_bytes", "gpk_nlml_grad", "gpk_assemble_ragged", "gpk_potrf_aug_ragged",
    "gpk_finalize_ragged", "gpk_nlml_ragged", "gpk_gemv",
    "gpk_assemble_dense", "gpk_dgemm", "gpk_syevj_workspace_bytes", "gpk_syevj", "gpk_pinv_factor",
    "gpk_ski_weights", "gpk_add_diagonal", "gpk_distance_matrix", "gpk_workspace_bytes", "gpk_nlml_batched", "gpk_potrf_lower", "gpk_trsv_lower", "gpk_posterior",
    "gpk_kernel_vjp_workspace_bytes", "gpk_kernel_vjp", "gpk_pinv_backward_scale", "gpk_syevd_workspace_bytes",
    "gpk_syevd", "gpk_chain_plan", "gpk_tune_thread", "gpk_chain_stats", "gpk_chain_plan_ex",
)


class NativeUnavailable(RuntimeError):
    """libgpk.so (the HIP path) is missing or cannot run here."""


class GpkError(RuntimeError):
    """A libgpk call returned an error code."""


class GpkNode(ctypes.Structure):
    _fields_ = [("op", c_int32), ("hyp_offset", c_int32), ("ard_slot", c_int32), ("flags", c_int32)]


class GpkKdesc(ctypes.Structure):
    _fields_ = [("n_nodes", c_int32), ("n_hyp", c_int32), ("dim", c_int32), ("n_ard", c_int32),
                ("nodes", GpkNode * MAX_NODES)]


class GpkLayout(ctypes.Structure):
    _fields_ = [("dtype", c_int32), ("batch", c_int32), ("n", c_int64), ("m", c_int64),
                ("d", c_int64), ("nb", c_int64), ("n_pad", c_int64), ("y_row", c_int64),
                ("p", c_int64), ("ld", c_int64), ("w_batch_stride", c_int64),
                ("inv_batch_stride", c_int64), ("w_bytes", c_size_t), ("inv_bytes", c_size_t)]


_lock = threading.Lock()
_lib = None


def _declare(lib):
    P, D = c_void_p, POINTER(c_double)
    sig = {
        "gpk_abi_version": (c_int, []),
        "gpk_last_error": (ctypes.c_char_p, []),
        "gpk_plan": (c_int, [c_int, c_int32, c_int64, c_int64, c_int64, POINTER(GpkLayout)]),
        "gpk_assemble": (c_int, [POINTER(GpkKdesc), POINTER(GpkLayout), P, c_int64, P, c_int64,
                                 P, c_int64, P, c_int64, P, c_int64, P, c_int64, P, P]),
        "gpk_potrf_aug": (c_int, [POINTER(GpkLayout), P, P, P, P]),
        "gpk_finalize": (c_int, [POINTER(GpkLayout), P, P, P, P, P, P]),
        "gpk_nlml": (c_int, [POINTER(GpkKdesc), POINTER(GpkLayout), P, c_int64, P, c_int64, P,
                             c_int64, P, c_int64, P, P, P, P, P]),
        "gpk_kernel_matrix": (c_int, [POINTER(GpkKdesc), P, c_int, c_int, P, c_int64, P, c_int64,
                                      c_int32, c_double, P, c_int64, P]),
        "gpk_trsv": (c_int, [POINTER(GpkLayout), c_int, P, P, P, P]),
        "gpk_timing_enable": (c_int, [c_int]),
        "gpk_timing_read": (c_int, [D, POINTER(c_int64), D, D]),
        "gpk_timing_reset": (c_int, []),
        "gpk_tune": (c_int, [ctypes.c_char_p, c_int64, ctypes.POINTER(c_int64)]),
        "gpk_potrf_aug_ex": (c_int, [POINTER(GpkLayout), P, P, P, c_int32, P]),
        "gpk_assemble_inverse": (c_int, [POINTER(GpkKdesc), POINTER(GpkLayout), P, c_int64, P, c_int64,
                                         P, c_int64, P, c_int64, P, P]),
        "gpk_grad_workspace_bytes": (c_size_t, [POINTER(GpkKdesc), POINTER(GpkLayout)]),
        "gpk_nlml_grad": (c_int, [POINTER(GpkKdesc), POINTER(GpkLayout), P, c_int64, P, c_int64, P,
                                  c_int64, P, c_int64, P, P, P, P, P, P, c_size_t, P]),
        "gpk_assemble_ragged": (c_int, [POINTER(GpkKdesc), POINTER(GpkLayout), P, c_int64, P, c_int64,
                                        P, c_int64, P, c_int64, P, c_int64, P, P, P, P]),
        "gpk_potrf_aug_ragged": (c_int, [POINTER(GpkLayout), P, P, P, P, P, P]),
        "gpk_finalize_ragged": (c_int, [POINTER(GpkLayout), P, P, P, P, P, P, P]),
        "gpk_nlml_ragged": (c_int, [POINTER(GpkKdesc), POINTER(GpkLayout), P, c_int64, P, c_int64, P,
                                    c_int64, P, c_int64, P, P, P, P, P, P]),
        "gpk_gemv": (c_int, [P, c_int64, c_int64, c_int64, P, P, c_double, c_double, P]),
        "gpk_assemble_dense": (c_int, [POINTER(GpkLayout), P, c_int64, c_int64, P, c_int64, P, c_int64,
                                       c_int32, P, c_int64, P, P]),
        "gpk_dgemm": (c_int, [c_int32, c_int32, c_int64, c_int64, c_int64, c_double, P, c_int64, c_int64,
                              P, c_int64, c_int64, c_double, P, c_int64, c_int64, c_int32, P]),
        "gpk_syevj_workspace_bytes": (c_size_t, [c_int64, c_int32]),
        "gpk_syevj": (c_int, [c_int64, c_int32, P, c_int64, c_int64, P, P, P, c_size_t, c_int32,
                              POINTER(c_int32), P]),
        "gpk_pinv_factor": (c_int, [c_int64, c_int32, P, P, c_double, c_int32, P, P, P, P]),
        "gpk_ski_weights": (c_int, [P, c_int64, P, c_int64, c_int32, P, P, P]),
        "gpk_add_diagonal": (c_int, [P, c_int64, c_int64, c_int64, c_int32, c_double, P]),
        "gpk_distance_matrix": (c_int, [c_int, P, c_int64, c_int64, P, c_int64, c_int64, c_int32, c_int32, P,
                                        c_int64, c_int64, P]),
        "gpk_workspace_bytes": (c_size_t, [c_int, c_int, c_int64, c_int64, c_int32]),
        "gpk_nlml_batched": (c_int, [POINTER(GpkKdesc), c_int32, P, P, c_int, P, P, c_int64, c_int32, P, c_size_t,
                                     P, P, P]),
        "gpk_potrf_lower": (c_int, [c_int, P, c_int64, c_int64, P, c_size_t, P, P, P]),
        "gpk_trsv_lower": (c_int, [c_int, c_int, P, c_int64, c_int64, P, P, c_size_t, P]),
        "gpk_posterior": (c_int, [P, P, c_int, P, c_int64, P, P, c_int64, P, c_int64, c_int32, c_int32, P, P,
                                  c_int64, P, c_size_t, P]),
        "gpk_pinv_backward_scale": (c_int, [c_int64, c_int32, P, P, P, P]),
        "gpk_syevd_workspace_bytes": (c_size_t, [c_int64]),
        "gpk_syevd": (c_int, [c_int64, c_int32, P, c_int64, c_int64, P, P, P, c_size_t, P]),
        "gpk_chain_plan": (c_int, [c_int64, c_int64, c_int32, P, c_int64, POINTER(c_int64)]),
        "gpk_chain_plan_ex": (c_int, [c_int64, c_int64, c_int32, c_int32, P, c_int64, POINTER(c_int64)]),
        "gpk_tune_thread": (c_int, [ctypes.c_char_p, c_int64, c_int32, POINTER(c_int64), POINTER(c_int32)]),
        "gpk_chain_stats": (c_int, [POINTER(c_int64), c_int32]),
        "gpk_chain_trace": (c_int, [P, c_int64]),
        "gpk_chain_times": (c_int, [P, c_int64]),
        "gpk_kernel_vjp_workspace_bytes": (c_size_t, [POINTER(GpkKdesc), c_int64, c_int64, c_int32, c_int32]),
        "gpk_kernel_vjp": (c_int, [POINTER(GpkKdesc), P, P, c_int64, P, c_int64, c_int32, P, c_int64, P, P, P, P,
                                   P, c_size_t, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def load_library(path: str = None):
    """Load libgpk.so (no GPU needed for loading).  Raises NativeUnavailable if absent."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or os.environ.get("GPK_LIB", _build.LIB_PATH)
        if not os.path.exists(p):
            raise NativeUnavailable(
                "libgpk.so not found at %s: build it with __graft_entry__.build() "
                "(hipcc --offload-arch=gfx950); there is no CPU fallback" % p)
        try:
            lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise NativeUnavailable("cannot load %s: %s" % (p, e)) from e
        _declare(lib)
        v = lib.gpk_abi_version()
        if v != GPK_ABI_VERSION:
            raise NativeUnavailable("libgpk ABI %d != expected %d (stale build?)" % (v, GPK_ABI_VERSION))
        if path is None:
            _lib = lib
        return lib


def lib():
    """The loaded library, with a GPU visible (the only configuration the product runs in)."""
    L = load_library()
    if not torch.cuda.is_available():
        raise NativeUnavailable("no ROCm GPU visible: the gpk engine runs only on MI355X (gfx950)")
    return L


def check(rc: int, what: str):
    if rc != 0:
        msg = _lib.gpk_last_error().decode() if _lib is not None else ""
        raise GpkError("%s failed (rc=%d): %s" % (what, rc, msg))


def ptr(t) -> c_void_p:
    if t is None:
        return None
    return c_void_p(t.data_ptr())


def stream_handle(device=None) -> c_void_p:
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


def plan(dtype_code: int, batch: int, n: int, m: int, d: int) -> GpkLayout:
    lay = GpkLayout()
    check(load_library().gpk_plan(dtype_code, batch, n, m, d, ctypes.byref(lay)), "gpk_plan")
    return lay


def dtype_code(torch_dtype) -> int:
    if torch_dtype == torch.float64:
        return GPK_F64
    if torch_dtype == torch.float32:
        return GPK_F32
    raise ValueError("unsupported dtype %r (float64 or float32)" % (torch_dtype,))


def timing_enable(on: bool = True):
    check(load_library().gpk_timing_enable(1 if on else 0), "gpk_timing_enable")


def tune(key: str, value: int) -> int:
    """Set a scheduling knob of libgpk (see gpk_tune in include/gpk.h); returns the old value."""
    old = c_int64(0)
    check(load_library().gpk_tune(key.encode(), int(value), ctypes.byref(old)), "gpk_tune")
    return int(old.value)


class thread_tune:
    """Context manager pinning libgpk knobs for the calling thread only (gpk_tune_thread), e.g.
    ``with thread_tune(chain=0, lookahead=0): ...``; the thread's previous overrides come back on exit."""

    def __init__(self, **knobs):
        self.knobs = {k: int(v) for k, v in knobs.items()}
        self.saved = []

    def __enter__(self):
        L = load_library()
        for k, v in self.knobs.items():
            ov, os_ = c_int64(0), c_int32(0)
            check(L.gpk_tune_thread(k.encode(), v, 1, ctypes.byref(ov), ctypes.byref(os_)), "gpk_tune_thread")
            self.saved.append((k, int(ov.value), int(os_.value)))
        return self

    def __exit__(self, *exc):
        L = load_library()
        for k, v, was_set in reversed(self.saved):
            check(L.gpk_tune_thread(k.encode(), v, was_set, None, None), "gpk_tune_thread")
        self.saved = []
        return False


def chain_stats() -> dict:
    """gpk_chain_stats: persistent launches, launch-path decisions while another stream was busy, whether
    this thread's last factorisation was persistent, forced timeouts pending."""
    out = (c_int64 * 4)()
    check(load_library().gpk_chain_stats(out, 4), "gpk_chain_stats")
    return {"launches": int(out[0]), "declined_busy": int(out[1]), "last_was_chain": bool(out[2]),
            "forced_pending": int(out[3])}


def chain_timeouts() -> int:
    """Persistent launches on the current device whose waits timed out since the library was loaded (each set
    info = -1 on its unfinished members; forced timeouts count too).  A device read: it waits for the work
    enqueued so far, so callers read it outside timed regions."""
    out = (c_int64 * 5)()
    check(load_library().gpk_chain_stats(out, 5), "gpk_chain_stats")
    return int(out[4])


def last_factorisation_was_chain() -> bool:
    out = (c_int64 * 3)()
    check(load_library().gpk_chain_stats(out, 3), "gpk_chain_stats")
    return bool(out[2])


CHAIN_PLAN_F32 = 256  # gpk_chain_plan_ex flag (include/gpk.h GPK_CHAIN_PLAN_F32)


def chain_plan(n_pad: int, y_row: int, grid: int, eye: bool = False, f32: bool = False):
    """Task list of the persistent single-member factorisation (gpk_chain_plan_ex; host only): an
    [ntasks, 4] int32 array of (type word, k, r, j) in claim order; eye: the identity-augmented list; f32: the
    plan of an f32 factorisation (chain_kernel<float>)."""
    import numpy as np
    L = load_library()
    nt = c_int64(0)
    fl = (AUG_EXTRA_IDENTITY if eye else 0) | (CHAIN_PLAN_F32 if f32 else 0)
    check(L.gpk_chain_plan_ex(int(n_pad), int(y_row), int(grid), fl, None, 0, ctypes.byref(nt)), "gpk_chain_plan_ex")
    out = np.zeros((int(nt.value), 4), dtype=np.int32)
    check(L.gpk_chain_plan_ex(int(n_pad), int(y_row), int(grid), fl, c_void_p(out.ctypes.data), int(nt.value),
                              ctypes.byref(nt)), "gpk_chain_plan_ex")
    return out


def timing_reset():
    check(load_library().gpk_timing_reset(), "gpk_timing_reset")


def timing_read() -> dict:
    ms = (c_double * NUM_CLASSES)()
    nl = (c_int64 * NUM_CLASSES)()
    fl = (c_double * NUM_CLASSES)()
    by = (c_double * NUM_CLASSES)()
    check(load_library().gpk_timing_read(ms, nl, fl, by), "gpk_timing_read")
    return {name: {"ms": ms[i], "launches": nl[i], "flops": fl[i], "bytes": by[i]}
            for i, name in enumerate(TIMING_CLASSES)}
