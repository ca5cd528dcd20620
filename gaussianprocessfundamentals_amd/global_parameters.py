"""Process-wide configuration, mirroring gpbasics/global_parameters.py.

Same contract as the reference: call :func:`init` once before importing the kernel,
covariance, metric or GP modules; they call :func:`ensure_init` at import time and the process
exits with status -100 when it was never called (global_parameters.py:24-28).

Flags read on the hot path:
  p_dtype                    arithmetic type of the factorisation (global_parameters.py:43);
                             torch.float64 (default) or torch.float32 (f32 MFMA path)
  p_cov_matrix_jitter        default noise added to the training diagonal (:45)
  p_scaled_base_kernel       base kernels carry a signal-variance hyperparameter (:62)
  p_batch_metric_aggregator  reduction over BatchDataInput members (:64), torch.mean
Build-specific knobs (not in the reference):
  p_device                   torch device of the engine ("cuda" = the current MI355X)
  p_stationary_distance      "reference" (default: L1 distance in MAT / PER, as the reference) or
                             "standard" (Euclidean MAT, per-dimension PER; PD for any D)
  p_se_expanded_norm         SE distance by the reference's expanded norm (Distances.py:4-7,
                             NaN where rounding makes it negative) instead of the direct sum of
                             squares (default False; identical where the reference is finite)
"""
from __future__ import annotations

import logging
import os
import sys
from enum import Enum

import torch


class ChangePointOperatorType(Enum):
    SIGMOID = 0
    INDICATOR = 1
    APPROX_INDICATOR = 2


initiated = False
p_dtype = torch.float64
p_cov_matrix_jitter = None
p_scaled_base_kernel = False
p_batch_metric_aggregator = None
p_optimize_noise = False
p_check_hyper_parameters = False
p_nystroem_ratio = 0.1
p_max_threads = 1
p_logging_level = logging.INFO
p_scale_data_y = True
p_cp_operator_type = ChangePointOperatorType.INDICATOR
p_used_base_kernel = []
p_used_base_mean_functions = []
p_device = "cuda"
p_se_expanded_norm = False
p_stationary_distance = "reference"
pool = None


def ensure_init():
    if not initiated:
        logging.warning("Global parameters not initiated!")
        sys.exit(-100)


def init(tf_parallel: int = 0, worker: bool = False, device: str = "cuda"):
    """Initialise the globals.  ``tf_parallel`` sizes the host thread pool (the reference sized
    TensorFlow's intra/inter-op pools with it, global_parameters.py:38-39)."""
    global initiated, p_dtype, p_cov_matrix_jitter, p_scaled_base_kernel, p_batch_metric_aggregator
    global p_optimize_noise, p_check_hyper_parameters, p_nystroem_ratio, p_max_threads, p_logging_level
    global p_scale_data_y, p_cp_operator_type, p_used_base_kernel, p_used_base_mean_functions
    global p_device, p_se_expanded_norm, p_stationary_distance, pool
    if tf_parallel and tf_parallel > 0:
        torch.set_num_threads(int(tf_parallel))
    initiated = True
    p_dtype = torch.float64
    p_cov_matrix_jitter = torch.tensor(1e-8, dtype=torch.float64)
    p_optimize_noise = False
    p_check_hyper_parameters = False
    p_nystroem_ratio = 0.1
    p_used_base_kernel = []
    p_used_base_mean_functions = []
    p_max_threads = max(1, (os.cpu_count() or 1) - max(0, int(tf_parallel)))
    p_logging_level = logging.INFO
    p_scaled_base_kernel = False
    p_batch_metric_aggregator = torch.mean
    p_scale_data_y = True
    p_cp_operator_type = ChangePointOperatorType.INDICATOR
    p_device = device
    p_se_expanded_norm = False
    p_stationary_distance = "reference"
    pool = None
    logging.basicConfig(format="%(levelname)s: %(message)s", level=p_logging_level)
    logging.info("Process-%s:Initialization of global parameters finished." % os.getpid())


def set_up_pool(maxtasksperchild: int = -1):
    """The reference creates a multiprocessing pool that nothing uses; kept as a
    no-op for API compatibility: the engine's parallelism is the GPU and torch.distributed."""
    global pool
    pool = None


def shutdown_pool():
    global pool
    pool = None
