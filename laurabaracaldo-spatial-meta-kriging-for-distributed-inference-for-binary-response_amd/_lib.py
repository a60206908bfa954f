"""ctypes binding of include/mk.h (libmk.so, built in-tree for gfx950).

There is no fallback: if libmk.so is missing or cannot be loaded the import of
any compute entry point raises MkError.  Structures mirror include/mk.h field
for field.
"""
import ctypes
import os

import numpy as np

from ._build import LIB_PATH

MK_OK = 0
MK_E_ARG = -1
MK_E_HIP = -2
MK_E_NOMEM = -3
MK_E_NODEV = -4
MK_E_INTERRUPT = -5
MK_COMBINE_MEAN = 0
MK_COMBINE_MEDIAN = 1
MK_COV_EXPONENTIAL = 0
MK_COV_MATERN = 1
MK_LINK_LOGIT = 0
MK_LINK_PROBIT = 1
N_LEVELS = 200

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


class MkError(RuntimeError):
    """Raised for every non-zero libmk status (R glue: Rf_error)."""

    def __init__(self, code, msg):
        super().__init__(f"libmk error {code}: {msg}")
        self.code = code


class Problem(ctypes.Structure):
    _fields_ = [("n_subsets", ctypes.c_int32), ("subset_base", ctypes.c_int32), ("q", ctypes.c_int32),
                ("p", ctypes.c_int32), ("n_part", _ip), ("coords", _dp), ("y", _dp), ("weights", _dp),
                ("x", _dp), ("n_test", ctypes.c_int32), ("coords_test", _dp)]


class Config(ctypes.Structure):
    _fields_ = [("cov_model", ctypes.c_int32), ("n_batch", ctypes.c_int32), ("batch_length", ctypes.c_int32),
                ("accept_rate", ctypes.c_double), ("burn_in", ctypes.c_int32),
                ("beta_starting", _dp), ("beta_tuning", _dp), ("phi_starting", _dp), ("phi_tuning", _dp),
                ("A_starting", _dp), ("A_tuning", _dp), ("nu_starting", _dp), ("nu_tuning", _dp),
                ("w_starting", ctypes.c_double), ("w_tuning", ctypes.c_double),
                ("phi_unif_a", _dp), ("phi_unif_b", _dp), ("nu_unif_a", _dp), ("nu_unif_b", _dp),
                ("K_IW_df", ctypes.c_double), ("K_IW_S", _dp), ("seed", ctypes.c_uint64),
                ("record_samples", ctypes.c_int32), ("record_w", ctypes.c_int32), ("device", ctypes.c_int32),
                ("n_streams", ctypes.c_int32), ("predict_tile", ctypes.c_int32), ("link", ctypes.c_int32)]


class Outputs(ctypes.Structure):
    _fields_ = [("parameters", _dp), ("w_predict", _dp), ("samples", _dp), ("w_samples", _dp),
                ("w_pred_samples", _dp), ("acceptance", _dp), ("w_predict_sum", _dp)]


class Summary(ctypes.Structure):
    _fields_ = [("sample_par", _dp), ("sample_w", _dp), ("p_sample", _dp), ("w_quant", _dp),
                ("param_quant", _dp), ("p_quant", _dp), ("index", _ip)]


class Combined(ctypes.Structure):
    _fields_ = [("result", _dp), ("result2", _dp), ("method", ctypes.c_int32), ("max_iter", ctypes.c_int32),
                ("tol", ctypes.c_double), ("exchange", ctypes.c_int32), ("comm_ranks", ctypes.c_int32)]


# int (*mk_progress_fn)(void* user, int32_t iterations, int32_t n_samples)
PROGRESS_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32)

EXPORTS = {
    "mk_meta_fit": (ctypes.c_int, [ctypes.POINTER(Problem), ctypes.POINTER(Config), _ip, ctypes.c_int32,
                                   PROGRESS_FN, ctypes.c_void_p, ctypes.POINTER(Outputs), ctypes.POINTER(Combined)]),
    "mk_session_create": (ctypes.c_int, [ctypes.POINTER(Problem), ctypes.POINTER(Config), ctypes.POINTER(ctypes.c_void_p)]),
    "mk_session_run": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    "mk_session_iteration": (ctypes.c_int32, [ctypes.c_void_p]),
    "mk_session_predict_tile": (ctypes.c_int32, [ctypes.c_void_p]),
    "mk_session_chain_state": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, _dp, _dp, _dp, _dp, _dp]),
    "mk_session_set_lookahead": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    "mk_session_lookahead": (ctypes.c_int32, [ctypes.c_void_p]),
    "mk_session_outputs": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Outputs)]),
    "mk_session_set_test_sites": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]),
    "mk_session_grids": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]),
    "mk_session_tile_grids": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]),
    "mk_session_set_kept_window": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]),
    "mk_session_profile": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    "mk_session_profile_every": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    "mk_session_kernel_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64),
                                               _dp, _dp]),
    "mk_session_destroy": (None, [ctypes.c_void_p]),
    "mk_session_count": (ctypes.c_int32, []),
    "mk_fit_predict_batched": (ctypes.c_int, [ctypes.POINTER(Problem), ctypes.POINTER(Config), ctypes.POINTER(Outputs)]),
    "mk_combine": (ctypes.c_int, [_dp, ctypes.c_int32, ctypes.c_int64, _dp, ctypes.c_int32]),
    "mk_combine_sum": (ctypes.c_int, [_dp, ctypes.c_int32, ctypes.c_int64, _dp, ctypes.c_int32]),
    "mk_combine_median_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64,
                                                ctypes.c_int32, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_int32, ctypes.c_void_p]),
    "mk_combine_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]),
    "mk_combine_median": (ctypes.c_int, [_dp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                                         ctypes.c_double, _dp, _ip, ctypes.c_int32]),
    "mk_posterior_summary": (ctypes.c_int, [_dp, ctypes.c_int32, _dp, ctypes.c_int64, _dp, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_uint64, ctypes.POINTER(Summary),
                                            ctypes.c_int32]),
    "mk_posterior_summary_ex": (ctypes.c_int, [_dp, ctypes.c_int32, _dp, ctypes.c_int64, _dp, ctypes.c_int32,
                                               ctypes.c_int32, ctypes.c_uint64, _ip, ctypes.c_int32,
                                               ctypes.POINTER(Summary), ctypes.c_int32]),
    "mk_glm_binomial_link": (ctypes.c_int, [_dp, _dp, _dp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_double, ctypes.c_int32, _dp, _dp, _ip, ctypes.c_int32]),
    "mk_glm_binomial": (ctypes.c_int, [_dp, _dp, _dp, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                                       ctypes.c_int32, _dp, _dp, _ip, ctypes.c_int32]),
    "mk_correlation_batched": (ctypes.c_int, [_dp, ctypes.c_int32, ctypes.c_int32, _dp, _dp, ctypes.c_int32, _dp,
                                              ctypes.c_int32]),
    "mk_cholesky_batched": (ctypes.c_int, [_dp, ctypes.c_int32, ctypes.c_int32, _dp, _dp, _dp, ctypes.c_int32]),
    "mk_partition_r": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _ip, _ip]),
    "mk_r_sample": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _ip]),
    "mk_r_sample_replace": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _ip]),
    "mk_set_hw_queues": (ctypes.c_int, [ctypes.c_int32]),
    "mk_hip_initialized": (ctypes.c_int, []),
    "mk_shutdown": (None, []),
    "mk_set_watchdog": (ctypes.c_int, [ctypes.c_int32]),
    "mk_last_error": (ctypes.c_char_p, []),
    "mk_device_count": (ctypes.c_int, []),
    "mk_device_memory": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
}

_LIB = None
HW_QUEUES = None     # hardware queues of this process's HIP runtime, as passed to mk_set_hw_queues


def _hip_started():
    """True when this process's HIP runtime is already initialised (torch first, or any other
    library): a GPU_MAX_HW_QUEUES set now would no longer be read.  The process then holds /dev/kfd
    open (mk_hip_initialized checks the same without starting HIP)."""
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                if os.readlink("/proc/self/fd/" + fd) == "/dev/kfd":
                    return True
            except OSError:
                pass
    except OSError:
        pass
    return False


def load():
    """Load libmk.so (raises MkError if it is absent -- no CPU fallback exists)."""
    global _LIB, HW_QUEUES
    if _LIB is not None:
        return _LIB
    path = os.environ.get("MK_LIB") or LIB_PATH      # MK_LIB: a development build (tools/ probes)
    # the lookahead schedule runs up to five HIP streams: give the process 8 hardware queues when
    # HIP has not started yet (the variable is read once, when HIP initialises).  If it has started
    # (torch first), keep the count it started with and tell libmk, which then runs three streams
    # instead of five on too few queues.
    before = int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)
    if _hip_started():
        HW_QUEUES = before if before > 0 else 4
    else:
        if before < 8:
            os.environ["GPU_MAX_HW_QUEUES"] = "8"
        HW_QUEUES = max(before, 8)
    if not os.path.exists(path):
        raise MkError(MK_E_ARG, f"{path} not built; run __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    lib.mk_set_hw_queues(HW_QUEUES)
    # libmk's pooled streams (CU-masked / priority queues) are destroyed while the HIP runtime is
    # alive: Python's atexit runs before the C library's exit handlers (libmk registers mk_shutdown
    # there too; it is idempotent)
    import atexit
    atexit.register(lib.mk_shutdown)
    _LIB = lib
    return lib


def check(rc):
    if rc != MK_OK:
        raise MkError(rc, load().mk_last_error().decode())


def dptr(a):
    """Pointer to a C-contiguous float64 array (or NULL for None)."""
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


def iptr(a):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_ip)
