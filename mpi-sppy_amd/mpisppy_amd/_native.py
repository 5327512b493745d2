"""ctypes binding of libphgpu.so (the gfx950 HIP kernels behind include/phgpu.h).

The product path has no CPU fallback: if the library is missing, or no
MI355X is visible, the solver raises.  Device buffers are PyTorch-ROCm
tensors passed as raw pointers (``tensor.data_ptr()``).
"""
import ctypes
import os

import torch

_LIB_NAME = "libphgpu.so"
_LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")

_c_int = ctypes.c_int32
_c_dbl = ctypes.c_double
_c_ptr = ctypes.c_void_p


class PHGPUError(RuntimeError):
    """Raised when a libphgpu call returns a non-zero code."""


class SolveOpts(ctypes.Structure):
    _fields_ = [("tol", _c_dbl), ("max_iters", _c_int), ("check_every", _c_int),
                ("warm_start", _c_int), ("reflection", _c_dbl), ("polish", _c_int)]


DIAG_W = 5  # PH_DIAG_W in include/phgpu.h


class LoopPassArgs(ctypes.Structure):
    """ph_loop_pass_args of include/phgpu.h (field order and types exact)."""
    _fields_ = [("sums", _c_ptr), ("G", _c_int), ("gid", _c_ptr), ("rho", _c_ptr),
                ("w_coeff", _c_ptr), ("xbar", _c_ptr), ("xsqbar", _c_ptr), ("W", _c_ptr),
                ("absdiff", _c_ptr), ("wconv", _c_ptr), ("conv_hist", _c_ptr),
                ("conv_part", _c_ptr), ("x_save", _c_ptr), ("y_save", _c_ptr),
                ("status_save", _c_ptr), ("dbound_save", _c_ptr), ("w_on", _c_dbl),
                ("prox_on", _c_dbl), ("x", _c_ptr), ("y", _c_ptr), ("omega", _c_ptr),
                ("status", _c_ptr), ("iters", _c_ptr), ("pobj", _c_ptr), ("dbound", _c_ptr),
                ("opts", SolveOpts)]


# (name, restype, argtypes) -- must match include/phgpu.h exactly
SIGNATURES = [
    ("ph_version", ctypes.c_char_p, []),
    ("ph_last_error", ctypes.c_char_p, []),
    ("ph_batch_create", _c_int, [ctypes.POINTER(_c_ptr), _c_int, _c_int, _c_int, _c_int,
                                 _c_ptr, _c_ptr, _c_ptr]),
    ("ph_batch_set_stream", _c_int, [_c_ptr, _c_ptr]),
    ("ph_batch_bind", _c_int, [_c_ptr] + [_c_ptr] * 6),
    ("ph_batch_set_nonants", _c_int, [_c_ptr, _c_int, _c_ptr]),
    ("ph_batch_set_bounds", _c_int, [_c_ptr, _c_ptr, _c_ptr]),
    ("ph_pdhg_solve", _c_int, [_c_ptr, _c_ptr, _c_ptr, _c_ptr, _c_dbl, _c_dbl,
                               _c_ptr, _c_ptr, _c_ptr, _c_ptr, _c_ptr, _c_ptr, _c_ptr,
                               ctypes.POINTER(SolveOpts)]),
    ("ph_xbar_accum", _c_int, [_c_ptr, _c_ptr, _c_ptr, _c_int, _c_ptr, _c_ptr, _c_ptr, _c_ptr]),
    ("ph_update_w", _c_int, [_c_ptr, _c_ptr, _c_ptr, _c_int, _c_ptr, _c_ptr, _c_ptr,
                             _c_ptr, _c_ptr, _c_ptr, _c_ptr]),
    ("ph_segment_sum", _c_int, [_c_ptr, _c_ptr, _c_ptr, _c_int, _c_ptr, _c_ptr]),
    ("ph_eval_objective", _c_int, [_c_ptr, _c_ptr, _c_ptr, _c_ptr, _c_ptr, _c_dbl, _c_dbl, _c_ptr]),
    ("ph_gather", _c_int, [_c_ptr, _c_ptr, ctypes.c_int64, _c_ptr, _c_ptr, ctypes.c_int64, _c_ptr]),
    ("ph_batch_get_diag", _c_int, [_c_ptr, _c_ptr]),
    ("ph_batch_solve_summary", _c_int, [_c_ptr, _c_ptr]),
    ("ph_loop_reset", _c_int, [_c_ptr, _c_int, _c_int, _c_dbl]),
    ("ph_loop_enable", _c_int, [_c_ptr, _c_int]),
    ("ph_loop_set_xbar", _c_int, [_c_ptr, _c_ptr, _c_ptr, _c_int, _c_ptr, _c_ptr, _c_ptr, _c_ptr]),
    ("ph_loop_conv", _c_int, [_c_ptr, _c_ptr, _c_ptr, _c_int, _c_dbl, _c_ptr]),
    ("ph_loop_conv_local", _c_int, [_c_ptr, _c_ptr, _c_ptr, _c_int, _c_ptr, _c_dbl, _c_ptr,
                                    _c_ptr]),
    ("ph_loop_update_w_conv", _c_int, [_c_ptr, _c_ptr, _c_ptr, _c_int, _c_ptr, _c_ptr, _c_ptr,
                                       _c_ptr, _c_ptr, _c_ptr, _c_ptr, _c_ptr, _c_ptr]),
    ("ph_loop_conv_lagged", _c_int, [_c_ptr, _c_ptr, _c_ptr, _c_int, _c_dbl, _c_ptr]),
    ("ph_loop_backup", _c_int, [_c_ptr, _c_ptr, _c_ptr, ctypes.c_int64, _c_ptr, _c_ptr,
                                ctypes.c_int64]),
    ("ph_loop_backup_status", _c_int, [_c_ptr, _c_ptr, _c_ptr, _c_ptr, _c_ptr]),
    ("ph_loop_status", _c_int, [_c_ptr, _c_ptr]),
    ("ph_loop_bind_pass", _c_int, [_c_ptr, ctypes.POINTER(LoopPassArgs)]),
    ("ph_loop_pass", _c_int, [_c_ptr]),
    ("ph_loop_run", _c_int, [_c_ptr, _c_int]),
    ("ph_loop_persistent", _c_int, [_c_ptr]),
    ("ph_loop_fused", _c_int, [_c_ptr]),
    ("ph_loop_read_timing", _c_int, [_c_ptr, _c_ptr]),
    ("ph_batch_set_timing", _c_int, [_c_ptr, _c_int]),
    ("ph_batch_read_timing", _c_int, [_c_ptr, _c_ptr]),
    ("ph_batch_sync", _c_int, [_c_ptr]),
    ("ph_batch_destroy", None, [_c_ptr]),
]

_lib = None


def lib_path():
    return os.path.join(_LIB_DIR, _LIB_NAME)


def load():
    """Load libphgpu.so (once) and declare its C-ABI.  Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build the HIP library first "
            "(python -c 'import __graft_entry__ as g; g.build()' or make -C mpi-sppy_amd/csrc)")
    lib = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().ph_last_error().decode(errors="replace")
        raise PHGPUError(f"{what} failed (code {rc}): {msg}")


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("solvername 'mi355x_pdhg' needs a ROCm GPU (MI355X); none is visible")


def stream_handle(stream=None):
    s = torch.cuda.current_stream() if stream is None else stream
    return ctypes.c_void_p(s.cuda_stream)
