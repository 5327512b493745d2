"""mpisppy_amd -- MI355X-native progressive-hedging hot path.

A drop-in for mpi-sppy's PH solve loop and nonanticipativity updates
(``mpisppy/phbase.py``, ``mpisppy/opt/ph.py``): the scenario subproblems are
solved as one batch by hand-written gfx950 HIP kernels (libphgpu.so, C-ABI in
``include/phgpu.h``); xbar / W / convergence reductions run on device with
RCCL allreduce across ranks (one rank per GPU).
"""
import time

__version__ = "0.1.0"

SOLVER_NAMES = ("mi355x_pdhg", "pdhg_gpu")

_t0 = time.perf_counter()
_toc_quiet = False


def global_toc(msg, cond=True):
    """``mpisppy/__init__.py:26`` analogue: timestamped progress line."""
    if cond and not _toc_quiet:
        print(f"[{time.perf_counter() - _t0:8.2f}] {msg}", flush=True)


def disable_tictoc_output():
    global _toc_quiet
    _toc_quiet = True


def reenable_tictoc_output():
    global _toc_quiet
    _toc_quiet = False
