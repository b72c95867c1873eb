"""ctypes binding of the C-ABI in include/alll.h (liballl.so, built in-tree by `make`).

The product path is liballl.so only: if the library is missing or fails to load, every
entry point raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "liballl.so")
if os.environ.get("ALLL_LIB_AB"):  # development A/B timing of two builds (tools/ab_bench.sh)
    LIB_PATH = os.path.abspath(os.environ["ALLL_LIB_AB"])

ALLL_OK = 0
ALLL_ERR_INVALID_ARG = 1
ALLL_ERR_BAD_INPUT = 2
ALLL_ERR_LITERAL_RANGE = 3
ALLL_ERR_HIP = 4
ALLL_ERR_RCCL = 5
ALLL_ERR_MAX_ITERS = 6
ALLL_ERR_NO_DEVICE = 7
ALLL_ERR_OOM = 8
ALLL_ERR_IO = 9
ALLL_ERR_UNSUPPORTED = 10

FLAG_NO_GRAPH = 1 << 0
FLAG_EXCHANGE_ALLREDUCE = 1 << 1
FLAG_GENERIC_CSR = 1 << 2
FLAG_NO_RANGED = 1 << 3
FLAG_KERNEL_TIMING = 1 << 4
FLAG_ATOMIC_CLAIMS = 1 << 5
FLAG_LFMIS = 1 << 6
FLAG_REFERENCE_RNG = 1 << 7

MAX_GPU_STATS = 64

# Every symbol include/alll.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "alll_version", "alll_last_error", "alll_default_options", "alll_device_count",
    "alll_comm_unique_id", "alll_create", "alll_destroy", "alll_set_host_exchange", "alll_solve", "alll_run",
    "alll_get_stats", "alll_verify", "alll_get_assignment", "alll_set_assignment",
    "alll_get_assignment_words", "alll_set_assignment_words", "alll_get_violated_mask",
    "alll_get_mis", "alll_bench_eval", "alll_profile", "alll_loop_times", "alll_synchronize", "alll_eval_bytes",
    "alll_layout", "alll_eval_kernel", "alll_comm_size", "alll_uses_graphs", "alll_rr_pass_log", "alll_rr_barrier_timeouts", "alll_initial_assignment", "alll_reference_initial_assignment", "alll_shard_plan", "alll_plan_multi_gpu", "alll_dimacs_parse", "alll_dimacs_read", "alll_generate_ksat",
]


class AlllError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"alll error {code}: {msg}")
        self.code = code


class Problem(ctypes.Structure):
    _fields_ = [
        ("n_vars", ctypes.c_uint32),
        ("pad", ctypes.c_uint32),
        ("n_clauses", ctypes.c_uint64),
        ("offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("literals", ctypes.POINTER(ctypes.c_uint32)),
    ]


class Options(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("max_iters", ctypes.c_uint64),
        ("device", ctypes.c_int32),
        ("n_threads", ctypes.c_int32),
        ("rank", ctypes.c_int32),
        ("world", ctypes.c_int32),
        ("comm_id", ctypes.c_uint8 * 128),
        ("flags", ctypes.c_uint32),
        ("grid_rounds", ctypes.c_uint32),
        ("stream_batch", ctypes.c_uint64),
        ("set_starts", ctypes.POINTER(ctypes.c_uint64)),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("n_iterations", ctypes.c_uint64),
        ("n_resamples", ctypes.c_uint64),
        ("avg_mis_size", ctypes.c_uint64),
        ("sum_mis_size", ctypes.c_uint64),
        ("n_violated", ctypes.c_uint64),
        ("solved", ctypes.c_int32),
        ("n_gpus", ctypes.c_int32),
        ("lfmis_rounds_max", ctypes.c_uint32),
        ("lfmis_tail_rounds", ctypes.c_uint32),
        ("gpu_resamples", ctypes.c_uint64 * MAX_GPU_STATS),
    ]

    def as_dict(self):
        d = {k: int(getattr(self, k)) for k, _ in self._fields_ if k != "gpu_resamples"}
        d["gpu_resamples"] = [int(x) for x in self.gpu_resamples[: max(1, self.n_gpus)]]
        return d


class PhaseTimes(ctypes.Structure):
    _fields_ = [
        ("eval_ms", ctypes.c_double),
        ("exchange_ms", ctypes.c_double),
        ("mis_ms", ctypes.c_double),
        ("resample_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double),
        ("iterations", ctypes.c_uint64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p

EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_uint64)
XCHG_ALLGATHER = 0
XCHG_ALLREDUCE_SUM_U32 = 1

_SIGS = {
    "alll_version": ([], ctypes.c_char_p),
    "alll_last_error": ([], ctypes.c_char_p),
    "alll_default_options": ([ctypes.POINTER(Options)], None),
    "alll_device_count": ([], ctypes.c_int),
    "alll_comm_unique_id": ([ctypes.POINTER(ctypes.c_uint8)], ctypes.c_int),
    "alll_create": ([ctypes.POINTER(Problem), ctypes.POINTER(Options), ctypes.POINTER(_vp)], ctypes.c_int),
    "alll_destroy": ([_vp], ctypes.c_int),
    "alll_set_host_exchange": ([_vp, EXCHANGE_FN, _vp], ctypes.c_int),
    "alll_solve": ([_vp, ctypes.POINTER(Stats)], ctypes.c_int),
    "alll_run": ([_vp, ctypes.c_uint64, ctypes.POINTER(Stats)], ctypes.c_int),
    "alll_get_stats": ([_vp, ctypes.POINTER(Stats)], ctypes.c_int),
    "alll_verify": ([_vp, ctypes.POINTER(ctypes.c_int), _u64p], ctypes.c_int),
    "alll_get_assignment": ([_vp, _u8p, ctypes.c_uint64], ctypes.c_int),
    "alll_set_assignment": ([_vp, _u8p, ctypes.c_uint64], ctypes.c_int),
    "alll_get_assignment_words": ([_vp, _u32p, ctypes.c_uint64], ctypes.c_int),
    "alll_set_assignment_words": ([_vp, _u32p, ctypes.c_uint64], ctypes.c_int),
    "alll_get_violated_mask": ([_vp, _u64p, ctypes.c_uint64], ctypes.c_int),
    "alll_get_mis": ([_vp, _u32p, ctypes.c_uint64, _u64p], ctypes.c_int),
    "alll_bench_eval": ([_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double), _u64p], ctypes.c_int),
    "alll_profile": ([_vp, ctypes.c_uint64, ctypes.POINTER(PhaseTimes)], ctypes.c_int),
    "alll_loop_times": ([_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(PhaseTimes)], ctypes.c_int),
    "alll_synchronize": ([_vp], ctypes.c_int),
    "alll_eval_bytes": ([_vp], ctypes.c_uint64),
    "alll_layout": ([_vp], ctypes.c_int),
    "alll_eval_kernel": ([_vp], ctypes.c_char_p),
    "alll_comm_size": ([_vp], ctypes.c_int),
    "alll_uses_graphs": ([_vp, ctypes.POINTER(ctypes.c_char_p)], ctypes.c_int),
    "alll_rr_pass_log": ([_vp, _u32p, ctypes.c_uint32], ctypes.c_int),
    "alll_rr_barrier_timeouts": ([_vp], ctypes.c_int64),
    "alll_shard_plan": ([ctypes.c_uint64, ctypes.c_int, ctypes.c_int, _u64p, _u64p, _u64p], ctypes.c_int),
    "alll_reference_initial_assignment": ([ctypes.c_uint64, ctypes.c_uint32, _u8p], ctypes.c_int),
    "alll_plan_multi_gpu": ([ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p],
                            ctypes.c_int),
    "alll_initial_assignment": ([ctypes.c_uint64, ctypes.c_uint32, _u8p], ctypes.c_int),
    "alll_dimacs_parse": ([ctypes.c_char_p, ctypes.c_uint64, _u32p, _u64p, _u64p, _u32p, _u64p], ctypes.c_int),
    "alll_dimacs_read": ([ctypes.c_char_p, _u32p, _u64p, _u64p, _u32p, _u64p], ctypes.c_int),
    "alll_generate_ksat": ([ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                            ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, _u32p], ctypes.c_int),
}

_lib = None


def build(force: bool = False):
    """Compile liballl.so for gfx950 in-tree (hipcc via the top-level Makefile)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", ROOT, "all"], check=True)


def lib():
    """Load liballl.so; raises if it is absent (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def last_error() -> str:
    return lib().alll_last_error().decode(errors="replace")


def check(rc: int, what: str = ""):
    if rc != ALLL_OK:
        raise AlllError(rc, f"{what}: {last_error()}" if what else last_error())
    return rc
