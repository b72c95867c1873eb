"""MI355X-native Moser-Tardos (Algorithmic Lovasz Local Lemma) SAT solver.

The hot path -- clause evaluation, violated-clause compaction, exact lexicographically-first
MIS and Philox resampling -- runs in hand-written gfx950 HIP kernels behind the C-ABI of
include/alll.h (liballl.so).  This package is the Python front-end of that library.
"""
from ._native import AlllError, build, lib  # noqa: F401
from .solver import (Clause, SATInstance, Solver, Statistics, VariablesArray,  # noqa: F401
                     assignment_digest, comm_unique_id, device_count, generate_ksat, generate_mixed, gloo_exchange,
                     parse_dimacs,
                     read_dimacs, shard_plan, plan_multi_gpu)

__version__ = "0.1.0"
