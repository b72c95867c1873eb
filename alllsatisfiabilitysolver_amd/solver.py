"""Host-side Python front-end of the MI355X solver (over the C-ABI, liballl.so).

Two layers:
  * `Solver` -- a thin owner of one `alll_ctx` with numpy in/out (tests, bench, CLI).
  * `SATInstance` / `VariablesArray` / `Clause` / `Statistics` -- the reference's API shape
    (library/include/SATInstance.h:25-66, :156-173; VariablesArray.h:17-35; Clause.h:17-28)
    for Python callers.  C++ callers use include/alll_compat/SATInstance.h instead.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _native as N

_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def _p(a, t):
    return a.ctypes.data_as(t)


# ------------------------------------------------------------------ instance helpers
def generate_ksat(gen_seed: int, n_vars: int, n_clauses: int, k: int, kind: int = 0,
                  c_begin: int = 0, c_end: Optional[int] = None):
    """Random k-SAT, k distinct variables per clause (kind 0 uniform, 1 power-law).
    Returns (offsets uint64[m+1], literals uint32[m*k]) for clauses [c_begin, c_end)."""
    c_end = n_clauses if c_end is None else c_end
    lits = np.empty((c_end - c_begin) * k, np.uint32)
    N.check(N.lib().alll_generate_ksat(gen_seed, n_vars, n_clauses, k, kind, c_begin, c_end,
                                       _p(lits, _u32p)), "generate_ksat")
    offs = np.arange(c_end - c_begin + 1, dtype=np.uint64) * np.uint64(k)
    return offs, lits


def generate_mixed(gen_seed: int, n_vars: int, n_clauses: int, w_min: int, w_max: int):
    """Random clauses of mixed widths (uniform in [w_min, w_max]), variables and signs uniform
    (a variable may repeat inside a clause, as DIMACS allows).  Returns (offsets uint64[m+1],
    literals uint32[L]); deterministic for a seed (numpy PCG64)."""
    rng = np.random.default_rng(gen_seed)
    w = rng.integers(w_min, w_max + 1, n_clauses, dtype=np.int64)
    offs = np.zeros(n_clauses + 1, np.uint64)
    np.cumsum(w, out=offs[1:])
    L = int(offs[-1])
    v = rng.integers(0, n_vars, L, dtype=np.uint32)
    sgn = rng.integers(0, 2, L, dtype=np.uint32)
    return offs, (v << np.uint32(1)) | sgn


def assignment_digest(words) -> str:
    """64-bit FNV-1a over the bit-packed assignment's uint32 words (one xor-multiply step per
    word), as 16 hex digits: the trajectory digest of tests/golden/bench_trajectory.json."""
    h = 0xCBF29CE484222325
    for w in np.ascontiguousarray(words, np.uint32).tolist():
        h = ((h ^ w) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def parse_dimacs(text: bytes):
    """DIMACS text -> (n_vars, offsets, literals) with the reference loader semantics."""
    L = N.lib()
    v, c, ln = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_uint64()
    rc = L.alll_dimacs_parse(text, len(text), ctypes.byref(v), ctypes.byref(c), None, None,
                             ctypes.byref(ln))
    if rc == N.ALLL_ERR_BAD_INPUT:
        N.check(rc, "dimacs")
    offs = np.zeros(c.value + 1, np.uint64)
    lits = np.zeros(max(1, ln.value), np.uint32)
    N.check(L.alll_dimacs_parse(text, len(text), ctypes.byref(v), ctypes.byref(c), _p(offs, _u64p),
                                _p(lits, _u32p), ctypes.byref(ln)), "dimacs")
    return int(v.value), offs, lits[: ln.value]


def read_dimacs(path: str):
    L = N.lib()
    v, c, ln = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_uint64()
    bp = os.fsencode(path)
    rc = L.alll_dimacs_read(bp, ctypes.byref(v), ctypes.byref(c), None, None, ctypes.byref(ln))
    if rc in (N.ALLL_ERR_BAD_INPUT, N.ALLL_ERR_IO):
        N.check(rc, f"dimacs {path}")
    offs = np.zeros(c.value + 1, np.uint64)
    lits = np.zeros(max(1, ln.value), np.uint32)
    N.check(L.alll_dimacs_read(bp, ctypes.byref(v), ctypes.byref(c), _p(offs, _u64p),
                               _p(lits, _u32p), ctypes.byref(ln)), f"dimacs {path}")
    return int(v.value), offs, lits[: ln.value]


# ----------------------------------------------------------------------------- Solver
class Solver:
    """Owns one device solver context (alll_ctx)."""

    def __init__(self, n_vars: int, offsets, literals, seed: int = 1, max_iters: int = 0,
                 device: int = -1, n_threads: int = 1, rank: int = 0, world: int = 1,
                 comm_id: Optional[bytes] = None, flags: int = 0, grid_rounds: int = 0,
                 exchange=None, stream_batch: int = 0, set_starts=None):
        self._L = N.lib()
        self.n_vars = int(n_vars)
        self.offsets = np.ascontiguousarray(offsets, np.uint64)
        self.literals = np.ascontiguousarray(literals, np.uint32)
        self.m = self.offsets.size - 1
        prob = N.Problem(self.n_vars, 0, self.m, _p(self.offsets, _u64p), _p(self.literals, _u32p))
        opt = N.Options()
        self._L.alll_default_options(ctypes.byref(opt))
        opt.seed, opt.max_iters, opt.device = seed, max_iters, device
        opt.n_threads, opt.rank, opt.world = n_threads, rank, world
        opt.flags, opt.grid_rounds = flags, grid_rounds
        opt.stream_batch = stream_batch  # > 0: streaming solve semantics (alll.h)
        # n_threads > 1: round-robin MIS over n_threads chunks (alll.h); set_starts = the
        # n_threads + 1 chunk boundaries, None = the example/main.cpp chunking
        if set_starts is not None:
            self._set_starts = np.ascontiguousarray(set_starts, np.uint64)
            opt.set_starts = _p(self._set_starts, _u64p)
        if comm_id is not None:
            ctypes.memmove(opt.comm_id, comm_id, 128)
        self._ctx = ctypes.c_void_p()
        N.check(self._L.alll_create(ctypes.byref(prob), ctypes.byref(opt), ctypes.byref(self._ctx)),
                "alll_create")
        self.world = world
        self.rank = rank
        self._xfn = None
        if exchange is not None:
            self.set_host_exchange(exchange)

    def set_host_exchange(self, exchange):
        """exchange(op, buf: numpy uint8 view, bytes_per_rank_or_total) -> None; see
        include/alll.h (ALLL_XCHG_*).  Used instead of RCCL (e.g. several ranks on one GPU)."""
        world = self.world

        def fn(user, op, buf, nbytes):
            try:
                total = nbytes * world if op == N.XCHG_ALLGATHER else nbytes
                arr = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(buf))
                exchange(op, arr, nbytes)
                return 0
            except Exception:  # reported as ALLL_ERR_RCCL by the library
                import traceback

                traceback.print_exc()
                return 1

        self._xfn = N.EXCHANGE_FN(fn)
        N.check(self._L.alll_set_host_exchange(self._ctx, self._xfn, None), "set_host_exchange")

    # lifecycle
    def close(self):
        if getattr(self, "_ctx", None) and self._ctx.value:
            self._L.alll_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # loop
    def solve(self) -> dict:
        st = N.Stats()
        rc = self._L.alll_solve(self._ctx, ctypes.byref(st))
        if rc not in (N.ALLL_OK, N.ALLL_ERR_MAX_ITERS):
            N.check(rc, "alll_solve")
        return st.as_dict()

    def run(self, n_iters: int, sync: bool = True) -> Optional[dict]:
        if sync:
            st = N.Stats()
            N.check(self._L.alll_run(self._ctx, n_iters, ctypes.byref(st)), "alll_run")
            return st.as_dict()
        N.check(self._L.alll_run(self._ctx, n_iters, None), "alll_run")
        return None

    def synchronize(self):
        N.check(self._L.alll_synchronize(self._ctx), "alll_synchronize")

    def stats(self) -> dict:
        st = N.Stats()
        N.check(self._L.alll_get_stats(self._ctx, ctypes.byref(st)), "alll_get_stats")
        return st.as_dict()

    def verify(self):
        ok = ctypes.c_int()
        nv = ctypes.c_uint64()
        N.check(self._L.alll_verify(self._ctx, ctypes.byref(ok), ctypes.byref(nv)), "alll_verify")
        return bool(ok.value), int(nv.value)

    # state access
    def assignment_words(self) -> np.ndarray:
        w = np.zeros((self.n_vars + 31) // 32, np.uint32)
        N.check(self._L.alll_get_assignment_words(self._ctx, _p(w, _u32p), w.size), "get_assignment")
        return w

    def set_assignment_words(self, w):
        w = np.ascontiguousarray(w, np.uint32)
        N.check(self._L.alll_set_assignment_words(self._ctx, _p(w, _u32p), w.size), "set_assignment")

    def assignment(self) -> np.ndarray:
        a = np.zeros(max(1, self.n_vars), np.uint8)
        N.check(self._L.alll_get_assignment(self._ctx, _p(a, _u8p), a.size), "get_assignment")
        return a[: self.n_vars]

    def set_assignment(self, a):
        a = np.ascontiguousarray(a, np.uint8)
        N.check(self._L.alll_set_assignment(self._ctx, _p(a, _u8p), a.size), "set_assignment")

    def violated_mask(self) -> np.ndarray:
        w = np.zeros(max(1, (self.m + 63) // 64), np.uint64)
        N.check(self._L.alll_get_violated_mask(self._ctx, _p(w, _u64p), w.size), "violated_mask")
        return w

    def mis(self) -> np.ndarray:
        n = ctypes.c_uint64()
        N.check(self._L.alll_get_mis(self._ctx, None, 0, ctypes.byref(n)), "get_mis")
        out = np.zeros(max(1, n.value), np.uint32)
        N.check(self._L.alll_get_mis(self._ctx, _p(out, _u32p), out.size, ctypes.byref(n)), "get_mis")
        return out[: n.value]

    # measurement
    def bench_eval(self, reps: int = 20):
        ms = ctypes.c_double()
        nv = ctypes.c_uint64()
        N.check(self._L.alll_bench_eval(self._ctx, reps, ctypes.byref(ms), ctypes.byref(nv)), "bench_eval")
        return float(ms.value), int(nv.value)

    def profile(self, n_iters: int) -> dict:
        pt = N.PhaseTimes()
        N.check(self._L.alll_profile(self._ctx, n_iters, ctypes.byref(pt)), "profile")
        return pt.as_dict()

    def loop_times(self, first_iter: int, n_iters: int) -> dict:
        """In-loop phase times of iterations [first_iter, first_iter+n_iters) from the kernels'
        own wall-clock stamps (needs flags |= FLAG_KERNEL_TIMING)."""
        pt = N.PhaseTimes()
        N.check(self._L.alll_loop_times(self._ctx, first_iter, n_iters, ctypes.byref(pt)), "loop_times")
        return pt.as_dict()

    def eval_bytes(self) -> int:
        return int(self._L.alll_eval_bytes(self._ctx))

    def layout(self) -> int:
        return int(self._L.alll_layout(self._ctx))

    def eval_kernel(self) -> str:
        return self._L.alll_eval_kernel(self._ctx).decode()

    def uses_graphs(self):
        """(True, "") when the loop replays captured hipGraphs; (False, reason) when it launches
        eagerly (ALLL_FLAG_NO_GRAPH, a host-staged exchange, or a failed capture)."""
        why = ctypes.c_char_p()
        r = int(self._L.alll_uses_graphs(self._ctx, ctypes.byref(why)))
        return r == 1, (why.value or b"").decode()

    def rr_pass_log(self):
        """Round robin: per pass of the last iteration (dirty entries, repair rounds, entries
        decided, decisions changed) of its incremental passes (measurement)."""
        return self._rr_log()[0]

    def rr_round_log(self):
        """Round robin: per pass of the last iteration, the repair's clock stamps (100 MHz;
        detect, wide repair, repair, rounds end, repair end, LDS loaded) and its rounds
        {entries, stamp}, then a row of k_fp_bbuild's phase stamps (measurement, written only
        with FLAG_KERNEL_TIMING; rows of 64 words, zeros where not reached)."""
        return self._rr_log()[1]

    def _rr_log(self):
        out = np.zeros(256 + 64 * 65, np.uint32)
        n = self._L.alll_rr_pass_log(self._ctx, _p(out, _u32p), out.size)
        if n < 0:
            N.check(n, "rr_pass_log")
        return out[:min(n, 256)].reshape(-1, 4), out[256:max(n, 256)].reshape(-1, 64)

    def rr_barrier_timeouts(self) -> int:
        """Round robin: wide-repair grid barriers that timed out since create (measurement)."""
        n = int(self._L.alll_rr_barrier_timeouts(self._ctx))
        if n < 0:
            raise N.AlllError(N.ALLL_ERR_HIP, "alll_rr_barrier_timeouts failed")
        return n

    def comm_size(self) -> int:
        """Ranks in the solve: the RCCL communicator's count (or world with a host exchange)."""
        n = int(self._L.alll_comm_size(self._ctx))
        if n < 1:
            raise N.AlllError(N.ALLL_ERR_RCCL, "ncclCommCount failed")
        return n


def device_count() -> int:
    return int(N.lib().alll_device_count())


def shard_plan(n_clauses: int, world: int, rank: int):
    """(clause_begin, clause_end, mask_words_per_rank) of `rank` in the clause-sharded mode."""
    b, e, w = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    N.check(N.lib().alll_shard_plan(n_clauses, world, rank, ctypes.byref(b), ctypes.byref(e),
                                    ctypes.byref(w)), "shard_plan")
    return int(b.value), int(e.value), int(w.value)


class _MultiPlan(ctypes.Structure):
    _fields_ = [("eval_us_1gpu", ctypes.c_double), ("eval_saved_us", ctypes.c_double),
                ("exchange_us", ctypes.c_double), ("violated_est", ctypes.c_double),
                ("plan", ctypes.c_int), ("pad", ctypes.c_int)]


def plan_multi_gpu(n_clauses: int, n_literals: int, n_vars: int, world: int) -> dict:
    """alll_plan_multi_gpu: {"plan": "shard" | "replicate", and the model's predicted
    microseconds} for one instance on `world` GPUs."""
    p = _MultiPlan()
    N.check(N.lib().alll_plan_multi_gpu(n_clauses, n_literals, n_vars, world, ctypes.byref(p)), "plan_multi_gpu")
    return {"plan": "shard" if p.plan == 1 else "replicate", "eval_us_1gpu": p.eval_us_1gpu,
            "eval_saved_us": p.eval_saved_us, "exchange_us": p.exchange_us, "violated_est": p.violated_est}


def gloo_exchange(group=None):
    """Host exchange over torch.distributed (gloo) for Solver(exchange=...)."""
    import torch
    import torch.distributed as dist

    def ex(op, arr, nbytes):
        world = dist.get_world_size(group)
        if op == N.XCHG_ALLGATHER:
            rank = dist.get_rank(group)
            mine = torch.from_numpy(arr[rank * nbytes:(rank + 1) * nbytes].copy())
            parts = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(world)]
            dist.all_gather(parts, mine, group=group)
            arr[:] = torch.cat(parts).numpy()
        else:
            t = torch.from_numpy(arr.view(np.uint32).astype(np.int64))
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            arr.view(np.uint32)[:] = (t.numpy() & 0xFFFFFFFF).astype(np.uint32)

    return ex


def comm_unique_id() -> bytes:
    buf = (ctypes.c_uint8 * 128)()
    N.check(N.lib().alll_comm_unique_id(buf), "comm_unique_id")
    return bytes(buf)


# ------------------------------------------------- reference-shaped API (SATInstance.h)
class Clause:
    """Clause<T> (Clause.h:17-28): encoded literals + the chunk id t_id."""

    def __init__(self, literals: Sequence[int], t_id: int = 0):
        self.literals = list(literals)
        self.t_id = t_id

    def is_not_satisfied(self, vars_) -> bool:  # Clause.h:34-46
        return not any((not vars_[l >> 1]) if (l & 1) else vars_[l >> 1] for l in self.literals)


class VariablesArray:
    """VariablesArray<T> (VariablesArray.h:17-35).  The initial values come from the device
    solver's Philox stream (seeded), not std::random_device."""

    def __init__(self, n_vars: int):
        self.n_vars = int(n_vars)
        self.vars = np.zeros(self.n_vars, np.bool_)


@dataclass
class Statistics:
    """Statistics (SATInstance.h:25-32)."""
    n_iterations: int = 0
    n_resamples: int = 0
    avg_mis_size: int = 0
    n_thread_resamples: List[int] = field(default_factory=list)


class SATInstance:
    """SATInstance<T> (SATInstance.h:39-452) over the MI355X solver.  `seed` and `device`
    are additive keyword arguments; existing call shapes are unchanged."""

    def __init__(self, var_arr: VariablesArray, n_threads: int, seed: int = 1, device: int = -1,
                 max_iters: int = 0):
        self.var_arr = var_arr
        self.n_vars = var_arr.n_vars
        self.n_clauses = 0
        self.n_threads = max(1, int(n_threads))
        self._seed, self._device, self._max_iters = seed, device, max_iters

    @staticmethod
    def _flatten(clauses):
        flat = [cl for chunk in clauses for cl in chunk]
        offs = np.zeros(len(flat) + 1, np.uint64)
        offs[1:] = np.cumsum([len(c.literals) for c in flat])
        lits = np.fromiter((l for c in flat for l in c.literals), np.uint32, int(offs[-1]))
        return offs, lits

    def solve(self, clauses, n_clauses: Optional[int] = None, batch_size: Optional[int] = None) -> Statistics:
        """solve(clauses) -- SATInstance.h:60-66; solve(getEnumeratedClause, n_clauses, batch_size)
        -- the streaming overload, SATInstance.h:70-153 (getEnumeratedClause(index, t_id) -> Clause)."""
        if callable(clauses):
            return self._solve_stream(clauses, int(n_clauses), int(batch_size))
        self.n_clauses += sum(len(c) for c in clauses)
        offs, lits = self._flatten(clauses)
        starts = None
        if self.n_threads > 1:  # the MIS works on the caller's chunks (SATInstance.h:270-276, 414-447)
            if len(clauses) != self.n_threads:
                raise ValueError(f"{self.n_threads} threads need {self.n_threads} clause chunks, got {len(clauses)}")
            starts = np.zeros(self.n_threads + 1, np.uint64)
            starts[1:] = np.cumsum([len(c) for c in clauses])
        with Solver(self.n_vars, offs, lits, seed=self._seed, device=self._device,
                    n_threads=self.n_threads, max_iters=self._max_iters, set_starts=starts) as s:
            d = s.solve()
            self.var_arr.vars[:] = s.assignment().astype(np.bool_)
        thr = [0] * self.n_threads
        thr[0] = d["n_resamples"]
        return Statistics(d["n_iterations"], d["n_resamples"], d["avg_mis_size"], thr)

    def _generated(self, fn, n_clauses: int):
        """Clauses 0 .. n-1 from the callback, each with the t_id of the generator whose range
        holds it (SATInstance.h:74-86: n / T each, the last one the remainder)."""
        T = self.n_threads
        per = n_clauses // T
        out = []
        for i in range(n_clauses):
            t = min(i // per, T - 1) if per else T - 1
            cl = fn(i, t)
            if cl is None:
                raise ValueError(f"clause generator returned None for index {i}")
            out.append(cl)
        return out

    def _solve_stream(self, fn, n_clauses: int, batch_size: int) -> Statistics:
        self.n_clauses = n_clauses
        offs, lits = self._flatten([self._generated(fn, n_clauses)])
        with Solver(self.n_vars, offs, lits, seed=self._seed, device=self._device, n_threads=self.n_threads,
                    max_iters=self._max_iters, stream_batch=max(1, batch_size)) as s:
            d = s.solve()
            self.var_arr.vars[:] = s.assignment().astype(np.bool_)
        thr = [0] * self.n_threads
        thr[0] = d["n_resamples"]
        return Statistics(d["n_iterations"], d["n_resamples"], d["avg_mis_size"], thr)

    def writeDIMACS(self, fn, n_clauses: int, out_f) -> None:  # SATInstance.h:175-203
        self.n_clauses = n_clauses
        out_f.write(f"p cnf {self.n_vars} {n_clauses}\n")
        for i in range(n_clauses):
            cl = fn(i, 0)
            if cl is None:
                raise ValueError(f"clause generator returned None for index {i}")
            toks = [str(-(l >> 1) - 1) if (l & 1) else str((l >> 1) + 1) for l in cl.literals]
            out_f.write("".join(" " + x for x in toks) + " 0\n")

    def verify_validity(self, clauses) -> bool:  # SATInstance.h:156-173
        v = self.var_arr.vars
        return not any(cl.is_not_satisfied(v) for chunk in clauses for cl in chunk)
