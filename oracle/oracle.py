"""TEST INFRASTRUCTURE ONLY -- numpy/ctypes front-end of the plain-C oracle.

The oracle (oracle/alll_oracle.c) is a CPU restatement of the reference's serial
Moser-Tardos loop (SATInstance.h:217-320 with one thread).  It is the parity checker
for the HIP product path: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and never as the thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PROBE = os.path.join(HERE, "_ref", "ref_probe")

_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u8p = ctypes.POINTER(ctypes.c_uint8)


class OrcStats(ctypes.Structure):
    _fields_ = [
        ("n_iterations", ctypes.c_uint64),
        ("n_resamples", ctypes.c_uint64),
        ("avg_mis_size", ctypes.c_uint64),
        ("sum_mis_size", ctypes.c_uint64),
        ("last_violated", ctypes.c_uint64),
        ("solved", ctypes.c_int32),
        ("pad", ctypes.c_int32),
    ]


ITER_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                           ctypes.c_uint64, ctypes.c_uint64, _u32p)

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_philox4x32_10.argtypes = [_u32p, _u32p, _u32p]
        L.orc_init_assignment.argtypes = [ctypes.c_uint64, ctypes.c_uint32, _u32p]
        L.orc_resample_bit.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        L.orc_resample_bit.restype = ctypes.c_uint32
        L.orc_generate_ksat.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                        ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64,
                                        ctypes.c_uint64, _u32p]
        L.orc_eval.argtypes = [ctypes.c_uint64, _u64p, _u32p, _u32p, _u64p]
        L.orc_eval.restype = ctypes.c_uint64
        L.orc_mask_to_list.argtypes = [ctypes.c_uint64, _u64p, _u32p]
        L.orc_mask_to_list.restype = ctypes.c_uint64
        L.orc_lfmis.argtypes = [ctypes.c_uint32, _u64p, _u32p, _u32p, ctypes.c_uint64, _u32p, _u8p]
        L.orc_lfmis.restype = ctypes.c_uint64
        L.orc_chunk_bounds.argtypes = [ctypes.c_uint64, ctypes.c_uint32, _u64p]
        L.orc_rr_mis.argtypes = [ctypes.c_uint32, _u64p, _u32p, _u32p, ctypes.c_uint64,
                                 ctypes.c_uint32, _u64p, _u32p, _u8p]
        L.orc_rr_mis.restype = ctypes.c_uint64
        L.orc_solve.argtypes = [ctypes.c_uint32, ctypes.c_uint64, _u64p, _u32p, ctypes.c_uint64,
                                ctypes.c_uint64, _u32p, ctypes.POINTER(OrcStats), ITER_CB,
                                ctypes.c_void_p]
        L.orc_solve.restype = ctypes.c_int
        L.orc_solve_rr.argtypes = [ctypes.c_uint32, ctypes.c_uint64, _u64p, _u32p, ctypes.c_uint64,
                                   ctypes.c_uint64, ctypes.c_uint32, _u64p, _u32p, ctypes.POINTER(OrcStats),
                                   ITER_CB, ctypes.c_void_p]
        L.orc_solve_rr.restype = ctypes.c_int
        L.orc_stream_order.argtypes = [ctypes.c_uint64, _u32p]
        L.orc_stream_order.restype = None
        L.orc_solve_stream.argtypes = [ctypes.c_uint32, ctypes.c_uint64, _u64p, _u32p, ctypes.c_uint64,
                                       ctypes.c_uint64, ctypes.c_uint64, _u32p, ctypes.POINTER(OrcStats),
                                       ITER_CB, ctypes.c_void_p]
        L.orc_solve_stream.restype = ctypes.c_int
        L.orc_solve_stream_rr.argtypes = [ctypes.c_uint32, ctypes.c_uint64, _u64p, _u32p, ctypes.c_uint64,
                                          ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                          _u32p, ctypes.POINTER(OrcStats), ITER_CB, ctypes.c_void_p]
        L.orc_solve_stream_rr.restype = ctypes.c_int
        L.orc_solve_refrng.argtypes = [ctypes.c_uint32, ctypes.c_uint64, _u64p, _u32p, ctypes.c_uint64,
                                       ctypes.c_uint64, _u32p, ctypes.POINTER(OrcStats), ITER_CB, ctypes.c_void_p]
        L.orc_solve_refrng.restype = ctypes.c_int
        L.orc_solve_stream_refrng.argtypes = [ctypes.c_uint32, ctypes.c_uint64, _u64p, _u32p, ctypes.c_uint64,
                                              ctypes.c_uint64, ctypes.c_uint64, _u32p, ctypes.POINTER(OrcStats),
                                              ITER_CB, ctypes.c_void_p]
        L.orc_solve_stream_refrng.restype = ctypes.c_int
        L.orc_refrng_init.argtypes = [_u64p, ctypes.c_uint32, _u32p]
        L.orc_refrng_init.restype = None
        L.orc_dimacs_parse.argtypes = [ctypes.c_char_p, ctypes.c_uint64, _u32p, _u64p, _u64p,
                                       _u32p, _u64p]
        L.orc_dimacs_parse.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


# --------------------------------------------------------------------------- RNG
def philox4x32_10(ctr, key):
    c = np.asarray(ctr, np.uint32).copy()
    k = np.asarray(key, np.uint32).copy()
    o = np.zeros(4, np.uint32)
    lib().orc_philox4x32_10(_p(c, _u32p), _p(k, _u32p), _p(o, _u32p))
    return o


def init_assignment(seed, n_vars):
    A = np.zeros((n_vars + 31) // 32, np.uint32)
    lib().orc_init_assignment(seed, n_vars, _p(A, _u32p))
    return A


def resample_bit(seed, it, v):
    return int(lib().orc_resample_bit(seed, it, v))


# --------------------------------------------------------------------- instances
def generate_ksat(gen_seed, n_vars, n_clauses, k, kind=0):
    """Uniform (kind=0) or power-law (kind=1) random k-SAT with distinct variables per
    clause.  Returns (offsets uint64[m+1], literals uint32[m*k])."""
    lits = np.zeros(n_clauses * k, np.uint32)
    rc = lib().orc_generate_ksat(gen_seed, n_vars, n_clauses, k, kind, 0, n_clauses,
                                 _p(lits, _u32p))
    if rc != 0:
        raise ValueError("bad generator arguments")
    offs = np.arange(n_clauses + 1, dtype=np.uint64) * np.uint64(k)
    return offs, lits


def csr_from_lists(clauses):
    """clauses: list of lists of encoded literals (2v + neg)."""
    offs = np.zeros(len(clauses) + 1, np.uint64)
    offs[1:] = np.cumsum([len(c) for c in clauses])
    lits = np.array([l for c in clauses for l in c], np.uint32)
    return offs, lits


def to_dimacs(n_vars, offs, lits, comments=()):
    out = [f"c {c}" for c in comments]
    m = len(offs) - 1
    out.append(f"p cnf {n_vars} {m}")
    for c in range(m):
        ls = lits[int(offs[c]):int(offs[c + 1])]
        toks = [str(int(l >> 1) + 1) if (l & 1) == 0 else str(-(int(l >> 1) + 1)) for l in ls]
        out.append(" ".join(toks + ["0"]))
    return "\n".join(out) + "\n"


def philox_bits(seed, it, vs):
    """Vectorised resample bits: bit v % 32 of Philox4x32-10(key=seed, ctr={v / 32, it_lo, 0,
    it_hi}).x; equals resample_bit() elementwise (checked in tests/test_oracle.py)."""
    M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    mask = np.uint64(0xFFFFFFFF)
    v = np.asarray(vs).astype(np.uint64)
    c0 = v >> np.uint64(5)
    c1 = np.full_like(c0, it & 0xFFFFFFFF)
    c2 = np.zeros_like(c0)
    c3 = np.full_like(c0, it >> 32)
    k0, k1 = np.uint64(seed & 0xFFFFFFFF), np.uint64(seed >> 32)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ k0) & mask, p1 & mask, \
            ((p0 >> np.uint64(32)) ^ c3 ^ k1) & mask, p0 & mask
        k0 = (k0 + np.uint64(0x9E3779B9)) & mask
        k1 = (k1 + np.uint64(0xBB67AE85)) & mask
    return ((c0 >> (v & np.uint64(31))) & np.uint64(1)).astype(np.uint32)


def resample_words(A, seed, it, vs):
    """Set bit v of A (uint32 words) to Philox(seed, it, v) for every v in vs (in place)."""
    vs = np.unique(np.asarray(vs, np.uint32))
    bits = philox_bits(seed, it, vs)
    w = (vs >> 5).astype(np.int64)
    sh = (vs & 31).astype(np.uint32)
    np.bitwise_and.at(A, w, ~(np.uint32(1) << sh))
    np.bitwise_or.at(A, w, bits << sh)
    return A


def clause_vars(offs, lits, C):
    C = np.asarray(C, np.int64)
    if C.size == 0:
        return np.zeros(0, np.uint32)
    idx = np.concatenate([np.arange(offs[c], offs[c + 1], dtype=np.int64) for c in C])
    return (lits[idx] >> 1).astype(np.uint32)


# ------------------------------------------------------------------------- path
def pack_bools(b):
    b = np.asarray(b, np.uint8)
    n = b.size
    nw = (n + 31) // 32
    pad = np.zeros(nw * 32, np.uint8)
    pad[:n] = b
    bits = pad.reshape(nw, 32).astype(np.uint32) << np.arange(32, dtype=np.uint32)
    return np.bitwise_or.reduce(bits, axis=1).astype(np.uint32)


def unpack_words(A, n):
    A = np.asarray(A, np.uint32)
    bits = (A[:, None] >> np.arange(32, dtype=np.uint32)) & 1
    return bits.reshape(-1)[:n].astype(np.uint8)


def eval_mask(offs, lits, A):
    m = len(offs) - 1
    vm = np.zeros(max(1, (m + 63) // 64), np.uint64)
    n = lib().orc_eval(m, _p(offs, _u64p), _p(lits, _u32p), _p(A, _u32p), _p(vm, _u64p))
    return int(n), vm


def mask_to_list(m, vm):
    U = np.zeros(max(1, m), np.uint32)
    n = lib().orc_mask_to_list(m, _p(vm, _u64p), _p(U, _u32p))
    return U[:n].copy()


def lfmis(n_vars, offs, lits, U):
    U = np.ascontiguousarray(U, np.uint32)
    M = np.zeros(max(1, U.size), np.uint32)
    used = np.zeros(max(1, n_vars), np.uint8)
    n = lib().orc_lfmis(n_vars, _p(offs, _u64p), _p(lits, _u32p), _p(U, _u32p), U.size,
                        _p(M, _u32p), _p(used, _u8p))
    return M[:n].copy()


def chunk_bounds(m, T):
    s = np.zeros(T + 1, np.uint64)
    lib().orc_chunk_bounds(m, T, _p(s, _u64p))
    return s


def rr_mis(n_vars, offs, lits, U, T, chunk_starts=None):
    U = np.ascontiguousarray(U, np.uint32)
    M = np.zeros(max(1, U.size), np.uint32)
    used = np.zeros(max(1, n_vars), np.uint8)
    cs = chunk_bounds(len(offs) - 1, T) if chunk_starts is None else np.ascontiguousarray(chunk_starts, np.uint64)
    n = lib().orc_rr_mis(n_vars, _p(offs, _u64p), _p(lits, _u32p), _p(U, _u32p), U.size, T,
                         _p(cs, _u64p), _p(M, _u32p), _p(used, _u8p))
    return M[:n].copy()


def solve(n_vars, offs, lits, seed, max_iters=0, A0=None, trace=False, T=1, chunk_starts=None):
    """Resample loop with Philox.  Returns (stats dict, final A words, per-iter trace).
    T > 1: the MIS is the round-robin greedy over T clause chunks (orc_rr_mis), chunk
    boundaries `chunk_starts` (T+1) or by the example/main.cpp rule."""
    m = len(offs) - 1
    A = init_assignment(seed, n_vars) if A0 is None else np.array(A0, np.uint32)
    st = OrcStats()
    rows = []

    def cb(user, it, nu, nm, dres, Ap):
        if trace:
            rows.append((int(it), int(nu), int(nm), int(dres),
                         np.ctypeslib.as_array(Ap, shape=(A.size,)).copy()))

    cbf = ITER_CB(cb)
    if T > 1:
        cs = chunk_bounds(m, T) if chunk_starts is None else np.ascontiguousarray(chunk_starts, np.uint64)
        lib().orc_solve_rr(n_vars, m, _p(offs, _u64p), _p(lits, _u32p), seed, max_iters, T, _p(cs, _u64p),
                           _p(A, _u32p), ctypes.byref(st), cbf, None)
    else:
        lib().orc_solve(n_vars, m, _p(offs, _u64p), _p(lits, _u32p), seed, max_iters, _p(A, _u32p),
                        ctypes.byref(st), cbf, None)
    stats = {k: int(getattr(st, k)) for k, _ in OrcStats._fields_ if k != "pad"}
    return stats, A, rows


def stream_order(m):
    """Yield order of the reference's ClauseGenerator over m clauses (ClauseGenerator.h:47)."""
    order = np.zeros(max(1, m), np.uint32)
    lib().orc_stream_order(m, _p(order, _u32p))
    return order[:m]


def solve_stream(n_vars, offs, lits, seed, batch, max_iters=0, A0=None, trace=False):
    """Streaming solve (SATInstance.h:70-153, one thread) with Philox.  Returns (stats dict,
    final A words, per-iteration rows (it, |U|, |M|, dres, A after))."""
    m = len(offs) - 1
    A = init_assignment(seed, n_vars) if A0 is None else np.array(A0, np.uint32)
    st = OrcStats()
    rows = []

    def cb(user, it, nu, nm, dres, Ap):
        if trace:
            rows.append((int(it), int(nu), int(nm), int(dres),
                         np.ctypeslib.as_array(Ap, shape=(A.size,)).copy()))

    cbf = ITER_CB(cb)
    lib().orc_solve_stream(n_vars, m, _p(offs, _u64p), _p(lits, _u32p), seed, max_iters, batch,
                           _p(A, _u32p), ctypes.byref(st), cbf, None)
    stats = {k: int(getattr(st, k)) for k, _ in OrcStats._fields_ if k != "pad"}
    return stats, A, rows


def solve_stream_rr(n_vars, offs, lits, seed, batch, T, max_iters=0, A0=None, trace=False, step_cap=1 << 24):
    """Streaming solve with T > 1 threads (SATInstance.h:70-153; orc_solve_stream_rr) with
    Philox.  Returns (rc, stats dict, final A words, per-iteration rows (it, |U|, |M|, dres,
    A after)); rc 0 solved, 1 capped, -1 step cap, -2 empty clause."""
    m = len(offs) - 1
    A = init_assignment(seed, n_vars) if A0 is None else np.array(A0, np.uint32)
    st = OrcStats()
    rows = []

    def cb(user, it, nu, nm, dres, Ap):
        if trace:
            rows.append((int(it), int(nu), int(nm), int(dres),
                         np.ctypeslib.as_array(Ap, shape=(A.size,)).copy()))

    cbf = ITER_CB(cb)
    rc = lib().orc_solve_stream_rr(n_vars, m, _p(offs, _u64p), _p(lits, _u32p), seed, max_iters, batch, T,
                                   step_cap, _p(A, _u32p), ctypes.byref(st), cbf, None)
    stats = {k: int(getattr(st, k)) for k, _ in OrcStats._fields_ if k != "pad"}
    return int(rc), stats, A, rows


def refrng_init(rd_seed, n_vars):
    """The reference's VariablesArray fill (VariablesArray.h:23-34) under the probe's random_device
    stand-in seeded with rd_seed: packed words, and the stand-in's state after the draw."""
    A = np.zeros(max(1, (n_vars + 31) // 32), np.uint32)
    st = ctypes.c_uint64(rd_seed)
    lib().orc_refrng_init(ctypes.byref(st), n_vars, _p(A, _u32p))
    return A, int(st.value)


def solve_refrng(n_vars, offs, lits, rd_seed, max_iters=0, trace=False):
    """orc_solve in the reference-RNG mode (orc_solve_refrng): the reference's own RBG /
    minstd_rand0 / uniform_int_distribution stream, engines seeded from the random_device
    stand-in.  Returns (stats dict, final A words, per-iteration rows (it, |U|, |M|, dres, A))."""
    m = len(offs) - 1
    A = np.zeros(max(1, (n_vars + 31) // 32), np.uint32)
    st = OrcStats()
    rows = []

    def cb(user, it, nu, nm, dres, Ap):
        if trace:
            rows.append((int(it), int(nu), int(nm), int(dres),
                         np.ctypeslib.as_array(Ap, shape=(A.size,)).copy()))

    cbf = ITER_CB(cb)
    lib().orc_solve_refrng(n_vars, m, _p(offs, _u64p), _p(lits, _u32p), rd_seed, max_iters, _p(A, _u32p),
                           ctypes.byref(st), cbf, None)
    stats = {k: int(getattr(st, k)) for k, _ in OrcStats._fields_ if k != "pad"}
    return stats, A, rows


def solve_stream_refrng(n_vars, offs, lits, rd_seed, batch, max_iters=0, trace=False):
    """orc_solve_stream in the reference-RNG mode (one thread).  Returns (stats dict, final A
    words, per-iteration rows (it, |U|, |M|, dres, A after))."""
    m = len(offs) - 1
    A = np.zeros(max(1, (n_vars + 31) // 32), np.uint32)
    st = OrcStats()
    rows = []

    def cb(user, it, nu, nm, dres, Ap):
        if trace:
            rows.append((int(it), int(nu), int(nm), int(dres),
                         np.ctypeslib.as_array(Ap, shape=(A.size,)).copy()))

    cbf = ITER_CB(cb)
    lib().orc_solve_stream_refrng(n_vars, m, _p(offs, _u64p), _p(lits, _u32p), rd_seed, max_iters, batch,
                                  _p(A, _u32p), ctypes.byref(st), cbf, None)
    stats = {k: int(getattr(st, k)) for k, _ in OrcStats._fields_ if k != "pad"}
    return stats, A, rows


# Pure-Python restatement of one streaming iteration with T threads (small cases; the maps the
# golden stream-rr fixtures pin, and the reference for orc_solve_stream_rr in tests/test_oracle.py).
STREAM_P = 9223372036854775783


def stream_gens(m, T):
    """The T ClauseGenerators of SATInstance.h:74-86: {base, n, c, ny, fin}."""
    tn = m // T
    return [dict(base=t * tn, n=(m - t * tn) if t == T - 1 else tn, c=0, ny=0, fin=False) for t in range(T)]


def stream_yield(g, bits, batch):
    """ClauseGenerator::yieldRandomUNSATClauseBatch (ClauseGenerator.h:32-71): the violated
    clauses of the next batch in yield order."""
    if g["fin"]:
        g["ny"], g["fin"] = 0, False
    n = g["n"] - g["ny"] if g["ny"] + batch >= g["n"] else batch
    out = []
    for _ in range(n):
        g["c"] = (g["c"] + STREAM_P) % g["n"]
        cl = g["base"] + g["c"]
        if bits[cl]:
            out.append(cl)
        g["ny"] += 1
    if g["ny"] == g["n"]:
        g["fin"] = True
    return out


def stream_rr_iteration(n_vars, offs, lits, A, batch, gens):
    """The batch loop of one streaming iteration (SATInstance.h:98-125) from generator states
    `gens` (updated in place): returns (per step the T violated lists, the MIS in pick order,
    the MIS size after every step)."""
    m = len(offs) - 1
    _, vm = eval_mask(offs, lits, A)
    bits = np.unpackbits(vm.view(np.uint8), bitorder="little")[:m]
    used = np.zeros(max(1, n_vars), bool)
    T = len(gens)
    steps, M, cum = [], [], []
    while True:
        lists = [stream_yield(g, bits, batch) for g in gens]
        steps.append(lists)
        fin = all(g["fin"] for g in gens)
        head, live, t = [0] * T, list(range(T)), 0   # populate_mis_parallel, SATInstance.h:391-451
        while live:
            t = (t + 1) % len(live)
            s = live[t]
            L = lists[s]
            while head[s] < len(L) and used[lits[int(offs[L[head[s]]]):int(offs[L[head[s]] + 1])] >> 1].any():
                head[s] += 1
            if head[s] == len(L):
                live.pop(t)
                continue
            c = L[head[s]]
            head[s] += 1
            M.append(c)
            used[lits[int(offs[c]):int(offs[c + 1])] >> 1] = True
        cum.append(len(M))
        if fin:
            return steps, np.array(M, np.uint32), cum


def stream_rr_check(offs, lits, A, gens):
    """End-of-iteration check (SATInstance.h:129-147) in lock step: True when solved, else the
    generators are left where the check stopped (min(n_t, f + 1) clauses yielded)."""
    m = len(offs) - 1
    nu, vm = eval_mask(offs, lits, A)
    if nu == 0:
        return True
    bits = np.unpackbits(vm.view(np.uint8), bitorder="little")[:m]
    f = min((int(np.argmax(bits[g["base"]:g["base"] + g["n"]])) for g in gens
             if g["n"] and bits[g["base"]:g["base"] + g["n"]].any()))
    for g in gens:
        g["ny"] = min(g["n"], f + 1)
        g["fin"] = g["ny"] == g["n"]
    return False


def stream_mis(n_vars, offs, lits, A, order):
    """Greedy MIS of the violated clauses in the given order (pick order)."""
    nu, vm = eval_mask(offs, lits, A)
    bits = np.unpackbits(vm.view(np.uint8), bitorder="little")
    used = np.zeros(n_vars, bool)
    M = []
    for c in order:
        c = int(c)
        if not bits[c]:
            continue
        vs = lits[int(offs[c]):int(offs[c + 1])] >> 1
        if used[vs].any():
            continue
        used[vs] = True
        M.append(c)
    return np.array(M, np.uint32)


def dimacs_parse(text: bytes):
    v = ctypes.c_uint32()
    c = ctypes.c_uint64()
    ln = ctypes.c_uint64()
    rc = lib().orc_dimacs_parse(text, len(text), ctypes.byref(v), ctypes.byref(c), None, None,
                                ctypes.byref(ln))
    if rc == -1:
        return rc, None
    offs = np.zeros(c.value + 1, np.uint64)
    lits = np.zeros(max(1, ln.value), np.uint32)
    rc = lib().orc_dimacs_parse(text, len(text), ctypes.byref(v), ctypes.byref(c),
                                _p(offs, _u64p), _p(lits, _u32p), ctypes.byref(ln))
    return rc, (int(v.value), offs, lits[:ln.value].copy())


# ----------------------------------------------------------------- reference run
def read_stream_trace(path):
    """Parse oracle/_ref/ref_probe `stream` output."""
    with open(path, "rb") as f:
        data = f.read()
    assert data[:4] == b"ALRS"
    n_vars, batch = struct.unpack_from("<II", data, 4)
    (m,) = struct.unpack_from("<Q", data, 12)
    p = 20
    iters = []

    def arr(dtype, p):
        (n,) = struct.unpack_from("<Q", data, p)
        p += 8
        a = np.frombuffer(data, dtype, n, p).copy()
        return a, p + a.nbytes

    while True:
        (it,) = struct.unpack_from("<Q", data, p)
        p += 8
        if it == 0xFFFFFFFFFFFFFFFF:
            break
        A = np.frombuffer(data, np.uint8, n_vars, p).copy()
        p += n_vars
        U, p = arr(np.uint32, p)
        M, p = arr(np.uint32, p)
        cum, p = arr(np.uint32, p)
        (dres,) = struct.unpack_from("<Q", data, p)
        p += 8
        iters.append(dict(it=it, A=A, U=U, M=M, cum=cum, dres=dres))
    n_it, n_res, avg = struct.unpack_from("<QQQ", data, p)
    p += 24
    Af = np.frombuffer(data, np.uint8, n_vars, p).copy()
    p += n_vars
    s_it, s_res, s_avg = struct.unpack_from("<QQQ", data, p)
    p += 24
    As = np.frombuffer(data, np.uint8, n_vars, p).copy()
    return dict(n_vars=n_vars, m=m, batch=batch, iters=iters,
                stats=dict(n_iterations=n_it, n_resamples=n_res, avg_mis_size=avg), A_final=Af,
                solve_stats=dict(n_iterations=s_it, n_resamples=s_res, avg_mis_size=s_avg), solve_A=As)


def read_stream_rr_trace(path):
    """Parse oracle/_ref/ref_probe `stream-rr` output (streaming solve, T > 1 threads)."""
    with open(path, "rb") as f:
        data = f.read()
    assert data[:4] == b"ALRQ"
    n_vars, batch, T, _ = struct.unpack_from("<IIII", data, 4)
    (m,) = struct.unpack_from("<Q", data, 20)
    p = 28
    iters = []

    def u64(p):
        return struct.unpack_from("<Q", data, p)[0], p + 8

    def gens(p):
        g = np.frombuffer(data, np.uint64, 3 * T, p).reshape(T, 3).copy()
        return g, p + 24 * T

    while True:
        it, p = u64(p)
        if it == 0xFFFFFFFFFFFFFFFF:
            break
        A = np.frombuffer(data, np.uint8, n_vars, p).copy()
        p += n_vars
        G, p = gens(p)
        ns, p = u64(p)
        steps, cum = [], []
        for _ in range(ns):
            lists = []
            for _ in range(T):
                n, p = u64(p)
                lists.append(np.frombuffer(data, np.uint32, n, p).copy())
                p += 4 * n
            steps.append(lists)
            c, p = u64(p)
            cum.append(c)
        nm, p = u64(p)
        M = np.frombuffer(data, np.uint32, nm, p).copy()
        p += 4 * nm
        dres, p = u64(p)
        solved, p = u64(p)
        iters.append(dict(it=it, A=A, G=G, steps=steps, cum=cum, M=M, dres=dres, solved=solved))
    n_it, n_res, avg = struct.unpack_from("<QQQ", data, p)
    p += 24
    Af = np.frombuffer(data, np.uint8, n_vars, p).copy()
    p += n_vars
    Gf, p = gens(p)
    return dict(n_vars=n_vars, m=m, batch=batch, T=T, iters=iters,
                stats=dict(n_iterations=n_it, n_resamples=n_res, avg_mis_size=avg), A_final=Af, G_final=Gf)


# ----------------------------------------------------------------- reference run
def read_trace(path):
    """Parse oracle/_ref/ref_probe `trace` output."""
    with open(path, "rb") as f:
        data = f.read()
    assert data[:4] == b"ALRT"
    n_vars, T = struct.unpack_from("<II", data, 4)
    (m,) = struct.unpack_from("<Q", data, 12)
    p = 20
    iters = []
    while True:
        (it,) = struct.unpack_from("<Q", data, p)
        p += 8
        if it == 0xFFFFFFFFFFFFFFFF:
            break
        A = np.frombuffer(data, np.uint8, n_vars, p).copy()
        p += n_vars
        (nu,) = struct.unpack_from("<Q", data, p)
        p += 8
        U = np.frombuffer(data, np.uint32, nu, p).copy()
        p += 4 * nu
        (nm,) = struct.unpack_from("<Q", data, p)
        p += 8
        M = np.frombuffer(data, np.uint32, nm, p).copy()
        p += 4 * nm
        (dres,) = struct.unpack_from("<Q", data, p)
        p += 8
        iters.append(dict(it=it, A=A, U=U, M=M, dres=dres))
    n_it, n_res, avg = struct.unpack_from("<QQQ", data, p)
    p += 24
    Af = np.frombuffer(data, np.uint8, n_vars, p).copy()
    return dict(n_vars=n_vars, m=m, T=T, iters=iters,
                stats=dict(n_iterations=n_it, n_resamples=n_res, avg_mis_size=avg), A_final=Af)
