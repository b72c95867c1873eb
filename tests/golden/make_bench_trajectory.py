"""Trajectory digests of the bench workloads, from the oracle (CPU restatement of the serial
path, SATInstance.h:217-320; round robin of n_threads = T chunks, :414-447).

bench.py compares its own final state against this DATA file after the timed region (it never
imports the oracle): for the iteration count the GPU reached, the violated count of the last
evaluation (SATInstance.h:264-280), the cumulative resample count and MIS-size sum
(:291, :363) and a 64-bit FNV-1a digest of the bit-packed assignment after that iteration
(`alllsatisfiabilitysolver_amd.assignment_digest`).

Instances: the bench generator (gen_seed 1), solve seed 1 (stored per trajectory), Philox
resampling.
  T=1: configs M (256 iterations), C2 and C5 (64 iterations), C3 (8-SAT: until it converges,
       at most 64), C4 (128M clauses, the 8-GPU config: 16 iterations), so that a sharded
       `bench.py --gpus N --config C4|C5` line checks itself.
  T>1: config M with T in {2, 4, 8, 16, 32} (the GPU round robin that bench.py's
       gpu_same_mis_as_cpu_baseline field runs at T = the CPU baseline's thread count), 32
       iterations; C5 with T = 16, 32 iterations.

Usage: python tests/golden/make_bench_trajectory.py [--check N | --add]
  (all entries: ~10 minutes on 8 cores, C4 most of it)
  --check N  recompute only the first N iterations of every entry of the smaller configs and
             compare them with the committed file (tests/test_oracle.py runs this with a small N).
  --add      compute only the entries the committed file lacks and merge them in.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as o  # noqa: E402

from alllsatisfiabilitysolver_amd.solver import assignment_digest  # noqa: E402

OUT = os.path.join(HERE, "bench_trajectory.json")
SEED = 1
# name: (n_vars, n_clauses, k, kind) -- bench.py CONFIGS
CONFIGS = {"M": (2_500_000, 10_000_000, 3, 0), "C2": (1_000_000, 4_000_000, 3, 0),
           "C3": (4_000_000, 6_000_000, 8, 0), "C4": (32_000_000, 128_000_000, 3, 0),
           "C5": (2_500_000, 10_000_000, 3, 1)}
PLAN = ([("M", 1, 256), ("C2", 1, 64), ("C5", 1, 64), ("C3", 1, 64), ("C4", 1, 16)]
        + [("M", T, 32) for T in (2, 4, 8, 16, 32)] + [("C5", 16, 32)])
CHECK_SKIP = {"C4"}  # (--check: 128M clauses take minutes per iteration set-up; --add recomputes it)


def trajectory(cfg, T, iters):
    n, m, k, kind = CONFIGS[cfg]
    offs, lits = o.generate_ksat(1, n, m, k, kind)
    rows = []
    acc = {"res": 0, "mis": 0}
    words = (n + 31) // 32

    def cb(user, it, nu, nm, dres, Ap):
        acc["res"] += int(dres)
        acc["mis"] += int(nm)
        A = np.ctypeslib.as_array(Ap, shape=(words,))
        rows.append([int(it), int(nu), acc["mis"], acc["res"], assignment_digest(A)])

    # the same loop as oracle.solve, with the digest taken inside the callback
    st = o.OrcStats()
    A = o.init_assignment(SEED, n)
    cbf = o.ITER_CB(cb)
    if T > 1:
        cs = o.chunk_bounds(m, T)
        o.lib().orc_solve_rr(n, m, o._p(offs, o._u64p), o._p(lits, o._u32p), SEED, iters, T,
                             o._p(cs, o._u64p), o._p(A, o._u32p), o.ctypes.byref(st), cbf, None)
    else:
        o.lib().orc_solve(n, m, o._p(offs, o._u64p), o._p(lits, o._u32p), SEED, iters,
                          o._p(A, o._u32p), o.ctypes.byref(st), cbf, None)
    if st.solved:  # the final pass found no violated clause: a row for the converged state
        rows.append([int(st.n_iterations), 0, acc["mis"], acc["res"], assignment_digest(A)])
    return rows


def key(cfg, T):
    return f"{cfg}_T{T}"


def main():
    check = None
    if len(sys.argv) > 2 and sys.argv[1] == "--check":
        check = int(sys.argv[2])
    if check is not None:
        ref = json.load(open(OUT))
        for cfg, T, iters in PLAN:
            if cfg in CHECK_SKIP:
                continue
            got = trajectory(cfg, T, min(iters, check))
            want = ref["trajectories"][key(cfg, T)]["rows"][: len(got)]
            if got != want:
                raise SystemExit(f"{key(cfg, T)}: recomputed rows differ from {OUT}")
            print(f"{key(cfg, T)}: first {len(got)} rows match")
        return
    add = len(sys.argv) > 1 and sys.argv[1] == "--add"
    out = {"generator": "bench.py CONFIGS via generate_ksat(gen_seed=1, n, m, k, kind)", "solve_seed": SEED,
           "rng": "Philox4x32-10 (DESIGN.md §1)",
           "digest": "64-bit FNV-1a over the uint32 assignment words after the iteration",
           "row": ["n_iterations", "n_violated (that iteration's evaluation)", "sum_mis_size",
                   "n_resamples", "assignment_digest"],
           "trajectories": {}}
    if add:
        out = json.load(open(OUT))
    for cfg, T, iters in PLAN:
        n, m, k, kind = CONFIGS[cfg]
        if add and key(cfg, T) in out["trajectories"]:
            out["trajectories"][key(cfg, T)].setdefault("solve_seed", SEED)
            continue
        rows = trajectory(cfg, T, iters)
        out["trajectories"][key(cfg, T)] = {"config": cfg, "n_vars": n, "n_clauses": m, "k": k, "kind": kind,
                                            "n_threads": T, "solve_seed": SEED, "rows": rows}
        print(f"{key(cfg, T)}: {len(rows)} iterations, last {rows[-1]}", flush=True)
    with open(OUT, "w") as f:
        json.dump(out, f, separators=(",", ":"))
        f.write("\n")


if __name__ == "__main__":
    main()
