"""Benchmark of the MI355X Moser-Tardos resample loop (BASELINE.json metric:
"clause-evals/sec + resample iters/sec, random 3-SAT 10M clauses, 1/2/4/8 GPUs").

A step is one resample iteration of SATInstance::parallel_solve (reference
SATInstance.h:260-311) over the whole instance: evaluate all m clauses, compact the violated
ones, exact LFMIS, Philox resample.  Ratio-4 random 3-SAT never converges under this
algorithm, so K fixed iterations are timed.

  value            = m * K / t  (clause-evals/s of the full loop, whole job)
  resample_iters_s = K / t
Inputs are resident in HBM before the timed region.  N>1: one process per GPU, clauses
sharded across ranks, per-iteration RCCL all-gather of the violated bitmask; the instance
size is fixed (strong scaling).  Under torch.distributed.run the ranks come from the
environment; `python bench.py --gpus N` alone starts the N ranks itself.  An RCCL failure is
fatal; the host-staged gloo exchange is only used with --exchange-impl host.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config M|C2|C3|C4|C5|R]
"""
import argparse
import faulthandler
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (n_vars, n_clauses, k, kind, description)
    "M": (2_500_000, 10_000_000, 3, 0, "random 3-SAT ratio 4, 2.5M vars / 10M clauses (metric anchor)"),
    "C2": (1_000_000, 4_000_000, 3, 0, "random 3-SAT ratio 4, 1M vars / 4M clauses"),
    "C3": (4_000_000, 6_000_000, 8, 0, "random 8-SAT m/n 1.5, 4M vars / 6M clauses"),
    "C4": (32_000_000, 128_000_000, 3, 0, "random 3-SAT ratio 4, 32M vars / 128M clauses"),
    "C5": (2_500_000, 10_000_000, 3, 1, "power-law (beta 0.8) 3-SAT, 2.5M vars / 10M clauses"),
    # ragged widths (DIMACS-like mixed clause lengths): the chunk-transposed ragged evaluation
    "R": (1_000_000, 4_000_000, (2, 12), 0, "mixed widths 2-12 (uniform), 1M vars / 4M clauses"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
TRAJECTORY_JSON = os.path.join(ROOT, "tests", "golden", "bench_trajectory.json")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_threads():
    """Host threads for the CPU baseline: the process's CPU affinity (the reference takes
    omp_get_num_procs(), example/main.cpp:77), capped by the cgroup CPU quota and by
    OMP_NUM_THREADS when the environment declares the job's CPU share.  Returns (threads, why)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    why = [f"affinity {n}"]
    quota = None
    try:  # cgroup v2
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(q) // int(per))
    except (OSError, ValueError):
        try:  # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    if quota is not None:
        why.append(f"cgroup quota {quota}")
        n = min(n, quota)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        why.append(f"OMP_NUM_THREADS {omp}")
        n = min(n, int(omp))
    return max(1, n), ", ".join(why)


def _probe(probe, n, m, k, kind, threads, budget, eval_reps, timeout=None):
    cmd = [probe, "bench-gen", str(n), str(m), str(k), str(kind), "1", str(threads), str(budget), str(eval_reps)]
    return json.loads(subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=timeout).stdout)


def cpu_baseline(cfg, budget_s, full_iteration_cap_s=0.0):
    """The reference's own -p OpenMP path (oracle/_ref/ref_probe, compiled from the reference
    sources) on the host cores: full resample iterations on bounded samples of the same
    generator (BASELINE.md "CPU-baseline plan"), plus the eval-phase rate at the full size."""
    n, m, k, kind, _ = CONFIGS[cfg]
    if isinstance(k, tuple):  # the reference probe only generates fixed-width k-SAT
        return {"value": None, "unit": "clause-evals/s", "cores": 0, "kind": "reference",
                "sample": "not measured: the reference generator has no mixed-width mode"}
    threads, why = cpu_threads()
    probe = os.path.join(ROOT, "oracle", "_ref", "ref_probe")
    if os.path.exists(probe):
        # headline sample: 1/100 of the instance (same ratio, same generator), budget_s of loop
        ns, ms = max(k, n // 100), m // 100
        r = _probe(probe, ns, ms, k, kind, threads, budget_s, 0)
        loop_rate = ms * r["iters"] / r["iters_s"] if r["iters"] else 0.0
        points = {f"m={ms}": {"iters": r["iters"], "s": r["iters_s"],
                              "iters_per_s": r["iters"] / r["iters_s"] if r["iters_s"] else 0.0}}
        # the plan's other full-loop points: m = 10k (a few seconds of loop) and m = 1M (one
        # iteration: the reference MIS is quadratic in |U|)
        for frac, budget in ((1000, min(3.0, budget_s)), (10, 1e-3)):
            if m // frac < 1000 or m // frac == ms:
                continue
            q = _probe(probe, max(k, n // frac), m // frac, k, kind, threads, budget, 0)
            points[f"m={m // frac}"] = {"iters": q["iters"], "s": q["iters_s"],
                                        "iters_per_s": q["iters"] / q["iters_s"] if q["iters_s"] else 0.0}
        # eval phase (P1, SATInstance.h:273-280) at the full size, best of 3
        e = _probe(probe, n, m, k, kind, threads, 0, 3)
        # the plan's wall-capped single iteration at the full size: ~1e3 s, so only
        # on request (--cpu-full-iteration SECONDS)
        if full_iteration_cap_s > 0:
            t0 = time.perf_counter()
            try:
                q = _probe(probe, n, m, k, kind, threads, 1e-3, 0, timeout=full_iteration_cap_s)
                full = {"measured": True, "iters": q["iters"], "s": q["iters_s"], "load_s": q["load_s"]}
            except subprocess.TimeoutExpired:
                full = {"measured": False, "why": f"one iteration did not finish within the {full_iteration_cap_s:.0f} s cap",
                        "s_lower_bound": time.perf_counter() - t0}
        else:
            full = {"measured": False,
                    "why": ("one reference iteration at the full size takes ~1e3 s (its populate_mis_parallel is "
                            "quadratic in |U|: 158 s at m=4M on 8 threads, BASELINE.md), beyond the default "
                            "line's few-minute budget; bench.py --cpu-full-iteration SECONDS runs it wall-capped")}
        points[f"m={m}"] = full
        return {
            "value": loop_rate,
            "unit": "clause-evals/s",
            "cores": threads,
            "kind": "reference",
            "sample": (f"reference -p path (T={threads}; {why}) full resample loop, {r['iters']} iterations in "
                       f"{r['iters_s']:.1f}s on a 1/100 sample (n={ns}, m={ms}, same generator); "
                       f"eval phase alone at full size m={m}: {e['eval_clause_evals_per_s']:.3e} "
                       f"clause-evals/s; the reference MIS is quadratic in |U| so the full-size loop "
                       f"is ~1e3 s/iteration (SURVEY.md §6); host {cpu_model()}"),
            "resample_iters_per_s": r["iters"] / r["iters_s"] if r["iters_s"] else 0.0,
            "eval_phase_clause_evals_per_s": e["eval_clause_evals_per_s"],
            "full_loop_points": points,
        }
    # fallback: the oracle's serial restatement (port)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    ns, ms = max(k, n // 100), m // 100
    offs, lits = oracle.generate_ksat(1, ns, ms, k, kind)
    t0 = time.perf_counter()
    it = 0
    while time.perf_counter() - t0 < budget_s:
        oracle.solve(ns, offs, lits, seed=1 + it, max_iters=10)
        it += 10
    dt = time.perf_counter() - t0
    return {"value": ms * it / dt, "unit": "clause-evals/s", "cores": 1, "kind": "port",
            "sample": f"oracle serial restatement, {it} iterations on n={ns}, m={ms}; host {cpu_model()}"}


def trajectory_check(cfg, T, st, words, seed):
    """Bit-exactness of the run, checked outside the timed region against the committed data
    file tests/golden/bench_trajectory.json (oracle trajectories of the same instance and seed,
    written by tests/golden/make_bench_trajectory.py; no oracle code runs here): after the
    iteration the GPU reached, the violated count, the cumulative MIS-size and resample counts
    and a 64-bit FNV-1a digest of the bit-packed assignment."""
    from alllsatisfiabilitysolver_amd import assignment_digest

    it = int(st["n_iterations"])
    out = {"iters": it, "n_threads": T, "match": None,
           "source": "tests/golden/bench_trajectory.json (oracle, SATInstance.h:217-320)"}
    try:
        tf = json.load(open(TRAJECTORY_JSON))
        tj = tf["trajectories"]
    except (OSError, ValueError, KeyError) as e:
        out["reason"] = f"no trajectory file: {e}"
        return out
    tr = tj.get(f"{cfg}_T{T}")
    if tr is None:
        out["reason"] = f"no committed trajectory for config {cfg} with n_threads {T}"
        return out
    tseed = int(tr.get("solve_seed", tf.get("solve_seed", 1)))
    if int(seed) != tseed:
        out["reason"] = f"solve seed {seed}: the committed trajectories were run with seed {tseed}"
        return out
    row = next((r for r in tr["rows"] if r[0] == it), None)
    if row is None:
        out["reason"] = f"iteration {it} lies beyond the committed {len(tr['rows'])} iterations"
        return out
    got = [it, int(st["n_violated"]), int(st["sum_mis_size"]), int(st["n_resamples"]), assignment_digest(words)]
    out["expected"] = dict(zip(("n_violated", "sum_mis_size", "n_resamples", "digest"), row[1:]))
    out["got"] = dict(zip(("n_violated", "sum_mis_size", "n_resamples", "digest"), got[1:]))
    out["match"] = got == list(row)
    return out


def rr_line(args, n, m, k, kind, Solver, generate_ksat, device, warmup=20, steps=10):
    """GPU resample loop with the reference's n_threads = T round-robin MIS, T = the CPU
    baseline's thread count: iterations 21-30 (past the first iterations' larger violated sets,
    as the T = 1 line skips its first five), checked against the committed oracle trajectory."""
    T = cpu_threads()[0]
    if isinstance(k, tuple):
        from alllsatisfiabilitysolver_amd import generate_mixed

        offs, lits = generate_mixed(1, n, m, *k)
    else:
        offs, lits = generate_ksat(1, n, m, k, kind)
    log(f"[rank 0] round-robin line: T={T}, creating the solver")
    with Solver(n, offs, lits, seed=args.seed, device=device, n_threads=T) as r:
        del offs, lits
        r.run(warmup)
        r.synchronize()
        log(f"[rank 0] round-robin line: {warmup} warmup iterations done, timing {steps}")
        it0 = r.stats()["n_iterations"]
        t0 = time.perf_counter()
        r.run(steps)
        r.synchronize()
        dt = time.perf_counter() - t0
        st = r.stats()
        traj = trajectory_check(args.config, T, st, r.assignment_words(), args.seed)
    log(f"[rank 0] round-robin line: {st['n_iterations'] - it0} iterations in {dt:.2f}s")
    done = st["n_iterations"] - it0
    return {"trajectory_check": traj, "value": m * done / dt if done else None, "unit": "clause-evals/s", "n_threads": T,
            "resample_iters_per_s": done / dt if done else None, "ms_per_step": dt * 1e3 / done if done else None,
            "steps": done, "warmup": warmup, "passes_last_iter": st["lfmis_tail_rounds"],
            "mis": "round robin over T clause chunks (SATInstance.h:414-447), as the cpu_baseline's -p T path"}


def stream_line(args, n, m, k, kind, T, bs, check_iters=2, warmup=3, steps=10):
    """The streaming solve with T > 1 generators, SATInstance::solve(getEnumeratedClause, n_clauses,
    batch) (SATInstance.h:70-153), on the bench instance: GPU iterations/s over
    `steps` iterations, and as its cpu_baseline the oracle's serial restatement
    (orc_solve_stream_rr) timed over the first `check_iters` iterations, whose statistics and
    assignment the GPU's must equal bit for bit (checked outside the timed region)."""
    from alllsatisfiabilitysolver_amd import Solver, assignment_digest, generate_ksat

    if isinstance(k, tuple):
        return {"value": None, "error": "the stream line runs on the fixed-width configurations"}
    offs, lits = generate_ksat(1, n, m, k, kind)
    log(f"[rank 0] stream line: T={T}, batch={bs}")
    with Solver(n, offs, lits, seed=args.seed, stream_batch=bs, n_threads=T) as s:
        s.run(check_iters)
        st_k = s.stats()
        words = s.assignment_words().copy()
        s.run(warmup)
        s.synchronize()
        it0 = s.stats()["n_iterations"]
        t0 = time.perf_counter()
        s.run(steps)
        s.synchronize()
        dt = time.perf_counter() - t0
        done = s.stats()["n_iterations"] - it0
    out = {"n_threads": T, "batch": bs, "steps": done, "warmup": warmup + check_iters,
           "resample_iters_per_s": done / dt if done else None,
           "value": m * done / dt if done else None, "unit": "clause-evals/s",
           "ms_per_step": dt * 1e3 / done if done else None}
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    t0 = time.perf_counter()
    rc, st_o, A_o, _ = oracle.solve_stream_rr(n, offs, lits, args.seed, bs, T, max_iters=check_iters)
    dtc = time.perf_counter() - t0
    keys = ("n_iterations", "n_resamples", "sum_mis_size", "avg_mis_size", "solved")
    match = rc in (0, 1) and all(int(st_k[q]) == int(st_o[q]) for q in keys) and \
        assignment_digest(words) == assignment_digest(A_o)
    out["check"] = {"iters": check_iters, "match": bool(match),
                    "gpu": {q: int(st_k[q]) for q in keys}, "oracle": {q: int(st_o[q]) for q in keys}}
    out["cpu_baseline"] = {"value": m * check_iters / dtc, "unit": "clause-evals/s", "cores": 1, "kind": "port",
                           "resample_iters_per_s": check_iters / dtc,
                           "sample": f"oracle serial restatement (orc_solve_stream_rr), the first {check_iters} "
                                     f"iterations of the same instance and seed; host {cpu_model()}"}
    return out


def shard_line(args, n, offs, lits, kw, rank, world, exchange_impl, comm_id, dist, barrier, torch, warmup=3, steps=20):
    """N>1 with the replicated plan: the clause-sharded loop (alll_shard_plan, the violated-bitmask
    exchange every iteration) on the same instance, `steps` iterations timed as the main line
    (barrier + max over ranks), checked against the committed oracle trajectory."""
    from alllsatisfiabilitysolver_amd import Solver

    kw = dict(kw, rank=rank, world=world)
    if exchange_impl == "host":
        from alllsatisfiabilitysolver_amd import gloo_exchange

        s = Solver(n, offs, lits, exchange=gloo_exchange(), **kw)
    else:
        s = Solver(n, offs, lits, comm_id=comm_id, **kw)
    try:
        s.run(warmup)
        s.synchronize()
        barrier()
        it0 = s.stats()["n_iterations"]
        t0 = time.perf_counter()
        s.run(steps, sync=False)
        s.synchronize()
        barrier()
        dt = time.perf_counter() - t0
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        st = s.stats()
        done = st["n_iterations"] - it0
        traj = trajectory_check(args.config, 1, st, s.assignment_words(), args.seed) if rank == 0 else None
        m = len(offs) - 1
        return {"value": m * done / dt if done else None, "unit": "clause-evals/s", "exchange": exchange_impl,
                "n_comm": s.comm_size(), "steps": done, "warmup": warmup,
                "resample_iters_per_s": done / dt if done else None,
                "ms_per_step": dt * 1e3 / done if done else None, "trajectory_check": traj}
    finally:
        s.close()


def rr_line_child(args, timeout_s=240):
    """The round-robin line in a child process (this script with --rr-child): its own HIP
    context and a time limit, so that it can neither disturb nor stall the main line."""
    cmd = [sys.executable, os.path.abspath(__file__), "--rr-child", "--config", args.config, "--seed", str(args.seed)]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"value": None, "error": f"round-robin line did not finish within {timeout_s} s"}
    sys.stderr.write(p.stderr)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"value": None, "error": f"round-robin child exited with {p.returncode}"}
    return json.loads(lines[-1])


def launch_ranks(args):
    """--gpus N > 1 without a launcher: start N rank processes (one per GPU) through
    torch.distributed.run and exit with its status.  This process never touches the GPU."""
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"launching {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="M", choices=list(CONFIGS))
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--exchange", default="allgather", choices=["allgather", "allreduce"])
    ap.add_argument("--exchange-impl", default="rccl", choices=["rccl", "host"],
                    help="N>1: RCCL collectives (default; a failure is fatal) or the host-staged gloo "
                         "exchange (rehearsal on one GPU, ALLL_BENCH_SAME_DEVICE=1)")
    ap.add_argument("--rccl-self", action="store_true",
                    help="N=1 only: run the multi-GPU exchange path over a one-rank RCCL communicator "
                         "(all-gather / all-reduce inside the captured graphs; rehearsal on one GPU)")
    ap.add_argument("--no-ranged", action="store_true", help="use the L2-gather eval kernel")
    ap.add_argument("--atomic-claims", action="store_true", help="LFMIS round 0 by global atomics")
    ap.add_argument("--grid-rounds", type=int, default=0, help="full-grid LFMIS rounds (0 = default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-rr-line", action="store_true",
                    help="skip the GPU run with the CPU baseline's round-robin MIS (n_threads = T)")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--cpu-full-iteration", type=float, default=0.0,
                    help="also time one reference iteration at the full size, capped at this many seconds")
    ap.add_argument("--event-iters", type=int, default=10,
                    help="iterations replayed eagerly with HIP events around each phase (cross-check)")
    ap.add_argument("--eval-b2b", type=int, default=20,
                    help="back-to-back eval-only launches timed with HIP events for the roofline (at least 20)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_eval_traffic.json"))
    ap.add_argument("--rr-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--plan", default="auto", choices=["auto", "shard", "replicate"],
                    help="N>1: clause-sharded loop with the per-iteration exchange, or every rank the whole "
                         "one-GPU loop; auto = alll_plan_multi_gpu's cost model (DESIGN.md §5.2)")
    ap.add_argument("--no-shard-line", action="store_true",
                    help="N>1 with the replicated plan: skip the secondary run of the sharded (exchange) path")
    ap.add_argument("--shard-line-timeout", type=float, default=180.0,
                    help="seconds the secondary sharded run may take before the line is written without it")
    ap.add_argument("--stream-line", default="4:100000",
                    help="T:BATCH -- also run the streaming solve with T generators of BATCH clauses "
                         "(GPU rate, and the oracle's first iterations as its CPU baseline and check); "
                         "'none' skips it")
    args = ap.parse_args()

    if args.rr_child:  # (rr_line_child): one JSON line on stdout, no torch in this process
        from alllsatisfiabilitysolver_amd import Solver, generate_ksat

        n, m, k, kind, _ = CONFIGS[args.config]
        print(json.dumps(rr_line(args, n, m, k, kind, Solver, generate_ksat, 0)), flush=True)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if os.environ.get("ALLL_BENCH_SAME_DEVICE"):  # rehearsal of the N>1 path on a 1-GPU box
        local_rank = 0
    # The result is ONE JSON line on stdout: keep a private handle on it and send everything
    # else written to file descriptor 1 (RCCL's version banner at communicator init, library
    # prints) to stderr.
    # a stalled native call shows where it stalled (stderr), instead of silence
    faulthandler.dump_traceback_later(120, repeat=True, file=sys.stderr)
    result_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    # The library (and with it the ROCm runtime it was built against) is loaded before torch:
    # torch's wheel bundles its own HIP runtime, which the library would otherwise bind to.
    # torch is used for the rendezvous and the host-side collectives only (gloo); device
    # synchronisation goes through the library (the solver's stream holds all of its work).
    from alllsatisfiabilitysolver_amd import Solver, comm_unique_id, generate_ksat
    from alllsatisfiabilitysolver_amd import _native as N

    N.lib()
    import torch

    dist = None
    comm_id = None
    exchange_impl = "none"
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)  # host-side control only
        exchange_impl = args.exchange_impl
        if exchange_impl == "rccl":
            obj = [comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            comm_id = obj[0]
    elif args.rccl_self:
        exchange_impl = "rccl-self"
        comm_id = comm_unique_id()

    n, m, k, kind, desc = CONFIGS[args.config]
    t0 = time.perf_counter()
    if isinstance(k, tuple):
        from alllsatisfiabilitysolver_amd import generate_mixed

        offs, lits = generate_mixed(1, n, m, *k)
    else:
        offs, lits = generate_ksat(1, n, m, k, kind)
    t_gen = time.perf_counter() - t0
    from alllsatisfiabilitysolver_amd import plan_multi_gpu

    mplan = plan_multi_gpu(m, int(len(lits)), n, world)
    plan = mplan["plan"] if args.plan == "auto" else args.plan
    if world == 1:
        plan = "single"
    log(f"[rank {rank}] multi-GPU plan: {plan} (model: evaluation {mplan['eval_us_1gpu']:.1f} us on one GPU, "
        f"sharding saves {mplan['eval_saved_us']:.1f}, exchange costs {mplan['exchange_us']:.1f})")
    flags = N.FLAG_KERNEL_TIMING  # kernels stamp device wall-clock times of every iteration
    if args.exchange == "allreduce":
        flags |= N.FLAG_EXCHANGE_ALLREDUCE
    if args.no_ranged:
        flags |= N.FLAG_NO_RANGED
    if args.atomic_claims:
        flags |= N.FLAG_ATOMIC_CLAIMS
    t0 = time.perf_counter()
    kw = dict(seed=args.seed, device=local_rank, rank=rank, world=world, flags=flags, grid_rounds=args.grid_rounds)
    if plan == "replicate":
        # every rank runs the whole one-GPU loop on its own device: no exchange, the same
        # trajectory on every rank (the sharded path runs afterwards as a secondary line)
        kw.update(rank=0, world=1)
        s = Solver(n, offs, lits, **kw)
    elif exchange_impl == "host":
        from alllsatisfiabilitysolver_amd import gloo_exchange

        s = Solver(n, offs, lits, exchange=gloo_exchange(), **kw)
    else:
        s = Solver(n, offs, lits, comm_id=comm_id, **kw)  # RCCL failure raises: fatal
    if not (plan == "replicate" and not args.no_shard_line):
        del offs, lits
    t_create = time.perf_counter() - t0
    log(f"[rank {rank}] generated {m} clauses in {t_gen:.2f}s, uploaded in {t_create:.2f}s, "
        f"layout k={s.layout()}, eval kernel {s.eval_kernel()}, exchange {exchange_impl}")

    def barrier():
        if dist is not None:
            dist.barrier()

    # warmup (untimed); an RCCL error here is fatal too
    s.run(args.warmup, sync=False)
    s.synchronize()
    n_comm = s.comm_size()
    ranks_seen = 1
    if dist is not None:
        t = torch.tensor([1], dtype=torch.int64)
        dist.all_reduce(t)
        ranks_seen = int(t.item())
        if ranks_seen != world or n_comm != (1 if plan == "replicate" else world):
            raise SystemExit(f"rank {rank}: {ranks_seen} ranks answered, communicator holds {n_comm}, "
                             f"expected {world}")

    barrier()
    s.synchronize()
    it0 = s.stats()["n_iterations"]
    t0 = time.perf_counter()
    s.run(args.steps, sync=False)
    s.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    st = s.stats()
    log(f"[rank {rank}] timed {st['n_iterations'] - it0} iterations in {dt:.3f}s")
    traj = trajectory_check(args.config, 1, st, s.assignment_words(), args.seed) if rank == 0 else None
    # the timed loop must have replayed the captured graphs; an eager fallback (a capture or an
    # RCCL call under capture that failed) would time a different launch pattern unannounced
    graphs, graph_note = s.uses_graphs()
    graphs_expected = exchange_impl != "host"
    create_max = t_create
    if dist is not None:
        tc = torch.tensor([t_create], dtype=torch.float64)
        dist.all_reduce(tc, op=dist.ReduceOp.MAX)
        create_max = float(tc.item())
    # iterations actually run: an instance that converges stops early (every kernel is gated
    # off after the final zero-violation pass), so m * K / t would overstate the rate
    steps_done = st["n_iterations"] - it0
    converged = bool(st["solved"])

    # in-loop phase times of exactly the timed iterations, from the kernels' own device
    # wall-clock stamps (the graph replays as timed; eval = first workgroup start to last
    # workgroup end); the eval kernel's average duration prices the roofline
    pt = s.loop_times(it0, max(1, steps_done))
    eval_bytes = s.eval_bytes()
    # The roofline's kernel is the evaluation alone (k_eval_hybrid<K>): HIP events on the
    # solver's stream around back-to-back eval-only launches after the timed region (on the
    # loop's last assignment).  In the loop the one-GPU bucketed round 0 runs the evaluation
    # fused with the round-0 scatter (k_eval_scatter<K>), whose duration is not the
    # evaluation's; its evaluation part (the kernels' wall-clock stamps) is reported beside it.
    # (a converging instance's clause-eval rate is the same eval-only rate.)
    ev_ms = s.bench_eval(max(args.eval_b2b, 20))[0]
    eval_ms = ev_ms
    achieved = eval_bytes / (eval_ms * 1e-3) / 1e9 if eval_ms > 0 else 0.0
    achieved_loop = eval_bytes / (pt["eval_ms"] * 1e-3) / 1e9 if pt["eval_ms"] > 0 else 0.0
    # cross-check with HIP events on the solver's stream: the same iteration replayed eagerly
    pe = s.profile(args.event_iters) if args.event_iters > 0 and not converged else None
    traffic = None
    try:
        tj = json.load(open(args.traffic_json))
        if tj.get("config") == args.config and tj.get("n_gpus", 1) == world:
            traffic = tj.get("hbm_bytes_per_launch")
            # (the roofline prices the evaluation alone: its own kernel's counters when recorded)
            for k, v in (tj.get("per_kernel") or {}).items():
                if s.eval_kernel() in k.split("(")[0] and "hbm_bytes_per_launch" in v:
                    traffic = v["hbm_bytes_per_launch"]
    except (OSError, ValueError):
        pass

    out = None
    if rank == 0:
        if steps_done == args.steps and not converged:
            value, iters_s, ms_step, vkind = m * steps_done / dt, steps_done / dt, dt * 1e3 / steps_done, "loop"
        else:
            # converged before or during the timed region: no loop rate exists; report the
            # evaluation pass rate and mark it
            value, iters_s, ms_step, vkind = m / (eval_ms * 1e-3), None, eval_ms, "eval-only (instance converged)"
        out = {
            "metric": "clause-evals/sec + resample iters/sec, random 3-SAT 10M clauses, 1/2/4/8 GPUs",
            "value": value,
            "unit": "clause-evals/s",
            "n_gpus": ranks_seen,
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "steps_done": steps_done,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded counter-based random k-SAT generator, gen_seed=1)",
            "config": {"workload": f"{args.config}: {desc}", "n_vars": n, "n_clauses": m, "k": k,
                       "solve_seed": args.seed,
                       "exchange": f"{args.exchange}/{exchange_impl}" if world > 1 or comm_id else "none",
                       "parallelism": (f"replicated x{world}" if plan == "replicate" else
                                       f"clause-shard x{world}" if world > 1 else "one GPU")},
            "multi_gpu_plan": dict(mplan, chosen=plan, requested=args.plan) if world > 1 else None,
            "value_kind": vkind,
            "trajectory_check": traj,
            "graphs": graphs,
            "graph_note": graph_note or None,
            "create_s_max_over_ranks": create_max,
            "resample_iters_per_s": iters_s,
            "violated_last": st["n_violated"],
            "avg_mis_size": st["avg_mis_size"],
            "lfmis_rounds_max": st["lfmis_rounds_max"],
            "phase_ms": {k2: pt[k2] for k2 in ("eval_ms", "exchange_ms", "mis_ms", "resample_ms", "total_ms")},
            "phase_iters": pt["iterations"],
            "phase_note": ("device wall-clock stamps per timed iteration: eval = evaluation kernel; "
                           "exchange = evaluation end to the reduce's start (N>1: bitmask all-gather "
                           "+ k_collect; one GPU: the rest of the LFMIS round-0 bucket scatter, fused "
                           "into the evaluation kernel k_eval_scatter); "
                           "mis = reduce start to LFMIS tail end; resample = tail end to the next "
                           "evaluation start (k_resample_vars + launch gaps)"),
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": s.eval_kernel(),
                "algorithmic_bytes_per_launch": eval_bytes,
                "eval_ms": eval_ms,
                # (named for what it is -- the eval-only kernel's launches over the loop's
                # final assignment; the committed rocprof summaries, profiles/r*_<cfg>/, average the
                # same eval-only launches of bench_eval, and the in-loop figure is eval_ms_in_loop)
                "eval_ms_b2b_fixed_assignment": eval_ms,
                "traffic_source": (f"{os.path.relpath(args.traffic_json, ROOT)}: PMC FETCH_SIZE x2 + WRITE_SIZE of "
                                   f"{s.eval_kernel()} per launch (committed, not measured in this run)"
                                   if traffic is not None else None),
                "timing": (f"HIP events on the solver's stream around {max(args.eval_b2b, 20)} back-to-back "
                           f"launches of the evaluation kernel alone ({s.eval_kernel()}, alll_bench_eval), "
                           f"after the timed region"),
                "eval_ms_in_loop": pt["eval_ms"],
                "frac_in_loop": achieved_loop / HBM_PEAK_GBS,
                "in_loop_note": ("the evaluation part of the loop's evaluation kernel, from its workgroups' "
                                 "device wall-clock stamps (s_memrealtime) over the timed iterations; one "
                                 "GPU's bucketed round 0 fuses the round-0 scatter into it (k_eval_scatter)"),
                "eval_ms_hip_events_eager_iterations": pe["eval_ms"] if pe else None,
            },
        }
    s.close()
    run_done = __import__("threading").Event()  # (set once the line is out and the ranks are torn down)
    emitted = []

    def emit(o):
        if not emitted:
            emitted.append(True)
            result_out.write(json.dumps(o) + "\n")
            result_out.flush()

    if world > 1 and plan == "replicate" and not args.no_shard_line:
        # the clause-sharded path (exchange every iteration) on the same instance, so that a
        # multi-GPU run still exercises and checks it: its own rate and trajectory check
        # (a watchdog keeps the headline: if the sharded run and the teardown after it have not
        # finished in time -- a collective that never completes -- rank 0 writes the line as it
        # stands and every rank exits; an error inside the sharded run is reported, not fatal)
        import threading

        def _watchdog():
            if not run_done.wait(args.shard_line_timeout):
                if rank == 0:
                    out.setdefault("shard_line", {"value": None,
                                                  "error": f"did not finish within {args.shard_line_timeout:.0f} s"})
                    emit(out)
                log(f"[rank {rank}] sharded line timed out; exiting")
                os._exit(0)

        threading.Thread(target=_watchdog, daemon=True).start()
        try:
            sh = shard_line(args, n, offs, lits, kw, rank, world, exchange_impl, comm_id, dist, barrier, torch)
        except Exception as e:
            sh = {"value": None, "error": f"{type(e).__name__}: {e}"}
        del offs, lits
        if rank == 0:
            out["shard_line"] = sh
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.no_rr_line:
        # the CPU baseline runs the reference's -p T path, whose MIS is the T-set round robin
        # (SATInstance.h:414-447), not the one-set LFMIS timed above: the same workload with that
        # same MIS on the GPU, for a like-for-like ratio
        try:
            out["gpu_same_mis_as_cpu_baseline"] = rr_line_child(args)
        except Exception as e:  # reported, never fatal for the GPU number
            out["gpu_same_mis_as_cpu_baseline"] = {"value": None, "error": str(e)}
    if rank == 0 and world == 1 and args.stream_line and args.stream_line != "none" and not args.rccl_self:
        try:
            st_T, st_b = (int(x) for x in args.stream_line.split(":"))
            n0, m0, k0, kind0, _ = CONFIGS[args.config]
            out["stream_line"] = stream_line(args, n0, m0, k0, kind0, st_T, st_b)
        except Exception as e:  # reported, never fatal for the GPU number
            out["stream_line"] = {"value": None, "error": str(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("[rank 0] cpu baseline: the reference's -p path on bounded samples")
        try:
            out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_budget, args.cpu_full_iteration)
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"value": None, "error": str(e)}
    if rank == 0:
        emit(out)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    run_done.set()
    rr = (out or {}).get("gpu_same_mis_as_cpu_baseline") or {}
    bad = [name for name, t in (("T=1 loop", traj), ("round robin", rr.get("trajectory_check")),
                                ("streaming solve", ((out or {}).get("stream_line") or {}).get("check")),
                                ("sharded path", ((out or {}).get("shard_line") or {}).get("trajectory_check")))
           if t and t.get("match") is False]
    if rank == 0 and bad:
        log(f"[rank 0] FAIL: the {' and '.join(bad)} left a state that differs from the committed oracle trajectory")
        sys.exit(4)
    if rank == 0 and rr.get("error"):
        # a round-robin line that stalled, crashed or timed out is a failure of the run, not a
        # missing number (the line above still carries the T = 1 result and the error)
        log(f"[rank 0] FAIL: round-robin line: {rr['error']}")
        sys.exit(5)
    if graphs_expected and not graphs:
        log(f"[rank {rank}] FAIL: the loop fell back to eager launches ({graph_note}); the line above "
            f"does not time the graph-replayed loop")
        sys.exit(3)


if __name__ == "__main__":
    main()
