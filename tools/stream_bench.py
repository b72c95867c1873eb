"""Streaming solve (SATInstance::solve(getEnumeratedClause, n, batch)) on the
GPU: iterations/s and clause-evals/s of the host-planned loop for several thread counts and batch
sizes, with the trajectory checked against the committed oracle digests when given.  One JSON line
per (T, batch).  usage: python tools/stream_bench.py [--config C2] [--threads 1 4 16] [--batches 1000 100000]
[--iters 20] [--warmup 2]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from alllsatisfiabilitysolver_amd import Solver, generate_ksat  # noqa: E402

CONFIGS = {"M": (2_500_000, 10_000_000, 3, 0), "C2": (1_000_000, 4_000_000, 3, 0), "R": (100_000, 400_000, 3, 0),
           "S": (10_000, 40_000, 3, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2", choices=list(CONFIGS))
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 4, 16])
    ap.add_argument("--batches", type=int, nargs="+", default=[1000, 100000])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    n, m, k, kind = CONFIGS[a.config]
    offs, lits = generate_ksat(1, n, m, k, kind)
    for T in a.threads:
        for bs in a.batches:
            try:
                with Solver(n, offs, lits, seed=a.seed, stream_batch=bs, n_threads=T) as s:
                    s.run(a.warmup)
                    st0 = s.stats()
                    t0 = time.perf_counter()
                    st = s.run(a.iters)
                    dt = time.perf_counter() - t0
                    it = st["n_iterations"] - st0["n_iterations"]
                    print(json.dumps({"config": a.config, "n_threads": T, "batch": bs, "iters": it, "s": dt,
                                      "iters_per_s": it / dt if dt > 0 else None,
                                      "clause_evals_per_s": m * it / dt if dt > 0 else None,
                                      "violated_last": st["n_violated"], "avg_mis_size": st["avg_mis_size"],
                                      "solved": st["solved"], "mis_last": int(s.mis().size),
                                      "gathers_last": st["lfmis_tail_rounds"]}), flush=True)
            except Exception as e:  # e.g. generators that never finish together (the reference hangs)
                print(json.dumps({"config": a.config, "n_threads": T, "batch": bs, "error": str(e)}), flush=True)


if __name__ == "__main__":
    main()
