"""Round-robin MIS (n_threads = T > 1) throughput on one MI355X: resample iterations/s of the
full loop for several T, next to the one-set LFMIS loop on the same instance.

Usage: python tools/rr_bench.py [--config M] [--threads 4,16,64,256] [--iters 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {"M": (2_500_000, 10_000_000, 3, 0), "C2": (1_000_000, 4_000_000, 3, 0),
           "C3": (4_000_000, 6_000_000, 8, 0), "C5": (2_500_000, 10_000_000, 3, 1),
           "S": (250_000, 1_000_000, 3, 0),
           "R": (25_000, 100_000, 3, 0)}  # bench.py's cpu_baseline sample of the reference -p path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="M")
    ap.add_argument("--threads", default="1,4,16,64,256")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m, k, kind = CONFIGS[a.config]
    offs, lits = generate_ksat(1, n, m, k, kind)
    for T in [int(x) for x in a.threads.split(",")]:
        with Solver(n, offs, lits, seed=1, n_threads=T) as s:
            s.run(a.warmup)
            s.synchronize()
            before = s.stats()
            t0 = time.perf_counter()
            s.run(a.iters)
            s.synchronize()
            dt = time.perf_counter() - t0
            after = s.stats()
            print(json.dumps({"config": a.config, "T": T, "iters": a.iters, "ms_per_iter": 1e3 * dt / a.iters,
                              "iters_per_s": a.iters / dt,
                              "mis_per_iter": (after["sum_mis_size"] - before["sum_mis_size"]) / a.iters,
                              "violated_last": after["n_violated"],
                              "batches_last_iter": after["lfmis_tail_rounds"]}), flush=True)


if __name__ == "__main__":
    main()
