"""Round robin at one config: per iteration, the incremental passes' log (dirty entries, repair
rounds, entries decided, decisions changed; alll_rr_pass_log) and the iteration time.
usage: python tools/rr_log.py [--config M] [--threads 16] [--iters 6] [--warmup 20]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="M")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat
    from rr_bench import CONFIGS

    n, m, k, kind = CONFIGS[a.config]
    offs, lits = generate_ksat(1, n, m, k, kind)
    with Solver(n, offs, lits, seed=1, n_threads=a.threads) as s:
        s.run(a.warmup)
        for _ in range(a.iters):
            t0 = time.perf_counter()
            st = s.run(1)
            dt = time.perf_counter() - t0
            lg = s.rr_pass_log()
            rows = [tuple(int(x) for x in r) for r in lg if r.any()]
            print(f"iter {st['n_iterations']}: {1e3 * dt:.3f} ms, |U| {st['n_violated']}, passes {st['lfmis_tail_rounds']}: "
                  + " ".join(f"[d{r[0]} r{r[1] if r[1] != 0xFFFFFFFF else 'BAIL'} w{r[2]} c{r[3]}]" for r in rows), flush=True)


if __name__ == "__main__":
    main()
