"""k_fp_bbuild's phase stamps (bucket 0, 100 MHz wall clock; FLAG_KERNEL_TIMING) over a few
steady-state round-robin iterations: init, count+scan+place, list rows, per-variable pass.
usage: python tools/rr_bbuild_phases.py [--config M] [--threads 16] [--iters 4] [--warmup 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="M")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat
    from alllsatisfiabilitysolver_amd import _native as N
    from rr_bench import CONFIGS

    n, m, k, kind = CONFIGS[a.config]
    offs, lits = generate_ksat(1, n, m, k, kind)
    with Solver(n, offs, lits, seed=1, n_threads=a.threads, flags=N.FLAG_KERNEL_TIMING) as s:
        s.run(a.warmup)
        for _ in range(a.iters):
            s.run(1)
            t = [int(x) for x in s.rr_round_log()[-1][:5]]
            d = [(t[i + 1] - t[i]) / 100.0 if t[i + 1] >= t[i] > 0 else None for i in range(4)]
            print(f"bbuild bucket 0 (us): init {d[0]}, count/scan/place {d[1]}, list rows {d[2]}, per-variable {d[3]}",
                  flush=True)


if __name__ == "__main__":
    main()
