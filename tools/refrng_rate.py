"""Iterations/s of the resample loop with the Philox stream and with the reference's own stream
(ALLL_FLAG_REFERENCE_RNG) on one instance.
usage: python tools/refrng_rate.py [--config M] [--iters 20] [--warmup 5]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from alllsatisfiabilitysolver_amd import Solver, generate_ksat  # noqa: E402
from alllsatisfiabilitysolver_amd import _native as N  # noqa: E402

CONFIGS = {"M": (2_500_000, 10_000_000), "C2": (1_000_000, 4_000_000)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="M", choices=list(CONFIGS))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    n, m = CONFIGS[a.config]
    offs, lits = generate_ksat(1, n, m, 3, 0)
    for name, fl in (("philox", 0), ("reference_rng", N.FLAG_REFERENCE_RNG)):
        with Solver(n, offs, lits, seed=3, flags=fl) as s:
            s.run(a.warmup)
            s.synchronize()
            t0 = time.perf_counter()
            s.run(a.iters)
            s.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"config": a.config, "rng": name, "iters_per_s": a.iters / dt}), flush=True)


if __name__ == "__main__":
    main()
