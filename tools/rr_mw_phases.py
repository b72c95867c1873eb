"""Phase profile of the multi-workgroup round-robin kernel k_rr_mw (diagnostics,
ALLL_DEBUG_PHASES): workgroup 0's time per batch in its scan, its global hash inserts, the
first grid barrier (waiting for the slowest group), its commit and the second barrier.

Usage: ALLL_DEBUG_PHASES=1 python tools/rr_mw_phases.py [--config M] [--threads 4,16]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CONFIGS = {"M": (2_500_000, 10_000_000, 3, 0), "R": (25_000, 100_000, 3, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="M")
    ap.add_argument("--threads", default="4,16,64")
    ap.add_argument("--iters", type=int, default=2)
    a = ap.parse_args()
    os.environ.setdefault("ALLL_DEBUG_PHASES", "1")
    import numpy as np
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat
    from alllsatisfiabilitysolver_amd import _native as N

    n, m, k, kind = CONFIGS[a.config]
    offs, lits = generate_ksat(1, n, m, k, kind)
    for T in [int(x) for x in a.threads.split(",")]:
        with Solver(n, offs, lits, seed=1, n_threads=T) as s:
            for it in range(a.iters):
                s.run(1)
                out = np.zeros(4 * 8192 * 8, np.uint64)
                khz = ctypes.c_int()
                N.check(N.lib().alll_debug_phases(s._ctx, out.ctypes.data_as(N._u64p), out.size, ctypes.byref(khz)))
                d = out[3 * 8192 * 8: 3 * 8192 * 8 + 24].astype(np.float64)
                nb = max(1.0, d[4])
                us = lambda x: x / (khz.value / 1e3) / nb  # noqa: E731
                print(json.dumps({"T": T, "iter": it + 1, "batches": int(d[4]), "picks": int(d[7]),
                                  "per_batch_us": {"scan": us(d[8]), "insert": us(d[9]), "barrier1": us(d[10]),
                                                   "commit": us(d[11]), "barrier2": us(d[12])},
                                  "scan_detail_us": {"loads": us(d[13]), "own": us(d[14]), "greedy": us(d[15]),
                                                     "picks": us(d[16])},
                                  "steps_per_batch": d[17] / nb, "stamp_pair_ticks": int(d[18])}), flush=True)


if __name__ == "__main__":
    main()
