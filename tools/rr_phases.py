"""Phase profile of the round-robin MIS kernel (diagnostics, ALLL_DEBUG_PHASES): time of
thread 0 in the prologue (set ranges), scan, validation and commit of the batches, and the
scan steps / in-step greedy rounds of all groups, for the last iteration.

Usage: ALLL_DEBUG_PHASES=1 python tools/rr_phases.py [--config M] [--threads 4,16,256]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CONFIGS = {"M": (2_500_000, 10_000_000, 3, 0), "S": (250_000, 1_000_000, 3, 0), "R": (25_000, 100_000, 3, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="M")
    ap.add_argument("--threads", default="4,16,64,256")
    ap.add_argument("--iters", type=int, default=3)
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
                d = out[3 * 8192 * 8: 3 * 8192 * 8 + 16].astype(np.float64)
                us = d[:4] / (khz.value / 1e3)
                print(json.dumps({"T": T, "iter": it + 1, "prologue_us": us[0], "scan_us": us[1], "validate_us": us[2],
                                  "commit_us": us[3], "batches": int(d[4]), "scan_steps": int(d[5]),
                                  "greedy_rounds": int(d[6]), "picks": int(d[7]),
                                  "us_per_batch": float(us[1:].sum() / max(1, d[4])),
                                  "group0": {"load_us": d[8] / (khz.value / 1e3), "steps_us": d[9] / (khz.value / 1e3),
                                             "rounds": int(d[10]), "scans": int(d[11])},
                                  "group_scan_us_sum": d[12] / (khz.value / 1e3), "group_scan_us_max_sum": d[13] / (khz.value / 1e3)}), flush=True)


if __name__ == "__main__":
    main()
