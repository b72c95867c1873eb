"""Diagnostics: per-workgroup phase timing of the instrumented LFMIS kernels (ALLL_DEBUG_PHASES).
usage: python tools/phase_probe.py [--config M] [--iters 6]"""
import argparse
import ctypes
import os
import sys

import numpy as np

os.environ["ALLL_DEBUG_PHASES"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from alllsatisfiabilitysolver_amd import Solver, generate_ksat  # noqa: E402
from alllsatisfiabilitysolver_amd import _native as N  # noqa: E402
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="M")
ap.add_argument("--iters", type=int, default=6)
args = ap.parse_args()
n, m, k, kind, _ = bench.CONFIGS[args.config]
offs, lits = generate_ksat(1, n, m, k, kind)
KER, BLK, FLD = 4, 8192, 8
names = {0: "k_bscatter", 1: "k_bresolve | k_bsort", 2: "k_bjoin | k_decide"}
with Solver(n, offs, lits, seed=1) as s:
    s.run(args.iters)
    buf = np.zeros(KER * BLK * FLD, np.uint64)
    khz = ctypes.c_int()
    N.check(N.lib().alll_debug_phases(s._ctx, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), buf.size,
                                      ctypes.byref(khz)), "debug_phases")
    tick_us = 1e3 / khz.value
    buf = buf.reshape(KER, BLK, FLD).astype(np.int64)
    for kr, name in names.items():
        t = buf[kr]
        used = t[:, 0] > 0
        if not used.any():
            continue
        t = t[used]
        t0 = t[:, 0].min()
        print(f"{name}: {used.sum()} workgroups, start spread {(t[:, 0].max() - t0) * tick_us:.2f} us")
        if kr == 2 and (t[:, 7] < 1 << 20).all() and t[:, 7].max() > 0:  # k_decide: field 7 = passes
            print(f"   passes per workgroup: med {np.median(t[:, 7]):.0f} max {t[:, 7].max()}")
        for p in range(FLD - (1 if kr == 2 else 0)):
            v = t[:, p]
            ok = v > 0
            if not ok.any():
                continue
            rel = (v[ok] - t0) * tick_us
            dur = (v[ok] - t[ok, 0]) * tick_us
            print(f"   phase {p}: since kernel start med {np.median(rel):7.2f} max {rel.max():7.2f} us | "
                  f"since own start med {np.median(dur):7.2f} max {dur.max():7.2f}")
