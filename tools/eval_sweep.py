"""Eval-kernel tuning sweep on the GPU (not a test): times alll_bench_eval for several
configurations and launch settings in one process (interleaved rounds, medians)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from alllsatisfiabilitysolver_amd import Solver, generate_ksat  # noqa: E402
from alllsatisfiabilitysolver_amd import _native as N  # noqa: E402

CFG = {"C2": (1_000_000, 4_000_000, 3, 0), "M": (2_500_000, 10_000_000, 3, 0),
       "C3": (4_000_000, 6_000_000, 8, 0)}
grids = [int(x) for x in os.environ.get("SWEEP_GRIDS", "256,248,240,224,192,128").split(",")]
for name, (n, m, k, kind) in CFG.items():
    offs, lits = generate_ksat(1, n, m, k, kind)
    sr = Solver(n, offs, lits, seed=1)
    sf = Solver(n, offs, lits, seed=1, flags=N.FLAG_NO_RANGED)
    nbytes = sr.eval_bytes()
    res = {g: [] for g in grids}
    res["l2gather"] = []
    for rnd in range(3):
        for g in grids:
            os.environ["ALLL_EVAL_GRID"] = str(g)
            res[g].append(sr.bench_eval(20)[0])
        res["l2gather"].append(sf.bench_eval(20)[0])
    print(name, sr.eval_kernel(), "bytes", nbytes)
    for key, v in res.items():
        med = statistics.median(v)
        print(f"  {str(key):10s} {med*1e3:8.1f} us  {nbytes/med/1e6:8.1f} GB/s")
    sr.close(); sf.close()
