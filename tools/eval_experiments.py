"""Timing-only eval-kernel variants (ALLL_EXPERIMENT, results invalid): back-to-back
alll_bench_eval on config M.  1 = no lookups, 2 = no entry lists, 3 = no LDS fill, 4 = 1+2, 5 = 1+2+3."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from alllsatisfiabilitysolver_amd import Solver, generate_ksat  # noqa: E402

n, m, k = 2_500_000, 10_000_000, 3
offs, lits = generate_ksat(1, n, m, k, 0)
solvers = {}
for x in os.environ.get("EXPS", "0,1,2,3,4,5").split(","):
    os.environ["ALLL_EXPERIMENT"] = x
    solvers[x] = Solver(n, offs, lits, seed=1)
os.environ.pop("ALLL_EXPERIMENT")
res = {x: [] for x in solvers}
for rnd in range(3):
    for x, s in solvers.items():
        res[x].append(s.bench_eval(20)[0])
nbytes = solvers["0"].eval_bytes()
for x, v in res.items():
    med = statistics.median(v)
    print(f"experiment {x}: {med*1e3:8.1f} us  {nbytes/med/1e6:8.1f} GB/s algorithmic")
