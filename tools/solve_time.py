"""Wall time of whole solves of converging instances (random 3-SAT below the threshold), after
create: the end of a solve runs many iterations with few violated clauses.
usage: python tools/solve_time.py [n_vars] [ratio] [repeats]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from alllsatisfiabilitysolver_amd import Solver, generate_ksat  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ratio = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
m = int(n * ratio)
offs, lits = generate_ksat(7, n, m, 3, 0)
for seed in range(1, reps + 1):
    with Solver(n, offs, lits, seed=seed, device=0, max_iters=20000) as s:
        t0 = time.perf_counter()
        st = s.solve()
        dt = time.perf_counter() - t0
        print(f"n={n} m={m} seed={seed} small_u={os.environ.get('ALLL_SMALL_U', 'default')}: {st['n_iterations']} "
              f"iterations in {dt * 1e3:.1f} ms ({dt / max(1, st['n_iterations']) * 1e6:.1f} us/iteration), "
              f"solved={st['solved']}", flush=True)
