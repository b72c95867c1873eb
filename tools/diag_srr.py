"""Diagnostic (not a test): streaming T > 1 on the GPU against the oracle's per-iteration MIS, with the
difference explained (dependent pair inside the GPU's MIS, or a clause missing)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
from alllsatisfiabilitysolver_amd import Solver, generate_ksat
import oracle as o

def main():
    n, m, bs, T = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    kind = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 3
    offs, lits = generate_ksat(2, n, m, 3, kind)
    seed = 41
    rc, st_o, A_o, rows = o.solve_stream_rr(n, offs, lits, seed, bs, T, max_iters=60, trace=True)
    gens = o.stream_gens(m, T)
    A = o.init_assignment(seed, n)
    Ms = []
    for it, nu, nm, dres, A_after in rows:
        steps, M, cum = o.stream_rr_iteration(n, offs, lits, A, bs, gens)
        Ms.append(np.sort(M))
        A = A_after
        if o.stream_rr_check(offs, lits, A, gens):
            break
    for rep in range(reps):
        bad = 0
        with Solver(n, offs, lits, seed=seed, stream_batch=bs, n_threads=T) as s:
            for i, (it, nu, nm, dres, A_after) in enumerate(rows[:len(Ms)]):
                s.run(1)
                g = s.mis()
                if not np.array_equal(g, Ms[i]):
                    extra = np.setdiff1d(g, Ms[i]); miss = np.setdiff1d(Ms[i], g)
                    vs = {}
                    dep = []
                    for c in g:
                        for v in lits[int(offs[c]):int(offs[c + 1])] >> 1:
                            if v in vs: dep.append((int(vs[v]), int(c), int(v)))
                            vs[v] = c
                    print(f"rep {rep} iter {it}: gpu {g.size} oracle {Ms[i].size} extra {extra[:8]} missing {miss[:8]} dependent pairs in gpu MIS {dep[:5]}", flush=True)
                    bad += 1
                    s.set_assignment_words(A_after)
        print(f"rep {rep}: {bad} iterations differ of {len(Ms)}", flush=True)

main()
