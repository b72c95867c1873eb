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
    ap.add_argument("--rounds", action="store_true", help="the repair rounds' clock stamps too")
    a = ap.parse_args()
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat
    from rr_bench import CONFIGS

    n, m, k, kind = CONFIGS[a.config]
    offs, lits = generate_ksat(1, n, m, k, kind)
    from alllsatisfiabilitysolver_amd import _native as N

    # (the round clock stamps are written only with FLAG_KERNEL_TIMING)
    with Solver(n, offs, lits, seed=1, n_threads=a.threads, flags=N.FLAG_KERNEL_TIMING if a.rounds else 0) as s:
        s.run(a.warmup)
        for _ in range(a.iters):
            t0 = time.perf_counter()
            st = s.run(1)
            dt = time.perf_counter() - t0
            lg = s.rr_pass_log()
            rows = [tuple(int(x) for x in r) for r in lg if r.any()]
            print(f"iter {st['n_iterations']}: {1e3 * dt:.3f} ms, |U| {st['n_violated']}, passes {st['lfmis_tail_rounds']}: "
                  + " ".join(f"[d{r[0]} r{r[1] if r[1] != 0xFFFFFFFF else 'BAIL'} w{r[2]} c{r[3]}]" for r in rows), flush=True)
            if a.rounds:
                tl = s.rr_round_log()
                for p, t in enumerate(tl):
                    if not t.any():
                        continue
                    if p == len(tl) - 1:  # k_fp_bbuild's phases (workgroup 0)
                        t0 = int(t[0])
                        print("  bbuild wg0: " + " ".join(f"{(int(t[q]) - t0) % (1 << 32) / 100.0:.1f}" for q in range(1, 5)), flush=True)
                        continue
                    t0 = int(t[0])
                    us = lambda x: (int(x) - t0) % (1 << 32) / 100.0  # 100 MHz ticks -> us
                    rr = [(int(t[8 + 2 * q]), us(t[9 + 2 * q])) for q in range(24) if t[9 + 2 * q]]
                    wb = [us(t[56 + 2 * q]) for q in range(4) if t[56 + 2 * q] and (q == 0 or t[56 + 2 * q] != t[57])]
                    print(f"  pass {p}: wide@{us(t[1]):.1f} rep@{us(t[2]):.1f} lds@{us(t[5]):.1f} "
                          f"rounds_end@{us(t[3]):.1f} cmp@{us(t[57]):.1f} recount@{us(t[59]):.1f} sched@{us(t[6]):.1f} phases@{us(t[7]):.1f} end@{us(t[4]):.1f} | "
                          + " ".join(f"{n}@{x:.1f}" for n, x in rr)
                          + (" | wide pre-barrier " + " ".join(f"{x:.1f}" for x in wb) if wb else ""), flush=True)


if __name__ == "__main__":
    main()
