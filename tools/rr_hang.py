"""Bisect helper: the round-robin solver at M after (optionally) the bench's T=1 solver and
torch device use in the same process; one logged iteration at a time.
usage: python tools/rr_hang.py [--t1] [--torch] [--iters 10]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--t1", action="store_true")
    ap.add_argument("--torch", action="store_true")
    ap.add_argument("--torch-after", action="store_true", help="load the library (ROCm runtime) before torch")
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    if a.torch and not a.torch_after:
        import torch
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat
    from alllsatisfiabilitysolver_amd import _native as N

    N.lib()
    if a.torch and a.torch_after:
        import torch
    maps = {l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l}
    log("HIP runtime:", " ".join(sorted(maps)))

    offs, lits = generate_ksat(1, 2_500_000, 10_000_000, 3, 0)
    if a.t1:
        s = Solver(2_500_000, offs, lits, seed=1, device=0, flags=N.FLAG_KERNEL_TIMING)
        s.run(5)
        s.synchronize()
        if a.torch:
            torch.cuda.synchronize(0)
        s.run(50)
        s.synchronize()
        if a.profile:
            s.profile(10)
        s.close()
        log("T=1 solver done")
    with Solver(2_500_000, offs, lits, seed=1, device=0, n_threads=16) as r:
        for i in range(2 + a.iters):
            t0 = time.perf_counter()
            st = r.run(1)
            if a.torch:
                torch.cuda.synchronize(0)
            log(f"iter {st['n_iterations']}: {1e3 * (time.perf_counter() - t0):.2f} ms, violated {st['n_violated']}, "
                f"passes {st['lfmis_tail_rounds']}")
    log("ok")


if __name__ == "__main__":
    main()
