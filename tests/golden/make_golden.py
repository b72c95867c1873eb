"""Generate the golden vectors in tests/golden/ from the REFERENCE's own code.

Runs oracle/_ref/ref_probe (compiled by oracle/Makefile from the reference sources under
/root/reference, never copied) in this container and stores, per instance:
  * the instance (CSR) and the reference's per-iteration records
    (A_i bit-packed, U_i violated clauses, M_i MIS in pick order, delta n_resamples),
  * final Statistics, and for T=1 the output of the real SATInstance::solve with the same
    interposed random_device (pins the probe's per-iteration loop to parallel_solve),
  * DIMACS loader edge cases with the reference cnf_header_read/cnf_data_read output.

Usage:  python tests/golden/make_golden.py [--stream-only] [--rewrite-rr]
        (needs /root/reference; not run on the GPU box)

T > 1 fixtures are NOT reproducible: the reference resamples inside an OpenMP
schedule(dynamic) loop (SATInstance.h:352), so which thread (and which interposed
random_device stream) resamples a clause varies from run to run, and A_1, A_2, ... differ
between runs.  Every such trajectory is equally valid for the tests (they set A_i and check
the maps A_i -> U_i -> M_i), but a rerun would silently replace the committed one, so the
existing T > 1 fixtures are kept unless --rewrite-rr is given.  T = 1 is deterministic.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as o  # noqa: E402

RD_SEED = 7


def edge_instance():
    """Hand-made clauses exercising the special cases of Appendix A."""
    L = lambda x: 2 * (abs(x) - 1) + (1 if x < 0 else 0)  # main.cpp:168 encoding
    cl = [
        [1, 1, 2],            # duplicate variable in a clause (counts twice in n_resamples)
        [3, -3],              # tautology: never violated
        [4],                  # unit clauses
        [-5],
        [6, 7, 8, 9, 10, 11, 12, 13, 14, 15],  # wide clause
        [-6, -7],
        [2, -4, 5],
        [-1, -2, -16],
        [16, 17],
        [-17, 18, -19, 20],
        [19],
        [-20, -18],
        [21, -21, 22],        # tautology with an extra literal
        [-22, -1, -2, -3],
        [-12, -13, 14],
        [1, -1],
    ]
    # variable 23 and 24 appear in no clause
    return 24, o.csr_from_lists([[L(x) for x in c] for c in cl])


def run_probe(cnf_path, T, max_iters, out):
    subprocess.run([o.REF_PROBE, "trace", cnf_path, str(T), str(max_iters), str(RD_SEED), out],
                   check=True)
    return o.read_trace(out)


def pack_fixture(name, n_vars, offs, lits, T, tr, solve_json=None):
    it = tr["iters"]
    A = np.stack([o.pack_bools(r["A"]) for r in it])
    U_ptr = np.cumsum([0] + [r["U"].size for r in it]).astype(np.uint64)
    M_ptr = np.cumsum([0] + [r["M"].size for r in it]).astype(np.uint64)
    U = np.concatenate([r["U"] for r in it]).astype(np.uint32)
    M = np.concatenate([r["M"] for r in it]).astype(np.uint32)
    dres = np.array([r["dres"] for r in it], np.uint64)
    st = tr["stats"]
    extra = {}
    if solve_json is not None:
        extra["solve_stats"] = np.array([solve_json["n_iterations"], solve_json["n_resamples"],
                                         solve_json["avg_mis_size"], solve_json["valid"]], np.uint64)
        extra["solve_A"] = o.pack_bools(np.frombuffer(solve_json["assignment"].encode(), np.uint8) - 48)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), n_vars=np.uint32(n_vars), offs=offs,
                        lits=lits, T=np.uint32(T), A=A, U=U, U_ptr=U_ptr, M=M, M_ptr=M_ptr,
                        dres=dres,
                        stats=np.array([st["n_iterations"], st["n_resamples"], st["avg_mis_size"]],
                                       np.uint64),
                        A_final=o.pack_bools(tr["A_final"]), **extra)


def stream_fixtures(tmp):
    """Streaming solve (SATInstance::solve(getEnumeratedClause, n, batch), T=1): per-iteration
    (A_i, violated clauses in yield order, MIS in pick order, MIS size after every batch, delta
    n_resamples), final Statistics of the probe loop and of the real solve (same RNG)."""
    specs = [
        # name, instance, batch sizes
        ("r2_3sat_200_400", (200, 400, 3, 0), [1, 64, 1000]),
        ("r2_3sat_2000_4000", (2000, 4000, 3, 0), [256]),
        ("edge", None, [5]),
    ]
    out = []
    for name, inst, batches in specs:
        if inst is None:
            n, (offs, lits) = edge_instance()
        else:
            n, m, k, kind = inst
            offs, lits = o.generate_ksat(1, n, m, k, kind)
        cnf = os.path.join(tmp, name + "_s.cnf")
        with open(cnf, "w") as f:
            f.write(o.to_dimacs(n, offs, lits))
        for bs in batches:
            path = os.path.join(tmp, "s.bin")
            subprocess.run([o.REF_PROBE, "stream", cnf, str(bs), str(RD_SEED), path], check=True)
            tr = o.read_stream_trace(path)
            it = tr["iters"]
            ptr = lambda key: np.cumsum([0] + [r[key].size for r in it]).astype(np.uint64)
            cat = lambda key: np.concatenate([r[key] for r in it]).astype(np.uint32)
            st, ss = tr["stats"], tr["solve_stats"]
            fx = f"stream_{name}_b{bs}"
            np.savez_compressed(
                os.path.join(HERE, fx + ".npz"), n_vars=np.uint32(n), offs=offs, lits=lits,
                batch=np.uint64(bs), A=np.stack([o.pack_bools(r["A"]) for r in it]),
                U=cat("U"), U_ptr=ptr("U"), M=cat("M"), M_ptr=ptr("M"), cum=cat("cum"),
                cum_ptr=ptr("cum"), dres=np.array([r["dres"] for r in it], np.uint64),
                stats=np.array([st["n_iterations"], st["n_resamples"], st["avg_mis_size"]], np.uint64),
                A_final=o.pack_bools(tr["A_final"]),
                solve_stats=np.array([ss["n_iterations"], ss["n_resamples"], ss["avg_mis_size"]], np.uint64),
                solve_A=o.pack_bools(tr["solve_A"]))
            out.append(dict(fixture=fx, n_vars=n, n_clauses=len(offs) - 1, batch=bs, iters=len(it)))
    return out


def stream_rr_fixtures(tmp, keep):
    """Streaming solve with T > 1 threads (ref_probe `stream-rr`): per iteration A_i, every
    generator's state {n_yielded, finished, c} at its start, per batch step the violated list of
    every generator and the MIS size after the step, the MIS in pick order, delta n_resamples and
    the check's verdict.  Not reproducible (T > 1 resampling, see the module docstring): an
    existing fixture is kept unless --rewrite-rr."""
    specs = [
        # name, instance, [(T, batch)]
        ("r2_3sat_200_400", (200, 400, 3, 0), [(2, 1), (2, 64), (3, 7), (4, 37)]),
        ("r2_3sat_2000_4000", (2000, 4000, 3, 0), [(2, 256), (4, 100)]),
        ("k8_4000_6000", (4000, 6000, 8, 0), [(4, 500)]),
        ("edge", None, [(3, 6), (5, 1), (20, 3)]),
    ]
    out = []
    for name, inst, runs in specs:
        if inst is None:
            n, (offs, lits) = edge_instance()
        else:
            n, m, k, kind = inst
            offs, lits = o.generate_ksat(1, n, m, k, kind)
        cnf = os.path.join(tmp, name + "_q.cnf")
        with open(cnf, "w") as f:
            f.write(o.to_dimacs(n, offs, lits))
        for T, bs in runs:
            fx = f"streamrr_{name}_T{T}_b{bs}"
            if keep(fx):
                continue
            path = os.path.join(tmp, "q.bin")
            subprocess.run([o.REF_PROBE, "stream-rr", cnf, str(bs), str(T), str(RD_SEED), path], check=True)
            tr = o.read_stream_rr_trace(path)
            it = tr["iters"]
            flat = [l for r in it for lists in r["steps"] for l in lists]
            st = tr["stats"]
            np.savez_compressed(
                os.path.join(HERE, fx + ".npz"), n_vars=np.uint32(n), offs=offs, lits=lits,
                batch=np.uint64(bs), T=np.uint32(T), A=np.stack([o.pack_bools(r["A"]) for r in it]),
                G=np.stack([r["G"] for r in it]).astype(np.uint64),
                nsteps=np.array([len(r["steps"]) for r in it], np.uint64),
                L=(np.concatenate(flat) if flat else np.zeros(0)).astype(np.uint32),
                L_ptr=np.cumsum([0] + [l.size for l in flat]).astype(np.uint64),
                cum=np.array([c for r in it for c in r["cum"]], np.uint64),
                M=np.concatenate([r["M"] for r in it]).astype(np.uint32),
                M_ptr=np.cumsum([0] + [r["M"].size for r in it]).astype(np.uint64),
                dres=np.array([r["dres"] for r in it], np.uint64),
                solved=np.array([r["solved"] for r in it], np.uint64),
                stats=np.array([st["n_iterations"], st["n_resamples"], st["avg_mis_size"]], np.uint64),
                A_final=o.pack_bools(tr["A_final"]), G_final=tr["G_final"].astype(np.uint64))
            out.append(dict(fixture=fx, n_vars=n, n_clauses=len(offs) - 1, T=T, batch=bs, iters=len(it),
                            reproducible=False))
    return out


def main():
    if "--stream-rr-only" in sys.argv:
        tmp = tempfile.mkdtemp()
        mf = os.path.join(HERE, "manifest.json")
        man = json.load(open(mf))
        old = {e["fixture"]: e for e in man.get("stream_rr_fixtures", [])}
        kept = []

        def keep(fx):
            if "--rewrite-rr" in sys.argv or fx not in old or not os.path.exists(os.path.join(HERE, fx + ".npz")):
                return False
            kept.append(old[fx])
            return True

        sm = stream_rr_fixtures(tmp, keep)
        man["stream_rr_fixtures"] = kept + sm
        with open(mf, "w") as f:
            json.dump(man, f, indent=1)
        print("wrote", len(sm), "streaming T > 1 fixtures, kept", len(kept))
        return
    if "--stream-only" in sys.argv:
        tmp = tempfile.mkdtemp()
        sm = stream_fixtures(tmp)
        mf = os.path.join(HERE, "manifest.json")
        man = json.load(open(mf))
        man["stream_fixtures"] = sm
        with open(mf, "w") as f:
            json.dump(man, f, indent=1)
        print("wrote", len(sm), "streaming fixtures")
        return
    if not os.path.exists(o.REF_PROBE):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    tmp = tempfile.mkdtemp()
    specs = [
        # name, (n, m, k, kind), [(T, max_iters)]
        ("c1_3sat_200_800", (200, 800, 3, 0), [(1, 60), (2, 40), (4, 40), (8, 40)]),
        ("u3sat_2500_10000", (2500, 10000, 3, 0), [(1, 20), (8, 10)]),
        ("r2_3sat_200_400", (200, 400, 3, 0), [(1, 0), (3, 0)]),
        ("k8_4000_6000", (4000, 6000, 8, 0), [(1, 0), (4, 0)]),
        ("pl3sat_2000_8000", (2000, 8000, 3, 1), [(1, 20)]),
    ]
    manifest = []
    rewrite_rr = "--rewrite-rr" in sys.argv
    old_man = {}
    mf_path = os.path.join(HERE, "manifest.json")
    if os.path.exists(mf_path):
        old_man = {e["fixture"]: e for e in json.load(open(mf_path)).get("fixtures", [])}

    def keep_rr(fx):  # an existing T > 1 fixture stays as committed (see the docstring)
        if rewrite_rr or fx not in old_man or not os.path.exists(os.path.join(HERE, fx + ".npz")):
            return False
        manifest.append(dict(old_man[fx], reproducible=False))
        return True

    for name, (n, m, k, kind), runs in specs:
        offs, lits = o.generate_ksat(1, n, m, k, kind)
        cnf = os.path.join(tmp, name + ".cnf")
        with open(cnf, "w") as f:
            f.write(o.to_dimacs(n, offs, lits))
        for T, mi in runs:
            if T > 1 and keep_rr(f"{name}_T{T}"):
                continue
            tr = run_probe(cnf, T, mi, os.path.join(tmp, "t.bin"))
            sj = None
            if T == 1 and mi == 0:
                out = subprocess.run([o.REF_PROBE, "solve", cnf, "1", str(RD_SEED)], check=True,
                                     capture_output=True, text=True).stdout
                sj = json.loads(out)
            fx = f"{name}_T{T}"
            pack_fixture(fx, n, offs, lits, T, tr, sj)
            manifest.append(dict(fixture=fx, n_vars=n, n_clauses=m, k=k, kind=kind, T=T,
                                 max_iters=mi, iters=len(tr["iters"]), reproducible=T == 1))
    n, (offs, lits) = edge_instance()
    cnf = os.path.join(tmp, "edge.cnf")
    with open(cnf, "w") as f:
        f.write(o.to_dimacs(n, offs, lits))
    for T in (1, 3):
        if T > 1 and keep_rr(f"edge_T{T}"):
            continue
        tr = run_probe(cnf, T, 0, os.path.join(tmp, "t.bin"))
        sj = None
        if T == 1:
            out = subprocess.run([o.REF_PROBE, "solve", cnf, "1", str(RD_SEED)], check=True,
                                 capture_output=True, text=True).stdout
            sj = json.loads(out)
        pack_fixture(f"edge_T{T}", n, offs, lits, T, tr, sj)
        manifest.append(dict(fixture=f"edge_T{T}", n_vars=n, n_clauses=len(offs) - 1, T=T,
                             iters=len(tr["iters"]), reproducible=T == 1))

    # ---- DIMACS loader edge cases: reference cnf_header_read + cnf_data_read output
    cases = {
        "basic": "c comment\np cnf 3 2\n1 -2 0\n2 3 0\n",
        "no_trailing_newline": "p cnf 3 3\n1 -2 0\n2 3 0\n-1 0\n3 0",
        "percent_terminator": "p cnf 3 2\n1 -2 0\n2 3 0\n%\n0\n\n",
        "multi_line_clause": "p cnf 4 2\n1 -2\n3 0 -4\n 2 0\n",
        "shared_line": "p cnf 3 3\n1 0 -2 0 3 -1 0\n",
        "comments_blank": "c a\nC b\n\n   \np cnf 2 2\nc mid\n1 2 0\n\n-1 -2 0\n",
        "upper_header": "P CNF 2 1\n-1 2 0\n",
        "tab_header": "p\tcnf\t2 1\n1 -2 0\n",
        "tab_in_clause": "p cnf 3 2\n1\t2 0\n3 0\n2 0\n",
        "plus_sign_crlf": "p cnf 3 2\r\n+1 -2 0\r\n3 0\r\n",
        "garbage_word": "p cnf 3 2\n1 x 2 0\n1 2 0\n-3 0\n",
        "leading_spaces": "p cnf 3 2\n   1   -3   0\n  2 0  \n",
        "extra_clauses": "p cnf 3 2\n1 0\n2 0\n3 0\n",
        "big_numbers": "p cnf 100000 1\n100000 -99999 1 0\n",
    }
    loader = {}
    for key, text in cases.items():
        p = os.path.join(tmp, key + ".cnf")
        with open(p, "w", newline="") as f:
            f.write(text)
        out = subprocess.run([o.REF_PROBE, "cnf", p], check=True, capture_output=True,
                             text=True).stdout
        loader[key] = dict(text=text, ref=json.loads(out))
    with open(os.path.join(HERE, "dimacs_cases.json"), "w") as f:
        json.dump(loader, f, indent=1)
    sm = stream_fixtures(tmp)
    old_q = {}
    if os.path.exists(mf_path):
        old_q = {e["fixture"]: e for e in json.load(open(mf_path)).get("stream_rr_fixtures", [])}
    kept_q = []

    def keep_q(fx):
        if rewrite_rr or fx not in old_q or not os.path.exists(os.path.join(HERE, fx + ".npz")):
            return False
        kept_q.append(old_q[fx])
        return True

    sq = stream_rr_fixtures(tmp, keep_q)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(dict(rd_seed=RD_SEED, generator="oracle.generate_ksat(gen_seed=1, ...)",
                       fixtures=manifest, stream_fixtures=sm, stream_rr_fixtures=kept_q + sq), f, indent=1)
    print("wrote", len(manifest), "trajectory fixtures and", len(loader), "loader cases")


if __name__ == "__main__":
    main()
