"""Pin the oracle (CPU restatement) against the reference's own outputs.

The golden vectors in tests/golden/ were produced by oracle/_ref/ref_probe, a driver
compiled from the reference sources (tests/golden/make_golden.py).  Every deterministic
map of the serial path is checked here: A_i -> U_i (eval, Clause.h:34-46 via
SATInstance.h:264-280), U_i -> M_i (LFMIS for T=1 / round-robin for T>1,
SATInstance.h:391-451), M_i -> delta n_resamples (SATInstance.h:363) and the Statistics
arithmetic (SATInstance.h:313-317).  Philox is pinned by the Random123 KAT vectors.
"""
import glob
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

FIXTURES = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not os.path.basename(p).startswith("stream"))
STREAM_FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "stream_*.npz")))


def load(path):
    return dict(np.load(path, allow_pickle=False))


def test_philox_kat(oracle_mod):
    o = oracle_mod
    # Random123 kat_vectors, philox4x32 10 rounds
    assert list(o.philox4x32_10([0, 0, 0, 0], [0, 0])) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert list(o.philox4x32_10([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2)) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert list(o.philox4x32_10([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                                [0xA4093822, 0x299F31D0])) == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_fixtures_present():
    assert len(FIXTURES) >= 10


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[:-4] for p in FIXTURES])
def test_oracle_matches_reference_trace(oracle_mod, path):
    o = oracle_mod
    f = load(path)
    n, T = int(f["n_vars"]), int(f["T"])
    offs, lits = f["offs"], f["lits"]
    m = offs.size - 1
    total_mis = 0
    n_it = f["A"].shape[0]
    for i in range(n_it):
        A = f["A"][i]
        nu, vm = o.eval_mask(offs, lits, A)
        U = o.mask_to_list(m, vm)
        U_ref = f["U"][int(f["U_ptr"][i]):int(f["U_ptr"][i + 1])]
        np.testing.assert_array_equal(U, U_ref, err_msg=f"U_{i}")
        M_ref = f["M"][int(f["M_ptr"][i]):int(f["M_ptr"][i + 1])]
        if nu == 0:
            assert M_ref.size == 0
            continue
        M = o.lfmis(n, offs, lits, U) if T == 1 else o.rr_mis(n, offs, lits, U, T)
        np.testing.assert_array_equal(M, M_ref, err_msg=f"M_{i}")  # same pick order
        dres = int(np.sum(offs[M.astype(np.int64) + 1] - offs[M.astype(np.int64)]))
        if int(f["dres"][i]) or i + 1 < n_it:
            assert dres == int(f["dres"][i])
            total_mis += M.size
        # the reference resampled exactly the variables of M_i (others unchanged)
        if i + 1 < n_it:
            a0 = o.unpack_words(A, n)
            a1 = o.unpack_words(f["A"][i + 1], n)
            changed = np.nonzero(a0 != a1)[0]
            vars_m = np.unique(lits[np.concatenate([np.arange(offs[c], offs[c + 1]) for c in M]).astype(np.int64)] >> 1)
            assert np.isin(changed, vars_m).all()
    # Statistics arithmetic (SATInstance.h:313-317) for runs that ended by convergence
    st = f["stats"]
    last_nu = int(f["U_ptr"][-1] - f["U_ptr"][-2])
    if last_nu == 0:
        assert int(st[0]) == n_it
        assert int(st[1]) == int(f["dres"].sum())
        assert int(st[2]) == total_mis // n_it


@pytest.mark.parametrize("path", [p for p in FIXTURES if "solve_stats" in np.load(p).files],
                         ids=lambda p: os.path.basename(p)[:-4])
def test_probe_loop_equals_real_solve(path):
    """The per-iteration probe loop reproduces SATInstance::solve exactly (same RNG)."""
    f = load(path)
    ss = f["solve_stats"]
    assert int(ss[3]) == 1  # verify_validity true
    np.testing.assert_array_equal(f["stats"], ss[:3])
    np.testing.assert_array_equal(f["A_final"], f["solve_A"])


def test_oracle_solve_semantics(oracle_mod):
    """Serial loop with Philox: converges on a ratio-2 instance, stats consistent with trace."""
    o = oracle_mod
    offs, lits = o.generate_ksat(3, 500, 1000, 3)
    st, A, rows = o.solve(500, offs, lits, seed=11, trace=True)
    assert st["solved"] == 1
    nu, _ = o.eval_mask(offs, lits, A)
    assert nu == 0
    assert st["n_iterations"] == len(rows) + 1
    assert st["n_resamples"] == sum(r[3] for r in rows)
    assert st["avg_mis_size"] == sum(r[2] for r in rows) // st["n_iterations"]


@pytest.mark.parametrize("T", [2, 5, 70])
def test_oracle_solve_rr_replays(oracle_mod, T):
    """T-chunk loop (orc_solve_rr): every iteration is eval -> round-robin MIS (orc_rr_mis,
    pinned above by the reference's T>1 fixtures) -> Philox resample of the MIS variables."""
    o = oracle_mod
    n = 400
    offs, lits = o.generate_ksat(4, n, 1600, 3)
    st, A_end, rows = o.solve(n, offs, lits, seed=9, max_iters=25, trace=True, T=T)
    A = o.init_assignment(9, n)
    for it, nu, nm, dres, A_after in rows:
        cnt, vm = o.eval_mask(offs, lits, A)
        assert cnt == nu
        M = o.rr_mis(n, offs, lits, o.mask_to_list(offs.size - 1, vm), T)
        assert M.size == nm
        assert dres == int(np.sum(offs[M.astype(np.int64) + 1] - offs[M.astype(np.int64)]))
        o.resample_words(A, 9, it - 1, o.clause_vars(offs, lits, M))
        np.testing.assert_array_equal(A, A_after, err_msg=f"iter {it}")
    np.testing.assert_array_equal(A, A_end)
    # T = 1 chunking and an explicit single chunk give the LFMIS loop
    st1, A1, _ = o.solve(n, offs, lits, seed=9, max_iters=25)
    stc, Ac, _ = o.solve(n, offs, lits, seed=9, max_iters=25, T=1, chunk_starts=[0, offs.size - 1])
    np.testing.assert_array_equal(A1, Ac)


def test_oracle_max_iters(oracle_mod):
    o = oracle_mod
    offs, lits = o.generate_ksat(1, 200, 800, 3)
    st, A, rows = o.solve(200, offs, lits, seed=5, max_iters=7, trace=True)
    assert st["n_iterations"] == 7 and st["solved"] == 0 and len(rows) == 6


def test_chunk_bounds_match_main_cpp(oracle_mod):
    """example/main.cpp:149-178: chunk 0 receives chunk_size+1 clauses."""
    o = oracle_mod
    for m, T in [(800, 2), (800, 3), (10, 3), (3, 8), (10000, 8), (1, 1)]:
        chunk = -(-m // T)
        t = 0
        owner = []
        for c in range(m):
            if c > (t + 1) * chunk:
                t += 1
            owner.append(t)
        s = o.chunk_bounds(m, T)
        for c in range(m):
            assert s[owner[c]] <= c < s[owner[c] + 1]


def _ref_lists(ref):
    lcn, lv = ref["l_c_num"], ref["l_val"]
    out, p = [], 0
    for n in lcn:
        out.append(lv[p:p + n])
        p += n
    return out


def test_oracle_dimacs_matches_reference_loader(oracle_mod):
    o = oracle_mod
    cases = json.load(open(os.path.join(GOLDEN, "dimacs_cases.json")))
    for key, case in cases.items():
        ref = case["ref"]
        rc, res = o.dimacs_parse(case["text"].encode())
        assert rc == 0, key
        v, offs, lits = res
        assert v == ref["v_num"] and offs.size - 1 == ref["c_num"], key
        enc = [[2 * x - 2 if x > 0 else -2 * x - 1 for x in cl] for cl in _ref_lists(ref)]
        got = [list(lits[offs[c]:offs[c + 1]]) for c in range(offs.size - 1)]
        assert got == enc, key


def test_oracle_generator_distinct(oracle_mod):
    o = oracle_mod
    for kind in (0, 1):
        offs, lits = o.generate_ksat(9, 50, 2000, 8, kind)
        v = (lits >> 1).reshape(-1, 8)
        assert all(len(set(r)) == 8 for r in v.tolist())
        assert v.max() < 50


def test_numpy_philox_matches_c_oracle(oracle_mod):
    o = oracle_mod
    vs = np.arange(0, 3000, 7, dtype=np.uint32)
    for seed, it in [(1, 0), (12345, 77), ((7 << 32) | 9, (3 << 32) | 5)]:
        ref = np.array([o.resample_bit(seed, it, int(v)) for v in vs], np.uint32)
        np.testing.assert_array_equal(o.philox_bits(seed, it, vs), ref)


# ---------------------------------------------------------------------------------------------
# Streaming solve (SATInstance::solve(getEnumeratedClause, n_clauses, batch), SATInstance.h:70-153,
# one thread): fixtures from the reference's own ClauseGenerator / populate_mis_parallel /
# resample_clauses (ref_probe `stream`).


def test_stream_fixtures_present():
    assert len(STREAM_FIXTURES) >= 4


def test_stream_order_is_the_generator_lcg():
    """ClauseGenerator.h:47: c <- (c + P) % m from c = 0, P = 9223372036854775783."""
    from conftest import ROOT  # noqa: F401
    import oracle as o

    P = 9223372036854775783
    for m in (1, 7, 10, 400, 4000, 99991):
        c, ref = 0, []
        for _ in range(m):
            c = (c + P) % m
            ref.append(c)
        np.testing.assert_array_equal(o.stream_order(m), np.array(ref, np.uint32))


@pytest.mark.parametrize("path", STREAM_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_matches_reference_stream(oracle_mod, path):
    """Per iteration the reference yields a window of the generator's sequence: all m steps in
    the first iteration, then m - k0 steps, k0 = first violated clause index + 1 (where its
    end-of-iteration check stopped; all m again when k0 == m)."""
    o = oracle_mod
    f = load(path)
    n, offs, lits, bs = int(f["n_vars"]), f["offs"], f["lits"], int(f["batch"])
    m = offs.size - 1
    period = o.stream_order(m)          # s_1 .. s_m; the sequence repeats with period m
    S, window = 0, m                    # steps taken before this iteration, window length
    n_it = f["A"].shape[0]
    total_w = 0
    for i in range(n_it):
        A = f["A"][i]
        U_ref = f["U"][int(f["U_ptr"][i]):int(f["U_ptr"][i + 1])]
        M_ref = f["M"][int(f["M_ptr"][i]):int(f["M_ptr"][i + 1])]
        cum = f["cum"][int(f["cum_ptr"][i]):int(f["cum_ptr"][i + 1])]
        order = period[(S + np.arange(window)) % m]
        _, vm = o.eval_mask(offs, lits, A)
        bits = np.unpackbits(vm.view(np.uint8), bitorder="little")[:m]
        np.testing.assert_array_equal(order[bits[order] == 1], U_ref, err_msg=f"U_{i} in yield order")
        M = o.stream_mis(n, offs, lits, A, order)
        np.testing.assert_array_equal(M, M_ref, err_msg=f"M_{i} (pick order)")
        nb = -(-window // bs)
        pos = {int(c): k for k, c in enumerate(order)}
        b_of = np.array([pos[int(c)] // bs for c in M], np.int64)
        assert cum.size == nb
        np.testing.assert_array_equal(cum, [(b_of <= b).sum() for b in range(nb)])
        w = int((nb - b_of).sum())
        assert w == int(cum.sum())
        total_w += w
        assert int(f["dres"][i]) == int(np.sum(offs[M.astype(np.int64) + 1] - offs[M.astype(np.int64)]))
        if i + 1 < n_it:
            a0 = o.unpack_words(A, n)
            a1 = o.unpack_words(f["A"][i + 1], n)
            changed = np.nonzero(a0 != a1)[0]
            idx = [np.arange(offs[c], offs[c + 1]) for c in M] or [np.zeros(0, np.int64)]
            vars_m = np.unique(lits[np.concatenate(idx).astype(np.int64)] >> 1)
            assert np.isin(changed, vars_m).all()
            # next window: where the reference's check stopped under the new assignment
            _, vm1 = o.eval_mask(offs, lits, f["A"][i + 1])
            bits1 = np.unpackbits(vm1.view(np.uint8), bitorder="little")[:m]
            k0 = int(np.nonzero(bits1)[0][0]) + 1
            S += window
            window = m if k0 == m else m - k0
    st = f["stats"]
    assert int(st[0]) == n_it
    assert int(st[1]) == int(f["dres"].sum())
    assert int(st[2]) == total_w // n_it
    # the probe's loop is the real streaming solve (same interposed random_device)
    np.testing.assert_array_equal(f["solve_stats"], st)
    np.testing.assert_array_equal(f["solve_A"], f["A_final"])


def test_oracle_solve_stream_semantics(oracle_mod):
    """Philox restatement: converges; stats consistent with the per-iteration rows."""
    o = oracle_mod
    offs, lits = o.generate_ksat(3, 500, 1000, 3)
    for bs in (1, 37, 5000):
        st, A, rows = o.solve_stream(500, offs, lits, 11, bs, trace=True)
        assert st["solved"] == 1 and o.eval_mask(offs, lits, A)[0] == 0
        assert st["n_iterations"] == len(rows)
        assert st["n_resamples"] == sum(r[3] for r in rows)
        assert st["avg_mis_size"] == st["sum_mis_size"] // st["n_iterations"]
    # the C restatement follows the same windows / MIS as the fixture-checked maps above
    m = offs.size - 1
    period = o.stream_order(m)
    for bs in (1, 50):
        st, A_end, rows = o.solve_stream(500, offs, lits, 13, bs, trace=True)
        A = o.init_assignment(13, 500)
        S, window, w_total = 0, m, 0
        for it, nu, nm, dres, A_after in rows:
            order = period[(S + np.arange(window)) % m]
            M = o.stream_mis(500, offs, lits, A, order)
            assert (nu, nm) == (o.eval_mask(offs, lits, A)[0], M.size)
            assert dres == int(np.sum(offs[M.astype(np.int64) + 1] - offs[M.astype(np.int64)]))
            pos = {int(c): k for k, c in enumerate(order)}
            nb = -(-window // bs)
            w_total += sum(nb - pos[int(c)] // bs for c in M)
            np.testing.assert_array_equal(
                o.resample_words(A.copy(), 13, it - 1, o.clause_vars(offs, lits, M)), A_after)
            A = A_after
            nu1, vm1 = o.eval_mask(offs, lits, A)
            if nu1:
                k0 = int(np.nonzero(np.unpackbits(vm1.view(np.uint8), bitorder="little")[:m])[0][0]) + 1
                S += window
                window = m if k0 == m else m - k0
        assert st["sum_mis_size"] == w_total
    # already satisfied: one iteration, nothing resampled
    offs1 = np.array([0, 1], np.uint64)
    A0 = o.init_assignment(2, 4)
    lit = np.array([0 if (A0[0] & 1) else 1], np.uint32)  # the literal of variable 0 that is true
    st, A, rows = o.solve_stream(4, offs1, lit, 2, 8, trace=True)
    assert st == {**st, "n_iterations": 1, "n_resamples": 0, "avg_mis_size": 0, "solved": 1}


# ---------------------------------------------------------------------------------------------
# Streaming solve with T > 1 threads: fixtures from the reference's own ClauseGenerators,
# populate_mis_parallel and resample_clauses (ref_probe `stream-rr`; its end-of-iteration check
# runs in lock step, see oracle/ref_probe.cpp).  Per iteration: set A_i and the generators'
# recorded state, replay the batch loop, compare every step's violated lists, the MIS (pick
# order), its size after every step; then the check's verdict and the generators it leaves.
STREAM_RR_FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "streamrr_*.npz")))


def test_stream_rr_fixtures_present():
    assert len(STREAM_RR_FIXTURES) >= 8
    Ts = {int(load(p)["T"]) for p in STREAM_RR_FIXTURES}
    assert {2, 4} <= Ts


def _gens_from(G, m, T):
    import oracle as o
    gens = o.stream_gens(m, T)
    for g, row in zip(gens, G):
        g["ny"], g["fin"], g["c"] = int(row[0]), bool(row[1]), int(row[2])
    return gens


def _gens_state(gens):
    return np.array([[g["ny"], int(g["fin"]), g["c"]] for g in gens], np.uint64)


@pytest.mark.parametrize("path", STREAM_RR_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_matches_reference_stream_rr(oracle_mod, path):
    o = oracle_mod
    f = load(path)
    n, offs, lits, bs, T = int(f["n_vars"]), f["offs"], f["lits"], int(f["batch"]), int(f["T"])
    m = offs.size - 1
    n_it = f["A"].shape[0]
    # the generators start fresh (SATInstance.h:74-86)
    np.testing.assert_array_equal(f["G"][0], _gens_state(o.stream_gens(m, T)))
    assert [g["n"] for g in o.stream_gens(m, T)] == [m // T] * (T - 1) + [m - (T - 1) * (m // T)]
    step0, total_w = 0, 0
    for i in range(n_it):
        gens = _gens_from(f["G"][i], m, T)
        steps, M, cum = o.stream_rr_iteration(n, offs, lits, f["A"][i], bs, gens)
        ns = int(f["nsteps"][i])
        assert len(steps) == ns, f"iteration {i}: batch steps"
        for s in range(ns):
            for t in range(T):
                q = (step0 + s) * T + t
                ref = f["L"][int(f["L_ptr"][q]):int(f["L_ptr"][q + 1])]
                np.testing.assert_array_equal(np.array(steps[s][t], np.uint32), ref,
                                              err_msg=f"iteration {i} step {s} generator {t}")
        np.testing.assert_array_equal(cum, f["cum"][step0:step0 + ns], err_msg=f"iteration {i}: MIS sizes")
        np.testing.assert_array_equal(M, f["M"][int(f["M_ptr"][i]):int(f["M_ptr"][i + 1])],
                                      err_msg=f"iteration {i}: MIS")
        assert int(f["dres"][i]) == int(np.sum(offs[M.astype(np.int64) + 1] - offs[M.astype(np.int64)]))
        total_w += int(np.sum(cum))
        step0 += ns
        # the check under the next assignment, and where it leaves the generators
        A_next = f["A"][i + 1] if i + 1 < n_it else f["A_final"]
        solved = o.stream_rr_check(offs, lits, A_next, gens)
        assert solved == bool(f["solved"][i])
        if not solved:
            G_next = f["G"][i + 1] if i + 1 < n_it else f["G_final"]
            np.testing.assert_array_equal(_gens_state(gens), G_next, err_msg=f"iteration {i}: check")
        if i + 1 < n_it:  # only MIS variables changed
            M64 = M.astype(np.int64)
            idx = [np.arange(offs[c], offs[c + 1]) for c in M64] or [np.zeros(0, np.int64)]
            vars_m = np.unique(lits[np.concatenate(idx).astype(np.int64)] >> 1)
            changed = np.nonzero(o.unpack_words(f["A"][i], n) != o.unpack_words(f["A"][i + 1], n))[0]
            assert np.isin(changed, vars_m).all()
    st = f["stats"]
    assert int(st[0]) == n_it
    assert int(st[1]) == int(f["dres"].sum())
    assert int(st[2]) == total_w // n_it


def test_oracle_solve_stream_rr_semantics(oracle_mod):
    """orc_solve_stream_rr (C, Philox) follows the fixture-pinned Python restatement: every
    iteration's MIS size, delta n_resamples and resampled assignment, and the statistics."""
    o = oracle_mod
    cases = [
        (o.generate_ksat(3, 300, 800, 3), 300, [(2, 1), (2, 50), (3, 133), (4, 1000), (7, 57)]),
        (o.generate_ksat(5, 900, 2000, 4), 900, [(4, 64), (16, 5)]),
        (o.generate_ksat(6, 40, 30, 3), 40, [(32, 2), (5, 1)]),  # m < T: empty generators
    ]
    for (offs, lits), n, runs in cases:
        m = offs.size - 1
        for T, bs in runs:
            seed = 17 + T
            rc, st, A_end, rows = o.solve_stream_rr(n, offs, lits, seed, bs, T, trace=True)
            assert rc == 0 and st["solved"] == 1 and o.eval_mask(offs, lits, A_end)[0] == 0
            gens = o.stream_gens(m, T)
            A = o.init_assignment(seed, n)
            w_total = 0
            for it, nu, nm, dres, A_after in rows:
                steps, M, cum = o.stream_rr_iteration(n, offs, lits, A, bs, gens)
                assert (nu, nm) == (o.eval_mask(offs, lits, A)[0], M.size), (T, bs, it)
                assert dres == int(np.sum(offs[M.astype(np.int64) + 1] - offs[M.astype(np.int64)]))
                w_total += sum(cum)
                np.testing.assert_array_equal(
                    o.resample_words(A.copy(), seed, it - 1, o.clause_vars(offs, lits, M)), A_after)
                A = A_after
                if o.stream_rr_check(offs, lits, A, gens):
                    break
            assert st["n_iterations"] == len(rows)
            assert st["sum_mis_size"] == w_total and st["avg_mis_size"] == w_total // len(rows)
    # T = 1 is the one-thread window rule
    offs, lits = o.generate_ksat(3, 300, 800, 3)
    for bs in (1, 77):
        a = o.solve_stream(300, offs, lits, 5, bs)
        b = o.solve_stream_rr(300, offs, lits, 5, bs, 1)
        assert a[0] == b[1] and np.array_equal(a[1], b[2])
    # refusals: an empty clause; generators that never finish together (the reference loops)
    offs_e, lits_e = o.csr_from_lists([[0, 2], [], [4]])
    assert o.solve_stream_rr(3, offs_e, lits_e, 1, 1, 2)[0] == -2
    # m = 800, T = 3: generators of 266, 266 and 268 clauses, batches of 9 (30 per walk each):
    # after a check that leaves them at 266 - r and 268 - r unyielded, the first two finish at
    # steps ceil((266 - r) / 9) + 30 j, the last at ceil((268 - r) / 9) + 30 j -- never together
    offs, lits = o.generate_ksat(3, 300, 800, 3)
    assert o.solve_stream_rr(300, offs, lits, 20, 9, 3, step_cap=10000)[0] == -1


def test_bench_trajectory_file_regenerates(oracle_mod):
    """tests/golden/bench_trajectory.json (what bench.py checks its final state against) is the
    oracle's trajectory of the bench instances: recompute the first iterations of every entry."""
    import subprocess
    import sys

    script = os.path.join(os.path.dirname(__file__), "golden", "make_bench_trajectory.py")
    r = subprocess.run([sys.executable, script, "--check", "4"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr


def test_bench_trajectory_check_logic():
    """bench.trajectory_check: match, mismatch and out-of-range reporting (no GPU)."""
    import json
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))
    import bench

    tr = json.load(open(bench.TRAJECTORY_JSON))["trajectories"]["C2_T1"]["rows"]
    it, nu, mis, res, dig = tr[9]
    st = {"n_iterations": it, "n_violated": nu, "sum_mis_size": mis, "n_resamples": res}

    class W:  # assignment words whose digest is the committed one
        pass

    import alllsatisfiabilitysolver_amd.solver as S

    orig = S.assignment_digest
    try:
        S.assignment_digest = lambda w: dig
        import alllsatisfiabilitysolver_amd as pkg

        pkg.assignment_digest = S.assignment_digest
        assert bench.trajectory_check("C2", 1, st, None, 1)["match"] is True
        assert bench.trajectory_check("C2", 1, {**st, "n_resamples": res + 1}, None, 1)["match"] is False
        assert bench.trajectory_check("C2", 1, {**st, "n_iterations": 10_000}, None, 1)["match"] is None
        assert bench.trajectory_check("C2", 7, st, None, 1)["match"] is None  # no such entry
        # another solve seed than the committed trajectories': not a mismatch, no check
        r = bench.trajectory_check("C2", 1, st, None, 2)
        assert r["match"] is None and "seed" in r["reason"]
        # the 8-GPU configs and the 8-SAT config have entries (a sharded line checks itself)
        for cfg in ("C3", "C4", "C5"):
            assert f"{cfg}_T1" in json.load(open(bench.TRAJECTORY_JSON))["trajectories"]
    finally:
        S.assignment_digest = orig
        pkg.assignment_digest = orig


REFRNG_FIXTURES = [p for p in FIXTURES if p.endswith("_T1.npz")]


@pytest.mark.parametrize("path", REFRNG_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reference_rng_reproduces_reference_trajectory(path, oracle_mod):
    """The reference-RNG mode (orc_solve_refrng): with the probe's random_device stand-in
    (rd_seed = 7, tests/golden/manifest.json), the restated RBG<minstd_rand0> /
    uniform_int_distribution<unsigned long long> stream reproduces the reference's whole T = 1
    trajectory -- the initial VariablesArray fill, the assignment after every iteration, the
    final statistics -- as recorded by the reference's own code (oracle/ref_probe.cpp trace)."""
    o = oracle_mod
    f = load(path)
    man = {d["fixture"]: d for d in json.load(open(os.path.join(GOLDEN, "manifest.json")))["fixtures"]}
    name = os.path.basename(path)[:-4]
    n, offs, lits = int(f["n_vars"]), f["offs"], f["lits"]
    rd_seed = json.load(open(os.path.join(GOLDEN, "manifest.json")))["rd_seed"]
    A0, _ = o.refrng_init(rd_seed, n)
    np.testing.assert_array_equal(A0, f["A"][0], err_msg="initial fill")
    its = f["A"].shape[0]
    st, A, rows = o.solve_refrng(n, offs, lits, rd_seed, max_iters=man[name].get("max_iters") or its + 5, trace=True)
    assert len(rows) >= its - 1
    for i in range(its - 1):
        np.testing.assert_array_equal(rows[i][4], f["A"][i + 1], err_msg=f"A after iteration {i + 1}")
        assert rows[i][3] == int(f["dres"][i])
    np.testing.assert_array_equal(A, f["A_final"])
    assert [st["n_iterations"], st["n_resamples"], st["avg_mis_size"]] == [int(x) for x in f["stats"]]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "stream_*.npz"))),
                         ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reference_rng_reproduces_reference_stream(path, oracle_mod):
    """The streaming overload (one thread) in the reference-RNG mode (orc_solve_stream_refrng)
    reproduces the reference's streaming runs (ref_probe `stream`, rd_seed 7): every iteration's
    assignment, the statistics, and the real solve(getEnumeratedClause, ...)'s result."""
    o = oracle_mod
    f = load(path)
    n, offs, lits, bs = int(f["n_vars"]), f["offs"], f["lits"], int(f["batch"])
    rd = json.load(open(os.path.join(GOLDEN, "manifest.json")))["rd_seed"]
    its = f["A"].shape[0]
    st, A, rows = o.solve_stream_refrng(n, offs, lits, rd, bs, max_iters=its + 5, trace=True)
    assert len(rows) >= its - 1
    for i in range(its - 1):
        np.testing.assert_array_equal(rows[i][4], f["A"][i + 1], err_msg=f"A after iteration {i + 1}")
    np.testing.assert_array_equal(A, f["solve_A"])
    assert [st["n_iterations"], st["n_resamples"], st["avg_mis_size"]] == [int(x) for x in f["solve_stats"]]
