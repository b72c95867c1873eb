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

FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


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
