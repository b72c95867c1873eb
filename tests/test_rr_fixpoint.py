"""The round-robin MIS (SATInstance.h:414-447, T > 1 sets) as a fixpoint of LFMIS passes
(DESIGN.md §4.3.2), restated in numpy and checked against the oracle's orc_rr_mis -- the
formulation the GPU's k_fp_* kernels implement:

  * turn(s, l): the step at which set s's scan passes the entries after its l-th pick, from the
    sets' pick counts alone (phases of fixed cyclic order between erasures; the set that moves
    into an erased set's index loses that cycle's turn);
  * P = LFMIS under the priority (turn(s, level_P(x)), clause order), iterated from an even
    guess until a pass reproduces its input.
"""
import numpy as np
import pytest


def schedule(n):
    """n[s] = picks of set s -> per set the phase records (first level, first step, stride,
    offset); turn(s, l) = step0 + (l - l0) * stride + offset in the last record with l0 <= l."""
    T = len(n)
    live, done, t, step = list(range(T)), [0] * T, 0, 0
    segs = [[] for _ in range(T)]
    while live:
        L = len(live)
        offs = [(i - t - 1) % L for i in range(L)]
        key, istar = min(((n[s] - done[s]) * L + offs[i], i) for i, s in enumerate(live))
        E = step + key
        for i, s in enumerate(live):
            segs[s].append((done[s], step, L, offs[i]))
            done[s] += n[s] - done[s] if i == istar else max(0, -(-(E - step - offs[i]) // L))
        live.pop(istar)
        t, step = istar, E + 1
    return segs


def turn_of(segs_s, level):
    rec = [g for g in segs_s if g[0] <= level][-1]
    return rec[1] + (level - rec[0]) * rec[2] + rec[3]


def lfmis(V, key):
    used, P = set(), np.zeros(len(key), bool)
    for i in np.argsort(key, kind="stable"):
        if not used.intersection(V[i]):
            P[i] = True
            used.update(V[i])
    return P


def rr_fixpoint(V, setof, T, density=0.45, max_passes=200):
    u = len(setof)
    pos = np.arange(u) - np.searchsorted(setof, np.arange(T))[setof]
    P = np.floor((pos + 1) * density) > np.floor(pos * density)
    for passes in range(max_passes):
        lev, n = np.zeros(u, np.int64), [0] * T
        for i in range(u):
            lev[i] = n[setof[i]]
            n[setof[i]] += int(P[i])
        segs = schedule(n)
        turn = np.array([turn_of(segs[setof[i]], lev[i]) for i in range(u)], np.int64)
        key = turn * (u + 1) + np.arange(u)
        Pn = lfmis(V, key)
        if passes > 0 and (Pn == P).all():
            return np.nonzero(P)[0][np.argsort(key[P])], passes
        P = Pn
    raise AssertionError("no fixpoint")


@pytest.mark.parametrize("seed", range(6))
def test_rr_fixpoint_matches_oracle(oracle_mod, seed):
    O = oracle_mod
    rng = np.random.default_rng(seed)
    for case in range(12):
        n_vars = int(rng.integers(4, 60)) if case % 2 else int(rng.integers(5, 3000))
        m, k, T = int(rng.integers(1, 2500)), int(rng.integers(1, 5)), int(rng.integers(2, 120))
        offs, lits = O.generate_ksat(int(rng.integers(1, 1 << 30)), n_vars, m, k)
        A = O.init_assignment(int(rng.integers(1, 1000)), n_vars)
        _, vm = O.eval_mask(offs, lits, A)
        U = O.mask_to_list(m, vm)
        if U.size == 0:
            continue
        cs = O.chunk_bounds(m, T)
        ref = O.rr_mis(n_vars, offs, lits, U, T, cs)
        V = [set(int(lits[j]) >> 1 for j in range(int(offs[c]), int(offs[c + 1]))) for c in U]
        setof = np.searchsorted(cs, U.astype(np.uint64), side="right") - 1
        got, _ = rr_fixpoint(V, setof, T)
        np.testing.assert_array_equal(U[got], ref, err_msg=f"seed {seed} case {case} T {T}")
