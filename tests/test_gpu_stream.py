"""Streaming solve with T > 1 threads on the GPU (SATInstance::solve(getEnumeratedClause, n, batch),
reference SATInstance.h:70-153), through the C-ABI.

Two anchors:
  * the reference's own runs (tests/golden/streamrr_*.npz, ref_probe `stream-rr`): the GPU is set
    to the fixture's A_i before each iteration, so its generators follow the fixture's (fresh at
    iteration 0, then where the lock-step check of A_i stops) -- the MIS of every iteration, the
    MIS-size statistic of its batch steps and delta n_resamples equal the reference's;
  * the oracle's streaming solve (orc_solve_stream_rr, pinned to the same fixtures by
    tests/test_oracle.py): whole trajectories with the Philox RNG, assignment after every
    iteration and the final statistics, bit-exact.
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

STREAM_RR_FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "streamrr_*.npz")))


@pytest.fixture(scope="module")
def gpu(native):
    from alllsatisfiabilitysolver_amd import device_count

    if device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return True


def load(path):
    return dict(np.load(path, allow_pickle=False))


@pytest.mark.parametrize("path", STREAM_RR_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_stream_rr_reference_maps_on_gpu(gpu, path):
    from alllsatisfiabilitysolver_amd import Solver

    f = load(path)
    n, offs, lits, bs, T = int(f["n_vars"]), f["offs"], f["lits"], int(f["batch"]), int(f["T"])
    n_it = f["A"].shape[0]
    step0 = 0
    with Solver(n, offs, lits, seed=5, stream_batch=bs, n_threads=T) as s:
        for i in range(n_it):
            s.set_assignment_words(f["A"][i])
            before = s.stats()
            s.run(1)
            after = s.stats()
            M_ref = f["M"][int(f["M_ptr"][i]):int(f["M_ptr"][i + 1])]
            np.testing.assert_array_equal(s.mis(), np.sort(M_ref), err_msg=f"M_{i}")
            ns = int(f["nsteps"][i])
            assert after["sum_mis_size"] - before["sum_mis_size"] == int(f["cum"][step0:step0 + ns].sum()), i
            assert after["n_resamples"] - before["n_resamples"] == int(f["dres"][i]), i
            step0 += ns


# (n, m, k or (w_min, w_max), kind, batch, T): several tiles, ragged last batches, both generator
# sizes (m % T != 0 with coprime walks per generator: long iterations past the materialised steps),
# power-law, 8-SAT, clauses wider than the 8 inline variables, more threads than clauses
STREAM_RR_CASES = {
    "u3_T2_b1": (200, 400, 3, 0, 1, 2),
    "u3_T2_b64": (2000, 4000, 3, 0, 64, 2),
    "u3_T4_b37": (2000, 4000, 3, 0, 37, 4),
    "u3_T4_b5000": (30000, 60000, 3, 0, 5000, 4),
    "u3_T3_b133_coprime": (300, 800, 3, 0, 133, 3),
    "u3_T7_b57_coprime": (300, 800, 3, 0, 57, 7),
    "u3_T16_b1000": (20000, 40000, 3, 0, 1000, 16),
    "pl3_T4_b256": (4000, 12000, 3, 1, 256, 4),
    "k8_T4_b500": (4000, 6000, 8, 0, 500, 4),
    "mixed_T3_b40": (600, 900, (1, 12), 0, 40, 3),
    "tiny_T32_b2": (40, 30, 3, 0, 2, 32),
    # k_srr_mis's large-T paths: more sets than candidate slots (512: the sets past them wait
    # for the next gather), more sets than threads, wide clauses among many sets
    "u3_T600_b20": (20000, 60000, 3, 0, 20, 600),
    "u3_T1100_b7": (20000, 55000, 3, 0, 7, 1100),
    "mixed_T40_b30": (3000, 6000, (1, 12), 0, 30, 40),
    "k8_T700_b3": (4000, 5600, 8, 0, 3, 700),
}


def _instance(n, m, k, kind):
    from alllsatisfiabilitysolver_amd import generate_ksat, generate_mixed

    if isinstance(k, tuple):
        return generate_mixed(3, n, m, k[0], k[1])
    return generate_ksat(2, n, m, k, kind)


@pytest.mark.parametrize("name", list(STREAM_RR_CASES))
def test_stream_rr_trajectory_matches_oracle(gpu, oracle_mod, name):
    from alllsatisfiabilitysolver_amd import Solver

    n, m, k, kind, bs, T = STREAM_RR_CASES[name]
    offs, lits = _instance(n, m, k, kind)
    seed = 41
    rc, st_o, A_o, rows = oracle_mod.solve_stream_rr(n, offs, lits, seed, bs, T, max_iters=400, trace=True)
    assert rc in (0, 1)
    with Solver(n, offs, lits, seed=seed, stream_batch=bs, n_threads=T) as s:
        assert s.uses_graphs()[0] is False
        for it, nu, nm, dres, A_after in rows[:60]:
            before = s.stats()
            s.run(1)
            after = s.stats()
            assert after["n_violated"] == nu, f"iter {it}"
            assert after["n_resamples"] - before["n_resamples"] == dres, f"iter {it}"
            assert s.mis().size == nm, f"iter {it}"
            np.testing.assert_array_equal(s.assignment_words(), A_after, err_msg=f"A after iter {it}")
    with Solver(n, offs, lits, seed=seed, stream_batch=bs, n_threads=T, max_iters=400) as s:
        st = s.solve()
        for key in ("n_iterations", "n_resamples", "avg_mis_size", "sum_mis_size", "solved"):
            assert st[key] == st_o[key], key
        np.testing.assert_array_equal(s.assignment_words(), A_o)
        ok, nv = s.verify()
        assert ok == bool(st_o["solved"])


def test_stream_rr_cap_and_satisfied_start(gpu, oracle_mod):
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m = 2000, 8000  # ratio 4: not solved within the cap
    offs, lits = generate_ksat(4, n, m, 3)
    rc, st_o, A_o, _ = oracle_mod.solve_stream_rr(n, offs, lits, 9, 100, 4, max_iters=6)
    assert rc == 1 and st_o["n_iterations"] == 6
    with Solver(n, offs, lits, seed=9, max_iters=6, stream_batch=100, n_threads=4) as s:
        st = s.solve()
        for key in ("n_iterations", "n_resamples", "avg_mis_size", "solved"):
            assert st[key] == st_o[key], key
        np.testing.assert_array_equal(s.assignment_words(), A_o)
    # one clause, satisfied by the initial assignment: one iteration, nothing resampled
    A0 = oracle_mod.init_assignment(2, 4)
    lit = np.array([0 if (A0[0] & 1) else 1], np.uint32)
    with Solver(4, np.array([0, 1], np.uint64), lit, seed=2, stream_batch=8, n_threads=3) as s:
        st = s.solve()
        assert (st["n_iterations"], st["n_resamples"], st["avg_mis_size"], st["solved"]) == (1, 0, 0, 1)


def test_stream_rr_refusals(gpu, oracle_mod):
    """Where the reference would not return: an empty clause (violated forever), generators that
    never finish at the same batch step.  Also world > 1 (one GPU only).  No silent fallback."""
    import alllsatisfiabilitysolver_amd._native as N
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    offs, lits = oracle_mod.csr_from_lists([[0, 2], [], [4]])
    with pytest.raises(N.AlllError) as e:
        Solver(3, offs, lits, seed=1, stream_batch=1, n_threads=2)
    assert e.value.code == N.ALLL_ERR_UNSUPPORTED
    offs, lits = generate_ksat(3, 300, 800, 3)
    with pytest.raises(N.AlllError) as e:
        Solver(300, offs, lits, seed=1, stream_batch=4, n_threads=2, world=2, rank=0)
    assert e.value.code == N.ALLL_ERR_UNSUPPORTED
    offs, lits = oracle_mod.generate_ksat(3, 300, 800, 3)
    assert oracle_mod.solve_stream_rr(300, offs, lits, 20, 9, 3, step_cap=10000)[0] == -1
    with Solver(300, offs, lits, seed=20, stream_batch=9, n_threads=3) as s:
        with pytest.raises(N.AlllError) as e:
            s.solve()
        assert e.value.code == N.ALLL_ERR_UNSUPPORTED and "never finish" in str(e.value)
    # ALLL_FLAG_LFMIS keeps the one-thread order for any n_threads
    offs, lits = oracle_mod.generate_ksat(3, 300, 600, 3)
    st_o, A_o, _ = oracle_mod.solve_stream(300, offs, lits, 7, 50)
    with Solver(300, offs, lits, seed=7, stream_batch=50, n_threads=4, flags=N.FLAG_LFMIS) as s:
        st = s.solve()
        assert st["n_iterations"] == st_o["n_iterations"]
        np.testing.assert_array_equal(s.assignment_words(), A_o)


def test_python_satinstance_stream_overload(gpu, oracle_mod):
    """The Python mirror's solve(getEnumeratedClause, n_clauses, batch_size) (SATInstance.h:70-153)
    with n_threads = 4 equals the oracle's streaming solve."""
    from alllsatisfiabilitysolver_amd import generate_ksat
    from alllsatisfiabilitysolver_amd.solver import Clause, SATInstance, VariablesArray

    n, m, bs, T = 400, 800, 25, 4
    offs, lits = generate_ksat(6, n, m, 3)
    seen = set()

    def gen(i, t_id):
        seen.add((i, t_id))
        return Clause(lits[int(offs[i]):int(offs[i + 1])].tolist(), t_id)

    va = VariablesArray(n)
    S = SATInstance(va, T, seed=13)
    st = S.solve(gen, m, bs)
    assert {t for i, t in seen if i < m // T} == {0} and {t for i, t in seen if i >= 3 * (m // T)} == {T - 1}
    rc, st_o, A_o, _ = oracle_mod.solve_stream_rr(n, offs, lits, 13, bs, T)
    assert rc == 0
    assert (st.n_iterations, st.n_resamples, st.avg_mis_size) == (
        st_o["n_iterations"], st_o["n_resamples"], st_o["avg_mis_size"])
    np.testing.assert_array_equal(oracle_mod.pack_bools(va.vars.astype(np.uint8)), A_o)
