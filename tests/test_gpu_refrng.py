"""The reference-RNG mode on the GPU (ALLL_FLAG_REFERENCE_RNG, alll_refrng.hip):
with the reference's own random stream -- RBG<default_random_engine> over libstdc++'s
minstd_rand0 and uniform_int_distribution<unsigned long long>, each engine seeded by the next
std::random_device value, whose stand-in (oracle/ref_probe.cpp) has state `seed` -- the GPU's
whole T = 1 trajectory equals the reference's, bit for bit.

Two anchors:
  * the reference's own runs (tests/golden/*_T1.npz, ref_probe `trace` with rd_seed 7): the
    initial VariablesArray fill, the assignment after every iteration, the final statistics;
  * the oracle's restatement (orc_solve_refrng, pinned to the same fixtures by
    tests/test_oracle.py) on larger instances, up to the bench instance M.
"""
import glob
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

REF_FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "*_T1.npz")))
RD_SEED = json.load(open(os.path.join(GOLDEN, "manifest.json")))["rd_seed"]
MANIFEST = {d["fixture"]: d for d in json.load(open(os.path.join(GOLDEN, "manifest.json")))["fixtures"]}


@pytest.fixture(scope="module")
def gpu(native):
    from alllsatisfiabilitysolver_amd import device_count

    if device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return True


def load(path):
    return dict(np.load(path, allow_pickle=False))


LAYOUTS = {"default": 0, "csr": "GENERIC_CSR", "no_ranged": "NO_RANGED", "atomic": "ATOMIC_CLAIMS"}


def _flags(native, layout):
    f = native.FLAG_REFERENCE_RNG
    if LAYOUTS[layout]:
        f |= getattr(native, "FLAG_" + LAYOUTS[layout])
    return f


@pytest.mark.parametrize("layout", list(LAYOUTS))
@pytest.mark.parametrize("path", REF_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_reference_trajectory_on_gpu(gpu, native, path, layout):
    from alllsatisfiabilitysolver_amd import Solver

    f = load(path)
    name = os.path.basename(path)[:-4]
    n, offs, lits = int(f["n_vars"]), f["offs"], f["lits"]
    its = f["A"].shape[0]
    flags = _flags(native, layout)
    with Solver(n, offs, lits, seed=RD_SEED, flags=flags) as s:
        np.testing.assert_array_equal(s.assignment_words(), f["A"][0], err_msg="initial fill")
        for i in range(its - 1):
            before = s.stats()
            s.run(1)
            after = s.stats()
            np.testing.assert_array_equal(s.assignment_words(), f["A"][i + 1], err_msg=f"A after iteration {i + 1}")
            assert after["n_resamples"] - before["n_resamples"] == int(f["dres"][i]), i
    mi = MANIFEST[name].get("max_iters") or 0
    with Solver(n, offs, lits, seed=RD_SEED, flags=flags, max_iters=mi) as s:
        st = s.solve()
        np.testing.assert_array_equal(s.assignment_words(), f["A_final"])
        assert [st["n_iterations"], st["n_resamples"], st["avg_mis_size"]] == [int(x) for x in f["stats"]]


REFRNG_CASES = {
    # name: (n, m, k, kind, rd_seed, iterations)
    "u3_20k": (20000, 80000, 3, 0, 11, 12),
    "pl3_40k": (40000, 160000, 3, 1, 12, 12),
    "k5_30k": (30000, 60000, 5, 0, 13, 8),
    "mixed_2_12": (8000, 20000, (2, 12), 0, 14, 10),
    "C2": (1_000_000, 4_000_000, 3, 0, 15, 3),
    "M": (2_500_000, 10_000_000, 3, 0, 16, 3),
}


def _instance(n, m, k, kind):
    from alllsatisfiabilitysolver_amd import generate_ksat, generate_mixed

    if isinstance(k, tuple):
        return generate_mixed(3, n, m, k[0], k[1])
    return generate_ksat(1, n, m, k, kind)


@pytest.mark.parametrize("name", list(REFRNG_CASES))
def test_reference_rng_matches_oracle(gpu, native, oracle_mod, name):
    from alllsatisfiabilitysolver_amd import Solver

    n, m, k, kind, rd, iters = REFRNG_CASES[name]
    offs, lits = _instance(n, m, k, kind)
    A0, _ = oracle_mod.refrng_init(rd, n)
    st_o, A_o, rows = oracle_mod.solve_refrng(n, offs, lits, rd, max_iters=iters + 1, trace=True)
    with Solver(n, offs, lits, seed=rd, flags=native.FLAG_REFERENCE_RNG) as s:
        np.testing.assert_array_equal(s.assignment_words(), A0, err_msg="initial fill")
        for it, nu, nm, dres, A_after in rows:
            before = s.stats()
            s.run(1)
            after = s.stats()
            assert after["n_violated"] == nu, it
            assert after["n_resamples"] - before["n_resamples"] == dres, it
            np.testing.assert_array_equal(s.assignment_words(), A_after, err_msg=f"A after iteration {it}")
    # the captured multi-iteration graphs replay the same rounds
    with Solver(n, offs, lits, seed=rd, flags=native.FLAG_REFERENCE_RNG, max_iters=iters + 1) as s:
        st = s.solve()
        np.testing.assert_array_equal(s.assignment_words(), A_o)
        for key in ("n_iterations", "n_resamples", "avg_mis_size", "solved"):
            assert st[key] == st_o[key], key


STREAM_FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "stream_*.npz")))


@pytest.mark.parametrize("path", STREAM_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_reference_stream_trajectory_on_gpu(gpu, native, path):
    """The streaming overload (one thread) with the reference's own stream: the reference's runs
    (ref_probe `stream`, rd_seed 7) -- every iteration's assignment, the statistics, and the real
    solve(getEnumeratedClause, ...)'s final assignment and statistics."""
    from alllsatisfiabilitysolver_amd import Solver

    f = load(path)
    n, offs, lits, bs = int(f["n_vars"]), f["offs"], f["lits"], int(f["batch"])
    its = f["A"].shape[0]
    with Solver(n, offs, lits, seed=RD_SEED, flags=native.FLAG_REFERENCE_RNG, stream_batch=bs) as s:
        np.testing.assert_array_equal(s.assignment_words(), f["A"][0], err_msg="initial fill")
        for i in range(its - 1):
            s.run(1)
            np.testing.assert_array_equal(s.assignment_words(), f["A"][i + 1], err_msg=f"A after iteration {i + 1}")
    with Solver(n, offs, lits, seed=RD_SEED, flags=native.FLAG_REFERENCE_RNG, stream_batch=bs) as s:
        st = s.solve()
        np.testing.assert_array_equal(s.assignment_words(), f["solve_A"])
        assert [st["n_iterations"], st["n_resamples"], st["avg_mis_size"]] == [int(x) for x in f["solve_stats"]]


@pytest.mark.parametrize("bs", [1000, 40000])
def test_reference_rng_stream_matches_oracle(gpu, native, oracle_mod, bs):
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m, rd = 20000, 80000, 21
    offs, lits = generate_ksat(1, n, m, 3, 0)
    st_o, A_o, rows = oracle_mod.solve_stream_refrng(n, offs, lits, rd, bs, max_iters=12, trace=True)
    with Solver(n, offs, lits, seed=rd, flags=native.FLAG_REFERENCE_RNG, stream_batch=bs) as s:
        for it, nu, nm, dres, A_after in rows:
            s.run(1)
            np.testing.assert_array_equal(s.assignment_words(), A_after, err_msg=f"A after iteration {it}")
    with Solver(n, offs, lits, seed=rd, flags=native.FLAG_REFERENCE_RNG, stream_batch=bs, max_iters=12) as s:
        st = s.solve()
        np.testing.assert_array_equal(s.assignment_words(), A_o)
        for key in ("n_iterations", "n_resamples", "avg_mis_size", "solved"):
            assert st[key] == st_o[key], key


def test_reference_rng_sequential_fallback(gpu, native, oracle_mod, monkeypatch):
    """ALLL_RRNG_NMAX caps the engine positions the parallel draws consider, so every round runs
    past them and the one-thread chain (k_rrng_seq) redoes it: the same trajectory."""
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m, rd = 20000, 80000, 23
    offs, lits = generate_ksat(1, n, m, 3, 0)
    st_o, A_o, rows = oracle_mod.solve_refrng(n, offs, lits, rd, max_iters=6, trace=True)
    monkeypatch.setenv("ALLL_RRNG_NMAX", "40")
    with Solver(n, offs, lits, seed=rd, flags=native.FLAG_REFERENCE_RNG) as s:
        for it, nu, nm, dres, A_after in rows:
            s.run(1)
            np.testing.assert_array_equal(s.assignment_words(), A_after, err_msg=f"A after iteration {it}")


def test_reference_rng_refusals(gpu, native):
    from alllsatisfiabilitysolver_amd import AlllError, Solver, generate_ksat

    offs, lits = generate_ksat(1, 200, 800, 3, 0)
    for kw in (dict(n_threads=2), dict(n_threads=2, stream_batch=64)):
        with pytest.raises(AlllError) as ei:
            Solver(200, offs, lits, seed=1, flags=native.FLAG_REFERENCE_RNG, **kw)
        assert ei.value.code == native.ALLL_ERR_UNSUPPORTED, kw
