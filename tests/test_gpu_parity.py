"""GPU parity: the HIP path through the C-ABI against the reference golden vectors and the
oracle (CPU restatement of the serial path), bit-exact.

  * reference maps on the GPU: for every T=1 golden trajectory, the device evaluates
    A_i -> U_i and picks M_i exactly as the reference did (SATInstance.h:264-280, 391-451);
  * full trajectories with Philox vs the oracle: assignment after every iteration,
    violated count, MIS, final Statistics (SATInstance.h:25-32, 313-317);
  * BASELINE sizes (10M clauses 3-SAT, 8-SAT 6M, power-law 10M): per-iteration bit-exact
    steps against the oracle for a few iterations;
  * edge cases: empty instance, empty clause (never solvable -> max_iters), tautologies,
    duplicate variables, unit / wide clauses, max_iters cap semantics.
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

T1_FIXTURES = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*_T1.npz")))
# name -> (flags, environment at create): the default policy picks the bucketed LFMIS round 0
# only for large violated sets, "buckets" forces it for every iteration
LAYOUTS = {"hybrid": (0, {}), "fixed": (1 << 3, {}), "csr": (1 << 2, {}), "atomic_claims": (1 << 5, {}),
           "buckets": (0, {"ALLL_BUCKET_MIN_U": "0"}), "windows": (0, {"ALLL_EVAL_WINDOWS": "1"}),
           "positions": (0, {"ALLL_PACKED_IDS": "0"}),
           # bucketed round 0 scattered by its own kernel k_bscatter (the default fuses the
           # scatter into the evaluation workgroups, k_eval_scatter)
           "bscatter": (0, {"ALLL_FUSE_SCATTER": "0", "ALLL_BUCKET_MIN_U": "0"}),
           # the large-instance evaluation (non-temporal literal loads, exec-masked L2 lookups)
           # with windows
           "nt_windows": (0, {"ALLL_EVAL_NT": "1", "ALLL_EVAL_WINDOWS": "1"}),
           # one grid round + the tail in every iteration after the first (variant 2), and never
           "tail_all": (0, {"ALLL_SMALL_U": str(1 << 62)}), "no_small_u": (0, {"ALLL_SMALL_U": "0"}),
           # many small LDS windows (64 words: 2048 variables; the C4 layout on small instances),
           # with the cached and with the non-temporal (C4) evaluation
           "small_windows": (0, {"ALLL_EVAL_WINDOWS": "1", "ALLL_WIN_WORDS": "64"}),
           "small_windows_nt": (0, {"ALLL_EVAL_WINDOWS": "1", "ALLL_WIN_WORDS": "64", "ALLL_EVAL_NT": "1"})}


def make_solver(layout, monkeypatch, *args, **kw):
    from alllsatisfiabilitysolver_amd import Solver

    flags, env = LAYOUTS[layout]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    s = Solver(*args, flags=flags, **kw)
    for k in env:
        monkeypatch.delenv(k)
    return s


@pytest.fixture(scope="module")
def gpu(native):
    from alllsatisfiabilitysolver_amd import device_count

    if device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return True


def mask_to_list(vm, m):
    bits = np.unpackbits(vm.view(np.uint8), bitorder="little")[:m]
    return np.nonzero(bits)[0].astype(np.uint32)


@pytest.mark.parametrize("layout", list(LAYOUTS))
@pytest.mark.parametrize("path", T1_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_reference_maps_on_gpu(gpu, path, layout, monkeypatch):
    f = dict(np.load(path, allow_pickle=False))
    n, offs, lits = int(f["n_vars"]), f["offs"], f["lits"]
    m = offs.size - 1
    with make_solver(layout, monkeypatch, n, offs, lits, seed=3) as s:
        for i in range(f["A"].shape[0]):
            s.set_assignment_words(f["A"][i])
            before = s.stats()
            s.run(1)
            U_ref = f["U"][int(f["U_ptr"][i]):int(f["U_ptr"][i + 1])]
            np.testing.assert_array_equal(mask_to_list(s.violated_mask(), m), U_ref, err_msg=f"U_{i}")
            after = s.stats()
            if U_ref.size == 0:
                assert after["solved"] == 1
                break
            M_ref = f["M"][int(f["M_ptr"][i]):int(f["M_ptr"][i + 1])]
            np.testing.assert_array_equal(s.mis(), np.sort(M_ref), err_msg=f"M_{i}")
            if int(f["dres"][i]):
                assert after["n_resamples"] - before["n_resamples"] == int(f["dres"][i])
            assert after["sum_mis_size"] - before["sum_mis_size"] == M_ref.size


def _instances():
    from alllsatisfiabilitysolver_amd import generate_ksat

    out = {}
    for name, (n, m, k, kind) in {
        "c1_ratio4": (200, 800, 3, 0),
        "u2500_ratio4": (2500, 10000, 3, 0),
        "ratio2_solves": (200, 400, 3, 0),
        "k8": (4000, 6000, 8, 0),
        "powerlaw": (2000, 8000, 3, 1),
        "k5_multi_tile": (30000, 60000, 5, 0),
        "powerlaw_hot": (20000, 80000, 3, 1),   # hub variables -> LDS-aggregated claims
        # the other fixed widths of the evaluation (no middle slot, one middle slot, several)
        "k1": (3000, 2000, 1, 0),
        "k2": (6000, 9000, 2, 0),
        "k4": (20000, 60000, 4, 0),
        "k7": (8000, 12000, 7, 0),
    }.items():
        out[name] = (n,) + generate_ksat(1, n, m, k, kind)
    f = dict(np.load(os.path.join(GOLDEN, "edge_T1.npz")))
    out["edge"] = (int(f["n_vars"]), f["offs"], f["lits"])
    # ragged widths across several tiles
    rng = np.random.default_rng(5)
    w = rng.integers(1, 12, 20000)
    offs = np.zeros(w.size + 1, np.uint64)
    offs[1:] = np.cumsum(w)
    lits = rng.integers(0, 2 * 9000, int(offs[-1])).astype(np.uint32)
    out["ragged"] = (9000, offs, lits)
    # ragged with a few very wide clauses (their chunks get wide) and empty clauses (always
    # violated: every slot is the padding literal)
    w = rng.integers(1, 9, 30000)
    w[rng.choice(w.size, 40, replace=False)] = rng.integers(40, 150, 40)
    w[rng.choice(w.size, 3, replace=False)] = 0
    offs = np.zeros(w.size + 1, np.uint64)
    offs[1:] = np.cumsum(w)
    lits = rng.integers(0, 2 * 12000, int(offs[-1])).astype(np.uint32)
    out["ragged_wide"] = (12000, offs, lits)
    return out


INSTANCES = None


def instances():
    global INSTANCES
    if INSTANCES is None:
        INSTANCES = _instances()
    return INSTANCES


@pytest.mark.parametrize("layout", list(LAYOUTS))
@pytest.mark.parametrize("name", ["c1_ratio4", "u2500_ratio4", "ratio2_solves", "k8", "powerlaw",
                                  "k5_multi_tile", "powerlaw_hot", "edge", "ragged", "ragged_wide",
                                  "k1", "k2", "k4", "k7"])
def test_trajectory_matches_oracle(gpu, oracle_mod, name, layout, monkeypatch):
    o = oracle_mod
    n, offs, lits = instances()[name]
    seed, K = 12345, 40
    st_o, A_o, rows = o.solve(n, offs, lits, seed, max_iters=K, trace=True)
    with make_solver(layout, monkeypatch, n, offs, lits, seed=seed) as s:
        np.testing.assert_array_equal(s.assignment_words(), o.init_assignment(seed, n))
        for it, nu, nm, dres, A_after in rows:
            before = s.stats()
            s.run(1)
            after = s.stats()
            assert after["n_violated"] == nu, f"iter {it}"
            assert after["sum_mis_size"] - before["sum_mis_size"] == nm, f"iter {it}"
            assert after["n_resamples"] - before["n_resamples"] == dres, f"iter {it}"
            np.testing.assert_array_equal(s.assignment_words(), A_after, err_msg=f"A after iter {it}")
    # whole solve with the same cap: identical Statistics and assignment
    with make_solver(layout, monkeypatch, n, offs, lits, seed=seed, max_iters=K) as s:
        st = s.solve()
        for k in ("n_iterations", "n_resamples", "avg_mis_size", "sum_mis_size", "solved"):
            assert st[k] == st_o[k], k
        np.testing.assert_array_equal(s.assignment_words(), A_o)


@pytest.mark.parametrize("layout", ["hybrid", "csr", "buckets", "positions"])
def test_long_run_across_cover_stamp_cycles(gpu, oracle_mod, layout, monkeypatch):
    """Cover marks are 8-bit stamps cycling through 1..255 (cleared at every wrap): a 600-
    iteration run crosses two wraps and stays bit-exact (checkpoints around each wrap)."""
    n, offs, lits = instances()["u2500_ratio4"]
    seed, K = 7, 600
    st_o, A_o, rows = oracle_mod.solve(n, offs, lits, seed, max_iters=K, trace=True)
    assert st_o["solved"] == 0 and len(rows) >= K - 1
    with make_solver(layout, monkeypatch, n, offs, lits, seed=seed) as s:
        done = 0
        for stop in (250, 254, 255, 256, 257, 509, 510, 511, 512, 599):
            s.run(stop - done)
            done = stop
            np.testing.assert_array_equal(s.assignment_words(), rows[stop - 1][4], err_msg=f"A after {stop}")
    with make_solver(layout, monkeypatch, n, offs, lits, seed=seed, max_iters=K) as s:
        st = s.solve()
        for k in ("n_iterations", "n_resamples", "avg_mis_size", "sum_mis_size", "solved"):
            assert st[k] == st_o[k], k
        np.testing.assert_array_equal(s.assignment_words(), A_o)


@pytest.mark.parametrize("m", [4096, 4097])
def test_packed_id_boundary(gpu, oracle_mod, m):
    """k = 2 over 2^24 variables: literals need 25 bits, leaving 6 id bits per slot.  4096
    clauses (12-bit ids) are packed exactly at the limit; 4097 (13 bits) fall back to
    evaluation positions translated through perm.  Both are bit-exact."""
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n = 1 << 24
    offs, lits = generate_ksat(3, n, m, 2, 0)
    seed, K = 9, 12
    _, A_o, rows = oracle_mod.solve(n, offs, lits, seed, max_iters=K, trace=True)
    with Solver(n, offs, lits, seed=seed) as s:
        for it, nu, nm, dres, A_after in rows:
            before = s.stats()
            s.run(1)
            after = s.stats()
            assert after["n_violated"] == nu, f"iter {it}"
            assert after["sum_mis_size"] - before["sum_mis_size"] == nm, f"iter {it}"
            np.testing.assert_array_equal(s.assignment_words(), A_after, err_msg=f"A after iter {it}")


def test_solve_converges_and_verifies(gpu, oracle_mod):
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m = 25000, 50000  # ratio 2: converges in ~100 iterations
    offs, lits = generate_ksat(2, n, m, 3)
    st_o, A_o, _ = oracle_mod.solve(n, offs, lits, 99)
    assert st_o["solved"] == 1
    with Solver(n, offs, lits, seed=99) as s:
        st = s.solve()
        assert st["solved"] == 1
        for k in ("n_iterations", "n_resamples", "avg_mis_size"):
            assert st[k] == st_o[k]
        np.testing.assert_array_equal(s.assignment_words(), A_o)
        ok, nv = s.verify()
        assert ok and nv == 0
        nu, _ = oracle_mod.eval_mask(offs, lits, s.assignment_words())
        assert nu == 0


def test_max_iters_and_unsolvable(gpu, oracle_mod):
    from alllsatisfiabilitysolver_amd import Solver

    # empty clause: always violated (reference loops forever; here max_iters ends it)
    offs = np.array([0, 2, 2, 3], np.uint64)
    lits = np.array([0, 3, 4], np.uint32)
    st_o, A_o, _ = oracle_mod.solve(3, offs, lits, 5, max_iters=9)
    with Solver(3, offs, lits, seed=5, max_iters=9) as s:
        st = s.solve()
        assert st["solved"] == 0 and st["n_iterations"] == 9
        for k in ("n_iterations", "n_resamples", "avg_mis_size"):
            assert st[k] == st_o[k]
        ok, nv = s.verify()
        assert not ok and nv >= 1


def test_empty_instance(gpu):
    from alllsatisfiabilitysolver_amd import Solver

    with Solver(10, np.zeros(1, np.uint64), np.zeros(0, np.uint32), seed=1) as s:
        st = s.solve()
        assert st["solved"] == 1 and st["n_iterations"] == 1 and st["n_resamples"] == 0


@pytest.mark.parametrize("grid_rounds", [1, 2, 3, 8])
def test_grid_round_split_is_invisible(gpu, oracle_mod, grid_rounds, monkeypatch):
    """The split between full-grid LFMIS rounds and the single-workgroup tail changes
    nothing: same trajectory as the oracle."""
    from alllsatisfiabilitysolver_amd import Solver

    n, offs, lits = instances()["k5_multi_tile"]
    st_o, A_o, rows = oracle_mod.solve(n, offs, lits, 77, max_iters=12, trace=True)
    monkeypatch.setenv("ALLL_BUCKET_MIN_U", "0")  # round 0 bucketed (incl. last-round hand-off at G=1)
    with Solver(n, offs, lits, seed=77, max_iters=12, grid_rounds=grid_rounds) as s:
        st = s.solve()
        assert st["n_resamples"] == st_o["n_resamples"]
        np.testing.assert_array_equal(s.assignment_words(), A_o)


@pytest.mark.parametrize("bucket_min_u", ["0", str(1 << 62)])
def test_fused_reduce_is_invisible(gpu, oracle_mod, bucket_min_u, monkeypatch):
    """The loop's reduce runs in an extra workgroup of the bucketed round 0 or as its own kernel
    (atomic round 0): same trajectory, statistics, stop and cap as the oracle."""
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n = 20000
    offs, lits = generate_ksat(3, n, 2 * n, 3, 0)  # ratio 2 over 10 tiles: converges
    st_o, A_o, rows = oracle_mod.solve(n, offs, lits, 5, max_iters=400, trace=True)
    assert st_o["solved"] == 1
    monkeypatch.setenv("ALLL_BUCKET_MIN_U", bucket_min_u)  # bucketed round 0 in every iteration, or never
    with Solver(n, offs, lits, seed=5, max_iters=400) as s:
        for it, nu, nm, dres, A_after in rows[:6]:
            s.run(1)
            assert s.stats()["n_violated"] == nu
            np.testing.assert_array_equal(s.assignment_words(), A_after)
        st = s.solve()
        for key in ("n_iterations", "n_resamples", "avg_mis_size", "solved"):
            assert st[key] == st_o[key], key
        np.testing.assert_array_equal(s.assignment_words(), A_o)
    # a cap that stops before convergence: the final pass evaluates without resampling
    st_c, A_c, _ = oracle_mod.solve(n, offs, lits, 5, max_iters=7, trace=True)
    with Solver(n, offs, lits, seed=5, max_iters=7) as s:
        st = s.solve()
        for key in ("n_iterations", "n_resamples", "avg_mis_size", "solved"):
            assert st[key] == st_c[key], key
        np.testing.assert_array_equal(s.assignment_words(), A_c)


def _oracle_step(o, n, offs, lits, A, seed, it):
    """One serial iteration (eval -> LFMIS -> Philox resample) on the CPU."""
    m = offs.size - 1
    nu, vm = o.eval_mask(offs, lits, A)
    U = o.mask_to_list(m, vm)
    M = o.lfmis(n, offs, lits, U)
    A2 = o.resample_words(A.copy(), seed, it, o.clause_vars(offs, lits, M))
    return nu, vm, M, A2


BIG = {
    "M_3sat_10M": (2_500_000, 10_000_000, 3, 0),
    "C2_3sat_4M": (1_000_000, 4_000_000, 3, 0),
    "C3_8sat_6M": (4_000_000, 6_000_000, 8, 0),
    "C5_powerlaw_10M": (2_500_000, 10_000_000, 3, 1),
    # power-law with the atomic round 0 (the default policy buckets it while |U| is large)
    "C5_atomic_round0": (2_500_000, 10_000_000, 3, 1, {"ALLL_BUCKET_MIN_U": str(1 << 62)}),
    "C5_bscatter": (2_500_000, 10_000_000, 3, 1, {"ALLL_FUSE_SCATTER": "0"}),
    "M_bscatter": (2_500_000, 10_000_000, 3, 0, {"ALLL_FUSE_SCATTER": "0"}),
    "W_3sat_4Mvars": (4_000_000, 2_000_000, 3, 0),  # 4 LDS blocks of variables: windowed eval
    "M_no_windows": (2_500_000, 10_000_000, 3, 0, {"ALLL_EVAL_WINDOWS": "0"}),
    "M_positions": (2_500_000, 10_000_000, 3, 0, {"ALLL_PACKED_IDS": "0"}),  # perm translation
    # C4 (the north star's 8-GPU instance) on one GPU: 27-bit clause ids do not fit in the
    # literals' spare bits (26-bit literals), so evaluation positions + perm; 26 LDS windows
    "C4_3sat_128M": (32_000_000, 128_000_000, 3, 0),
    # M through the large-instance evaluation variant (C4 takes it by default)
    "M_nt": (2_500_000, 10_000_000, 3, 0, {"ALLL_EVAL_NT": "1"}),
    # ragged widths 2-12 (bench config R): the chunk-transposed ragged evaluation, CSR LFMIS
    "R_mixed_4M": (1_000_000, 4_000_000, (2, 12), 0),
    # more variables than one LDS window: windowed ragged evaluation
    "R_mixed_windows": (4_000_000, 2_000_000, (1, 9), 0),
}


@pytest.mark.slow
@pytest.mark.parametrize("name", list(BIG))
def test_baseline_sizes_bit_exact_steps(gpu, oracle_mod, name, monkeypatch):
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m, k, kind = BIG[name][:4]
    for key, v in (BIG[name][4] if len(BIG[name]) > 4 else {}).items():
        monkeypatch.setenv(key, v)
    if isinstance(k, tuple):
        from alllsatisfiabilitysolver_amd import generate_mixed

        offs, lits = generate_mixed(1, n, m, *k)
    else:
        offs, lits = generate_ksat(1, n, m, k, kind)
    seed = 1
    with Solver(n, offs, lits, seed=seed) as s:
        A = s.assignment_words()
        np.testing.assert_array_equal(A, oracle_mod.init_assignment(seed, n))
        for it in range(2):
            nu, vm, M, A_next = _oracle_step(oracle_mod, n, offs, lits, A, seed, it)
            before = s.stats()
            s.run(1)
            after = s.stats()
            assert after["n_violated"] == nu
            np.testing.assert_array_equal(s.violated_mask(), vm[: (m + 63) // 64])
            np.testing.assert_array_equal(s.mis(), M)
            assert after["sum_mis_size"] - before["sum_mis_size"] == M.size
            A = s.assignment_words()
            np.testing.assert_array_equal(A, A_next)
        # size-independent properties on the device path
        ok, nv = s.verify()
        assert nv == oracle_mod.eval_mask(offs, lits, A)[0]


@pytest.mark.slow
@pytest.mark.parametrize("name", ["C2_3sat_4M", "M_3sat_10M", "C3_8sat_6M", "C5_powerlaw_10M", "C4_3sat_128M"])
def test_full_size_long_run_bit_exact(gpu, oracle_mod, name):
    """Every BASELINE config on the GPU at full size over 8 consecutive iterations, every one
    against the oracle's (violated count, MIS list, resampled assignment): the full-size cases
    above check 2 iterations, the bench digests only the end state of a longer run."""
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m, k, kind = BIG[name]
    offs, lits = generate_ksat(1, n, m, k, kind)
    seed = 1
    with Solver(n, offs, lits, seed=seed) as s:
        A = s.assignment_words()
        for it in range(8):
            nu, vm, M, A_next = _oracle_step(oracle_mod, n, offs, lits, A, seed, it)
            s.run(1)
            assert s.stats()["n_violated"] == nu, f"iteration {it}"
            np.testing.assert_array_equal(s.mis(), M, err_msg=f"iteration {it}")
            A = s.assignment_words()
            np.testing.assert_array_equal(A, A_next, err_msg=f"iteration {it}")


def test_bench_helpers(gpu, oracle_mod):
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m = 50000, 200000
    offs, lits = generate_ksat(1, n, m, 3)
    with Solver(n, offs, lits, seed=4) as s:
        ms, nv = s.bench_eval(5)
        assert ms > 0
        assert nv == oracle_mod.eval_mask(offs, lits, s.assignment_words())[0]
        assert s.eval_bytes() == 12 * m + (n + 7) // 8 + (m + 7) // 8
        pt = s.profile(3)
        assert pt["iterations"] == 3 and pt["eval_ms"] > 0 and pt["total_ms"] >= pt["eval_ms"]
        st = s.stats()
        assert st["n_iterations"] == 3


def test_loop_times_stamps_leave_trajectory_unchanged(gpu, oracle_mod):
    """ALLL_FLAG_KERNEL_TIMING: kernels stamp each iteration; results stay bit-exact."""
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat
    from alllsatisfiabilitysolver_amd import _native as N

    n, m = 30000, 120000
    offs, lits = generate_ksat(6, n, m, 3)
    st_o, A_o, _ = oracle_mod.solve(n, offs, lits, 21, max_iters=13, trace=True)
    for flags in (N.FLAG_KERNEL_TIMING, N.FLAG_KERNEL_TIMING | N.FLAG_NO_RANGED):
        with Solver(n, offs, lits, seed=21, flags=flags) as s:
            s.run(4)
            it0 = s.stats()["n_iterations"]
            s.run(8)
            np.testing.assert_array_equal(s.assignment_words(), oracle_mod.solve(n, offs, lits, 21, max_iters=13)[1])
            pt = s.loop_times(it0, 8)
            assert pt["iterations"] == 8
            assert 0 < pt["eval_ms"] < 50
            assert pt["mis_ms"] > 0 and pt["total_ms"] >= pt["eval_ms"] + pt["mis_ms"]
            # out-of-range requests are clipped, never read garbage
            assert s.loop_times(it0 + 8, 5)["iterations"] == 0
    with Solver(n, offs, lits, seed=21) as s:
        with pytest.raises(Exception):
            s.loop_times(0, 1)


# ---------------------------------------------------------------------------------------------
# Streaming solve (SATInstance::solve(getEnumeratedClause, n, batch), T=1; oracle.solve_stream is
# pinned to the reference by tests/test_oracle.py::test_oracle_matches_reference_stream)

STREAM_CASES = {
    "r2_200_400_b64": (200, 400, 3, 64),
    "r2_200_400_b1": (200, 400, 3, 1),
    "r2_5000_10000_b777": (5000, 10000, 3, 777),   # several tiles, ragged last batch
    "r2_30000_60000_b4096": (30000, 60000, 3, 4096),
}


@pytest.mark.parametrize("name", list(STREAM_CASES))
def test_stream_trajectory_matches_oracle(gpu, oracle_mod, name):
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m, k, bs = STREAM_CASES[name]
    offs, lits = generate_ksat(2, n, m, k)
    seed = 31
    st_o, A_o, rows = oracle_mod.solve_stream(n, offs, lits, seed, bs, trace=True)
    assert st_o["solved"] == 1
    with Solver(n, offs, lits, seed=seed, stream_batch=bs) as s:
        for it, nu, nm, dres, A_after in rows:
            before = s.stats()
            s.run(1)
            after = s.stats()
            assert after["n_violated"] == nu, f"iter {it}"
            assert after["n_resamples"] - before["n_resamples"] == dres, f"iter {it}"
            np.testing.assert_array_equal(s.assignment_words(), A_after, err_msg=f"A after iter {it}")
        assert len(s.mis()) == rows[-1][2]
    with Solver(n, offs, lits, seed=seed, stream_batch=bs) as s:
        st = s.solve()
        for key in ("n_iterations", "n_resamples", "avg_mis_size", "sum_mis_size", "solved"):
            assert st[key] == st_o[key], key
        np.testing.assert_array_equal(s.assignment_words(), A_o)


def test_stream_cap_and_satisfied_start(gpu, oracle_mod):
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m = 2000, 8000  # ratio 4: not solved within the cap
    offs, lits = generate_ksat(4, n, m, 3)
    st_o, A_o, _ = oracle_mod.solve_stream(n, offs, lits, 9, 100, max_iters=6)
    assert st_o["solved"] == 0 and st_o["n_iterations"] == 6
    with Solver(n, offs, lits, seed=9, max_iters=6, stream_batch=100) as s:
        st = s.solve()
        for key in ("n_iterations", "n_resamples", "avg_mis_size", "solved"):
            assert st[key] == st_o[key], key
        np.testing.assert_array_equal(s.assignment_words(), A_o)
    # one clause, satisfied by the initial assignment: one iteration, nothing resampled
    A0 = oracle_mod.init_assignment(2, 4)
    lit = np.array([0 if (A0[0] & 1) else 1], np.uint32)
    with Solver(4, np.array([0, 1], np.uint64), lit, seed=2, stream_batch=8) as s:
        st = s.solve()
        assert (st["n_iterations"], st["n_resamples"], st["avg_mis_size"], st["solved"]) == (1, 0, 0, 1)
