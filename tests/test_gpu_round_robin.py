"""GPU parity of the round-robin MIS (the reference's n_threads = T > 1: populate_mis_parallel
with T sets, SATInstance.h:414-447, over the chunks of example/main.cpp:149-178 or the
caller's vector<ClauseArray*>), bit-exact:

  * reference maps on the GPU: for every T > 1 golden trajectory, the device evaluates
    A_i -> U_i and picks exactly the reference's M_i;
  * full trajectories with Philox against the oracle's T-chunk loop (orc_solve_rr, whose MIS
    is pinned by the same fixtures): assignment after every iteration, statistics;
  * the batch paths of the kernel: few sets (one 64-lane group per set, many levels), more
    sets than groups (16-lane groups, one level), erasures of empty chunks, clauses too wide
    for a group's variable buffer, caller-given chunk boundaries;
  * ALLL_FLAG_LFMIS keeps the one-set MIS for T > 1.

Every test runs with each way of deciding the MIS: the fixpoint passes (default, DESIGN.md
§4.3.2; host-driven: a first graph with as many passes as the last iteration needed, then one
pass at a time until they settle), the same passes capped at one or two per iteration
(ALLL_RR_FP_MAX, so that most iterations fall back to the batch kernel mid-run), and the batch
kernel alone (k_rr_mw, ALLL_RR_FP=0).
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

RR_FIXTURES = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*_T*.npz"))
                     if not p.endswith("_T1.npz") and not os.path.basename(p).startswith("stream"))


@pytest.fixture(scope="module")
def gpu(native):
    from alllsatisfiabilitysolver_amd import device_count

    if device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return True


@pytest.fixture(params=["fp", "fp_cap1", "fp_cap2", "mw"], autouse=True)
def rr_kernel(request, monkeypatch):
    for k in ("ALLL_RR_FP", "ALLL_RR_FP_MAX"):
        monkeypatch.delenv(k, raising=False)
    if request.param.startswith("fp_cap"):
        monkeypatch.setenv("ALLL_RR_FP_MAX", request.param[-1])
    elif request.param == "mw":
        monkeypatch.setenv("ALLL_RR_FP", "0")
    return request.param


def mask_to_list(vm, m):
    bits = np.unpackbits(vm.view(np.uint8), bitorder="little")[:m]
    return np.nonzero(bits)[0].astype(np.uint32)


def test_fixtures_present():
    assert len(RR_FIXTURES) >= 6


@pytest.mark.parametrize("path", RR_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_reference_rr_maps_on_gpu(gpu, path):
    from alllsatisfiabilitysolver_amd import Solver

    f = dict(np.load(path, allow_pickle=False))
    n, offs, lits, T = int(f["n_vars"]), f["offs"], f["lits"], int(f["T"])
    m = offs.size - 1
    with Solver(n, offs, lits, seed=3, n_threads=T) as s:
        for i in range(f["A"].shape[0]):
            s.set_assignment_words(f["A"][i])
            before = s.stats()
            s.run(1)
            after = s.stats()
            U_ref = f["U"][int(f["U_ptr"][i]):int(f["U_ptr"][i + 1])]
            np.testing.assert_array_equal(mask_to_list(s.violated_mask(), m), U_ref, err_msg=f"U_{i}")
            if U_ref.size == 0:
                assert after["solved"] == 1
                break
            M_ref = f["M"][int(f["M_ptr"][i]):int(f["M_ptr"][i + 1])]
            np.testing.assert_array_equal(s.mis(), np.sort(M_ref), err_msg=f"M_{i}")
            assert after["sum_mis_size"] - before["sum_mis_size"] == M_ref.size
            if int(f["dres"][i]):
                assert after["n_resamples"] - before["n_resamples"] == int(f["dres"][i])


def _instance(name):
    from alllsatisfiabilitysolver_amd import generate_ksat

    if name == "ratio4":
        n, m = 3000, 12000
        return (n,) + generate_ksat(1, n, m, 3)
    if name == "ratio2_solves":
        n, m = 2000, 4000
        return (n,) + generate_ksat(2, n, m, 3)
    if name == "k5_multi_tile":
        n, m = 30000, 60000
        return (n,) + generate_ksat(1, n, m, 5)
    if name == "powerlaw":
        n, m = 5000, 20000
        return (n,) + generate_ksat(1, n, m, 3, 1)
    if name == "wide":  # clauses of up to 150 literals: wider than a group's variable buffer
        rng = np.random.default_rng(11)
        m, n = 3000, 4000
        w = rng.integers(1, 8, m)
        w[rng.choice(m, 40, replace=False)] = rng.integers(40, 150, 40)
        offs = np.zeros(m + 1, np.uint64)
        offs[1:] = np.cumsum(w)
        lits = rng.integers(0, 2 * n, int(offs[-1])).astype(np.uint32)
        return n, offs, lits
    if name == "edge":
        f = dict(np.load(os.path.join(GOLDEN, "edge_T1.npz")))
        return int(f["n_vars"]), f["offs"], f["lits"]
    raise KeyError(name)


CASES = [("ratio4", 2), ("ratio4", 3), ("ratio4", 8), ("ratio4", 16), ("ratio4", 17), ("ratio4", 64),
         ("ratio4", 65), ("ratio4", 300), ("ratio2_solves", 4), ("ratio2_solves", 100),
         ("k5_multi_tile", 7), ("k5_multi_tile", 40), ("powerlaw", 5), ("powerlaw", 33),
         ("wide", 4), ("wide", 20), ("wide", 90), ("edge", 3), ("edge", 8)]


@pytest.mark.parametrize("name,T", CASES, ids=[f"{a}-T{b}" for a, b in CASES])
def test_rr_trajectory_matches_oracle(gpu, oracle_mod, name, T):
    from alllsatisfiabilitysolver_amd import Solver

    o = oracle_mod
    n, offs, lits = _instance(name)
    seed, K = 4242, 30
    st_o, A_o, rows = o.solve(n, offs, lits, seed, max_iters=K, trace=True, T=T)
    with Solver(n, offs, lits, seed=seed, n_threads=T) as s:
        for it, nu, nm, dres, A_after in rows:
            before = s.stats()
            s.run(1)
            after = s.stats()
            assert after["n_violated"] == nu, f"iter {it}"
            assert after["sum_mis_size"] - before["sum_mis_size"] == nm, f"iter {it}"
            assert after["n_resamples"] - before["n_resamples"] == dres, f"iter {it}"
            np.testing.assert_array_equal(s.assignment_words(), A_after, err_msg=f"A after iter {it}")
    with Solver(n, offs, lits, seed=seed, n_threads=T, max_iters=K) as s:
        st = s.solve()
        for k in ("n_iterations", "n_resamples", "avg_mis_size", "sum_mis_size", "solved"):
            assert st[k] == st_o[k], k
        np.testing.assert_array_equal(s.assignment_words(), A_o)


def test_rr_long_run_across_cover_stamp_cycles(gpu, oracle_mod):
    """600 iterations of the T = 4 round robin cross two wraps of the 8-bit cover stamps."""
    from alllsatisfiabilitysolver_amd import Solver

    n, offs, lits = _instance("ratio4")
    seed, K, T = 31, 600, 4
    st_o, A_o, _ = oracle_mod.solve(n, offs, lits, seed, max_iters=K, T=T)
    assert st_o["solved"] == 0
    with Solver(n, offs, lits, seed=seed, n_threads=T, max_iters=K) as s:
        st = s.solve()
        for k in ("n_iterations", "n_resamples", "avg_mis_size", "sum_mis_size", "solved"):
            assert st[k] == st_o[k], k
        np.testing.assert_array_equal(s.assignment_words(), A_o)


def test_rr_caller_chunks(gpu, oracle_mod):
    """Chunk boundaries from the caller (the sizes of its vector<ClauseArray*>), including
    empty chunks at the front, middle and end."""
    from alllsatisfiabilitysolver_amd import Solver

    o = oracle_mod
    n, offs, lits = _instance("ratio4")
    m = offs.size - 1
    starts = np.array([0, 0, 100, 100, 5000, 5001, 11999, m, m], np.uint64)
    T = starts.size - 1
    st_o, A_o, _ = o.solve(n, offs, lits, 8, max_iters=20, T=T, chunk_starts=starts)
    with Solver(n, offs, lits, seed=8, n_threads=T, max_iters=20, set_starts=starts) as s:
        st = s.solve()
        for k in ("n_iterations", "n_resamples", "avg_mis_size"):
            assert st[k] == st_o[k], k
        np.testing.assert_array_equal(s.assignment_words(), A_o)


def test_rr_converges_and_verifies(gpu, oracle_mod):
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m, T = 25000, 50000, 12
    offs, lits = generate_ksat(2, n, m, 3)
    st_o, A_o, _ = oracle_mod.solve(n, offs, lits, 99, T=T)
    assert st_o["solved"] == 1
    with Solver(n, offs, lits, seed=99, n_threads=T) as s:
        st = s.solve()
        assert st["solved"] == 1
        for k in ("n_iterations", "n_resamples", "avg_mis_size"):
            assert st[k] == st_o[k]
        np.testing.assert_array_equal(s.assignment_words(), A_o)
        ok, nv = s.verify()
        assert ok and nv == 0


def test_rr_flag_lfmis_and_limits(gpu, oracle_mod, native):
    from alllsatisfiabilitysolver_amd import Solver, AlllError

    n, offs, lits = _instance("ratio4")
    st_o, A_o, _ = oracle_mod.solve(n, offs, lits, 5, max_iters=10)
    with Solver(n, offs, lits, seed=5, n_threads=8, max_iters=10, flags=native.FLAG_LFMIS) as s:
        s.solve()
        np.testing.assert_array_equal(s.assignment_words(), A_o)
    with pytest.raises(AlllError) as ei:
        Solver(n, offs, lits, n_threads=5000)
    assert ei.value.code == native.ALLL_ERR_UNSUPPORTED
    with pytest.raises(AlllError) as ei:
        Solver(n, offs, lits, n_threads=2, set_starts=np.array([0, 5, 7], np.uint64))
    assert ei.value.code == native.ALLL_ERR_INVALID_ARG


def test_rr_python_satinstance(gpu, oracle_mod):
    """SATInstance(var_arr, n_threads).solve(chunks) runs the round robin over the chunks."""
    from alllsatisfiabilitysolver_amd import Clause, SATInstance, VariablesArray

    o = oracle_mod
    n, offs, lits = _instance("ratio2_solves")
    m = offs.size - 1
    T = 3
    starts = o.chunk_bounds(m, T)
    chunks = [[Clause([int(x) for x in lits[offs[c]:offs[c + 1]]]) for c in range(int(starts[q]), int(starts[q + 1]))]
              for q in range(T)]
    va = VariablesArray(n)
    inst = SATInstance(va, T, seed=21)
    stats = inst.solve(chunks)
    st_o, A_o, _ = o.solve(n, offs, lits, 21, T=T)
    assert stats.n_iterations == st_o["n_iterations"] and stats.n_resamples == st_o["n_resamples"]
    assert inst.verify_validity(chunks)


@pytest.mark.parametrize("T", [16, 5])
def test_rr_full_size_c2_bit_exact(gpu, oracle_mod, rr_kernel, T):
    """BASELINE config C2 (random 3-SAT, 1M variables / 4M clauses) with the round robin of T
    sets: two iterations, every violated set, MIS and assignment against the oracle's
    orc_solve_rr (the fixpoint passes settle on ~500k violated clauses per iteration)."""
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m, seed, K = 1_000_000, 4_000_000, 12, 2
    offs, lits = generate_ksat(1, n, m, 3)
    st_o, A_o, rows = oracle_mod.solve(n, offs, lits, seed, max_iters=K + 1, trace=True, T=T)
    with Solver(n, offs, lits, seed=seed, n_threads=T) as s:
        for it, nu, nm, dres, A_after in rows[:K]:
            before = s.stats()
            s.run(1)
            after = s.stats()
            assert after["n_violated"] == nu, f"iter {it}"
            assert after["sum_mis_size"] - before["sum_mis_size"] == nm, f"iter {it}"
            assert after["n_resamples"] - before["n_resamples"] == dres, f"iter {it}"
            np.testing.assert_array_equal(s.assignment_words(), A_after, err_msg=f"A after iter {it}")


def test_rr_back_to_back_runs_without_sync(gpu, oracle_mod, monkeypatch):
    """Several run(1) calls with no stats() or synchronisation in between (the pass count of
    one iteration sizes the next one's first graph): the same trajectory as the oracle."""
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m, T, seed = 6000, 24000, 5, 9
    offs, lits = generate_ksat(4, n, m, 3, 0)
    st_o, A_o, rows = oracle_mod.solve(n, offs, lits, seed, max_iters=13, trace=True, T=T)
    with Solver(n, offs, lits, seed=seed, n_threads=T) as s:
        for _ in range(12):
            s.run(1, sync=False)
        s.synchronize()
        st = s.stats()
        assert st["n_iterations"] == 12
        assert st["n_resamples"] == sum(r[3] for r in rows)
        np.testing.assert_array_equal(s.assignment_words(), rows[-1][4])


# name: (environment, solver flag): every evaluation the round robin can run over
RR_LAYOUTS = {"positions": ({"ALLL_PACKED_IDS": "0"}, None),  # clause ids via perm (k_rr_mark's unpack)
              "small_windows": ({"ALLL_EVAL_WINDOWS": "1", "ALLL_WIN_WORDS": "64"}, None),
              "nt_windows": ({"ALLL_EVAL_WINDOWS": "1", "ALLL_WIN_WORDS": "64", "ALLL_EVAL_NT": "1"}, None),
              # the L2-gather evaluation k_eval_fixed writes the lists k_rr_mark reads
              "fixed": ({}, "FLAG_NO_RANGED"),
              # the clause-order CSR evaluation (its bitmask feeds k_rr_entries directly)
              "csr": ({}, "FLAG_GENERIC_CSR")}


@pytest.mark.parametrize("layout", list(RR_LAYOUTS))
@pytest.mark.parametrize("name,T", [("ratio4", 7), ("k5_multi_tile", 16)])
def test_rr_on_hybrid_eval_layouts(gpu, oracle_mod, native, name, T, layout, monkeypatch):
    """The round robin over every fixed-width evaluation: the hybrid kernel's per-tile lists in
    evaluation order become clause-order flags (k_rr_mark) under every layout; the L2-gather
    kernel's lists the same way; the CSR evaluation's clause-order bitmask directly."""
    from alllsatisfiabilitysolver_amd import Solver

    n, offs, lits = _instance(name)
    seed, K = 17, 10
    st_o, A_o, rows = oracle_mod.solve(n, offs, lits, seed, max_iters=K, trace=True, T=T)
    env, flag = RR_LAYOUTS[layout]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    flags = getattr(native, flag) if flag else 0
    with Solver(n, offs, lits, seed=seed, n_threads=T, flags=flags) as s:
        for k in env:
            monkeypatch.delenv(k)
        for it, nu, nm, dres, A_after in rows:
            s.run(1)
            assert s.stats()["n_violated"] == nu, f"iter {it}"
            np.testing.assert_array_equal(s.assignment_words(), A_after, err_msg=f"A after iter {it}")


_TORCH_FIRST_CHILD = r"""
import json, sys
import numpy as np
import torch  # first: its wheel's HIP runtime (same soname) then serves the library too
assert torch.cuda.is_available()
sys.path.insert(0, sys.argv[1])
from alllsatisfiabilitysolver_amd import Solver, generate_ksat
maps = sorted({l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l})
n, m, T, seed, K = (int(x) for x in sys.argv[3:8])
offs, lits = generate_ksat(1, n, m, 3)
with Solver(n, offs, lits, seed=seed, device=0, n_threads=T) as s:
    for _ in range(K):
        s.run(1)
    np.save(sys.argv[2], s.assignment_words())
    st = s.stats()
print(json.dumps({"hip_runtime": maps, "n_iterations": st["n_iterations"], "n_resamples": st["n_resamples"],
                  "sum_mis_size": st["sum_mis_size"]}))
"""


def test_rr_under_torch_runtime(gpu, oracle_mod, tmp_path):
    """The round robin in a process that imported torch first, so that the library runs on the
    HIP runtime bundled in torch's wheel (ROCm 7.0; the loop's graphs once stalled there,
    DESIGN.md §10): K iterations of host-driven pass graphs (every graph replayed several times)
    in a subprocess under a time limit, bit-exact against the oracle's T-chunk loop."""
    import json
    import subprocess
    import sys

    from alllsatisfiabilitysolver_amd import generate_ksat

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n, m, T, seed, K = 250_000, 1_000_000, 16, 3, 24
    out = str(tmp_path / "A.npy")
    r = subprocess.run([sys.executable, "-c", _TORCH_FIRST_CHILD, root, out] + [str(x) for x in (n, m, T, seed, K)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["hip_runtime"] and all("torch" in p for p in d["hip_runtime"]), d["hip_runtime"]
    offs, lits = generate_ksat(1, n, m, 3)
    _, _, rows = oracle_mod.solve(n, offs, lits, seed, max_iters=K + 1, trace=True, T=T)
    assert d["n_iterations"] == K == len(rows)
    assert d["n_resamples"] == sum(r[3] for r in rows) and d["sum_mis_size"] == sum(r[2] for r in rows)
    np.testing.assert_array_equal(np.load(out), rows[-1][4])


def test_rr_flags_cleared_when_the_loop_stops(gpu, oracle_mod):
    """The evaluation sets the clause-order violated flags before the reduce decides whether the
    iteration runs (k_eval_flags): a loop stopped by max_iters leaves them set unless cleared
    (ADVICE r5).  solve(max_iters) -> set_assignment -> run(1) must pick the oracle's MIS of the
    new assignment, and resample exactly its variables."""
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat

    n, m, T = 2000, 8000, 4  # ratio 4: not solved within the cap
    offs, lits = generate_ksat(4, n, m, 3)
    A_new = oracle_mod.init_assignment(77, n)
    with Solver(n, offs, lits, seed=3, n_threads=T, max_iters=3) as s:
        st = s.solve()
        assert st["solved"] == 0 and st["n_violated"] > 0
        s.set_assignment_words(A_new)
        s.run(1)
        nu, vm = oracle_mod.eval_mask(offs, lits, A_new)
        M = oracle_mod.rr_mis(n, offs, lits, mask_to_list(vm, m), T)
        np.testing.assert_array_equal(s.mis(), np.sort(M))
        it = s.stats()["n_iterations"] - 1
        A_exp = oracle_mod.resample_words(A_new.copy(), 3, it, oracle_mod.clause_vars(offs, lits, M))
        np.testing.assert_array_equal(s.assignment_words(), A_exp)


@pytest.mark.parametrize("knobs", [{"ALLL_RR_INC": "0"}, {"ALLL_RR_REP_CAP": "4"}, {"ALLL_RR_RW_MIN": "4"},
                                   {"ALLL_RR_RW_MIN": "4", "ALLL_RR_RW_TIMEOUT": "0"}],
                         ids=["full_passes_only", "repair_gives_up", "wide_rounds_small", "wide_barrier_timeout"])
def test_rr_incremental_pass_fallbacks(gpu, oracle_mod, rr_kernel, knobs, monkeypatch):
    """The incremental passes' fallbacks stay exact: full passes only
    (ALLL_RR_INC=0); a repair whose dirty set outgrows its cap gives up and a full pass follows;
    the wide (multi-workgroup) repair rounds on a small instance; wide rounds whose grid barrier
    times out (the pass gives up, counted by alll_rr_barrier_timeouts).  Trajectory against the
    oracle after every iteration, and the pass log shows the fallback happened."""
    from alllsatisfiabilitysolver_amd import Solver, generate_ksat
    from alllsatisfiabilitysolver_amd import _native as N

    if rr_kernel != "fp":
        pytest.skip("incremental passes: the default fixpoint mode")
    n, m, T, seed, K = 20000, 80000, 8, 3, 6
    offs, lits = generate_ksat(9, n, m, 3)
    st_o, A_o, rows = oracle_mod.solve(n, offs, lits, seed, max_iters=K + 1, trace=True, T=T)
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    logs, wide = [], 0
    with Solver(n, offs, lits, seed=seed, n_threads=T, flags=N.FLAG_KERNEL_TIMING) as s:
        for k in knobs:
            monkeypatch.delenv(k)
        for it, nu, nm, dres, A_after in rows[:K]:
            s.run(1)
            np.testing.assert_array_equal(s.assignment_words(), A_after, err_msg=f"iter {it}")
            logs.append(s.rr_pass_log().copy())
            wide += int((s.rr_round_log()[:64, 56] != 0).sum())  # a wide round's stamp per pass
        timeouts = s.rr_barrier_timeouts()
    inc = [r for lg in logs for r in lg if r.any()]
    bails = [r for r in inc if r[1] == 0xFFFFFFFF]
    if "ALLL_RR_INC" in knobs:
        assert not inc and timeouts == 0
    elif "ALLL_RR_REP_CAP" in knobs:
        assert bails, "no incremental pass gave up"
    elif "ALLL_RR_RW_TIMEOUT" in knobs:
        assert timeouts > 0 and bails
    else:
        assert wide > 0 and timeouts == 0, f"no wide repair round ran: passes {[tuple(map(int, r)) for r in inc][:12]}"
