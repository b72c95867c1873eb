"""The drop-in surface above the C-ABI: the CMake package (find_package + target, as the
reference's example/CMakeLists.txt consumes it), the SATInstance compatibility headers and the
Boost-free CLI with the flags and output of example/main.cpp (-h, -o, -p N, --sat)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT

CLI = os.path.join(ROOT, "tools", "alll_main")


def test_cmake_package_builds_consumer(native, tmp_path):
    if shutil.which("cmake") is None:
        pytest.skip("cmake not available")
    b = tmp_path / "b"
    r = subprocess.run(["cmake", "-S", os.path.join(ROOT, "tools", "cmake_consumer"), "-B", str(b),
                        f"-DALLLSatisfiabilitySolver_DIR={os.path.join(ROOT, 'cmake')}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run(["cmake", "--build", str(b)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert (b / "ALLLSatisfiabilitySolverMain").exists()


def test_cli_help_and_missing_sat(native):
    if not os.path.exists(CLI):
        subprocess.run(["make", "-s", "-C", ROOT, "cli"], check=True)
    r = subprocess.run([CLI, "-h"], capture_output=True, text=True)
    assert r.returncode == 0 and "--sat" in r.stdout and "--parallel" in r.stdout
    r = subprocess.run([CLI], capture_output=True, text=True)
    assert r.returncode == 1 and "sat" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [1, 4])
def test_cli_solves_and_matches_oracle(oracle_mod, native, tmp_path, threads):
    o = oracle_mod
    n, m, seed = 3000, 6000, 17  # ratio 2: converges
    offs, lits = o.generate_ksat(2, n, m, 3)
    path = tmp_path / "inst.cnf"
    path.write_text(o.to_dimacs(n, offs, lits, comments=["cli test"]))
    st, A, _ = o.solve(n, offs, lits, seed)
    assert st["solved"]
    r = subprocess.run([CLI, "-o", "-p", str(threads), "--seed", str(seed), "--sat", str(path)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout
    assert "SATISFIABLE" in out
    assert "# Clauses\t= 0" in out  # main.cpp prints n_clauses before solve() sets it
    assert f"# Iterations\t= {st['n_iterations']}" in out
    assert f"# Resamples\t= {st['n_resamples']}" in out
    assert f"Avg. UNSAT MIS Size = {st['avg_mis_size']}" in out
    assert out.count("\tThread ") == threads
    csv = (tmp_path / "inst.csv").read_text().strip().split(",")
    assert len(csv) == 6 and csv[1] == str(n) and csv[2] == "0" and csv[4] == str(threads)
    assert csv[5] == str(st["n_iterations"])
    dump = (tmp_path / "inst.out").read_text()
    vals = [int(line.split("= ")[1]) for line in dump.splitlines() if line.startswith("Variable ")]
    np.testing.assert_array_equal(np.array(vals, np.uint8), o.unpack_words(A, n))


@pytest.mark.gpu
def test_cli_unsolvable_cap_exit_code(native, tmp_path):
    path = tmp_path / "u.cnf"
    path.write_text("p cnf 2 4\n1 2 0\n1 -2 0\n-1 2 0\n-1 -2 0\n")  # UNSAT
    r = subprocess.run([CLI, "--max-iters", "50", "--sat", str(path)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 1
    assert "ERROR: Solver converged to an invalid solution!" in r.stdout
    assert "# Iterations\t= 50" in r.stdout
