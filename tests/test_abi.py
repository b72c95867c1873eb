"""C-ABI boundary checks that run without a GPU: liballl.so loads, exports every symbol
include/alll.h declares, the host-side helpers (DIMACS loader, generator) match the
reference loader fixtures / the oracle generator, and the device entry points fail loudly
(no CPU fallback) when no gfx950 device is visible."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, ROOT


def header_functions():
    text = open(os.path.join(ROOT, "include", "alll.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(alll_\w+)\(", text, re.M)))


def test_library_exports_every_declared_symbol(native):
    L = native.lib()
    declared = header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(declared) == sorted(native.EXPORTED)


def test_version_and_options(native):
    L = native.lib()
    assert b"gfx950" in L.alll_version()
    o = native.Options()
    L.alll_default_options(ctypes.byref(o))
    assert o.seed == 1 and o.world == 1 and o.n_threads == 1 and o.device == -1


def test_struct_layout(native):
    # must match include/alll.h on x86-64
    assert ctypes.sizeof(native.Problem) == 32
    assert ctypes.sizeof(native.Options) == 8 + 8 + 4 * 4 + 128 + 4 + 4 + 8 + 8
    assert ctypes.sizeof(native.Stats) == 5 * 8 + 8 + 8 + 64 * 8
    assert ctypes.sizeof(native.PhaseTimes) == 6 * 8


def test_multi_gpu_plan(native):
    """alll_plan_multi_gpu: the bench instance M and C2/C5 (10M clauses or fewer,
    3-SAT) replicate at every node size -- sharding their ~28 us evaluation saves less than the
    exchange costs; C4 (128M clauses) shards from 4 GPUs on; one GPU is never sharded."""
    from alllsatisfiabilitysolver_amd import plan_multi_gpu

    cfg = {"M": (2_500_000, 10_000_000, 3), "C2": (1_000_000, 4_000_000, 3), "C5": (2_500_000, 10_000_000, 3),
           "C4": (32_000_000, 128_000_000, 3)}
    for name, (n, m, k) in cfg.items():
        p1 = plan_multi_gpu(m, m * k, n, 1)
        assert p1["plan"] == "replicate" and p1["exchange_us"] == 0.0 and p1["eval_saved_us"] == 0.0
        for G in (2, 4, 8):
            p = plan_multi_gpu(m, m * k, n, G)
            assert p["eval_saved_us"] == pytest.approx(p["eval_us_1gpu"] * (1 - 1 / G))
            want = "shard" if name == "C4" and G >= 4 else "replicate"
            assert p["plan"] == want, (name, G, p)
            assert (p["eval_saved_us"] > p["exchange_us"]) == (want == "shard")
    # the evaluation model at M: 121.6 MB at 4.3 TB/s
    assert plan_multi_gpu(10_000_000, 30_000_000, 2_500_000, 8)["eval_us_1gpu"] == pytest.approx(28.3, abs=0.5)
    assert native.lib().alll_plan_multi_gpu(1, 3, 1, 0, None) != 0  # bad arguments


@pytest.mark.parametrize("name", ["c1_3sat_200_800_T1", "u3sat_2500_10000_T1", "k8_4000_6000_T1", "edge_T1"])
def test_reference_initial_assignment_matches_reference(native, name):
    """alll_reference_initial_assignment (the compatibility VariablesArray under
    ALLL_REFERENCE_RNG): the reference's own VariablesArray fill recorded by its trace (rd_seed 7)."""
    f = dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))
    n = int(f["n_vars"])
    rd = json.load(open(os.path.join(GOLDEN, "manifest.json")))["rd_seed"]
    out = np.zeros(n, np.uint8)
    assert native.lib().alll_reference_initial_assignment(rd, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) == 0
    want = np.array([(int(f["A"][0][v >> 5]) >> (v & 31)) & 1 for v in range(n)], np.uint8)
    np.testing.assert_array_equal(out, want)


def test_create_fails_loudly_without_gpu(native):
    from alllsatisfiabilitysolver_amd import Solver, AlllError

    offs = np.array([0, 2], np.uint64)
    lits = np.array([0, 3], np.uint32)
    if native.lib().alll_device_count() > 0:
        pytest.skip("GPU visible")
    with pytest.raises(AlllError) as ei:
        Solver(2, offs, lits)
    assert ei.value.code == native.ALLL_ERR_NO_DEVICE


def test_create_validates_input(native):
    from alllsatisfiabilitysolver_amd import Solver, AlllError

    with pytest.raises(AlllError) as ei:
        Solver(2, np.array([0, 2], np.uint64), np.array([0, 9], np.uint32))
    assert ei.value.code == native.ALLL_ERR_LITERAL_RANGE
    with pytest.raises(AlllError) as ei:
        Solver(2, np.array([1, 2], np.uint64), np.array([0, 1], np.uint32))
    assert ei.value.code == native.ALLL_ERR_BAD_INPUT


def _ref_lists(ref):
    out, p = [], 0
    for n in ref["l_c_num"]:
        out.append(ref["l_val"][p:p + n])
        p += n
    return out


def test_product_dimacs_matches_reference_loader(native):
    from alllsatisfiabilitysolver_amd import parse_dimacs

    cases = json.load(open(os.path.join(GOLDEN, "dimacs_cases.json")))
    for key, case in cases.items():
        ref = case["ref"]
        v, offs, lits = parse_dimacs(case["text"].encode())
        assert v == ref["v_num"] and offs.size - 1 == ref["c_num"], key
        enc = [[2 * x - 2 if x > 0 else -2 * x - 1 for x in cl] for cl in _ref_lists(ref)]
        got = [[int(x) for x in lits[offs[c]:offs[c + 1]]] for c in range(offs.size - 1)]
        assert got == enc, key


def test_product_dimacs_errors(native, tmp_path):
    from alllsatisfiabilitysolver_amd import parse_dimacs, read_dimacs, AlllError

    for text, code in [(b"q cnf 1 1\n1 0\n", native.ALLL_ERR_BAD_INPUT),
                       (b"p cnf 3 2\n1 0\n", native.ALLL_ERR_BAD_INPUT),         # missing clause
                       (b"p cnf 3 2\n1 0\n2 0", native.ALLL_ERR_BAD_INPUT),      # last line dropped
                       (b"p cnf 2 1\n1 -3 0\n", native.ALLL_ERR_LITERAL_RANGE),
                       (b"", native.ALLL_ERR_BAD_INPUT)]:
        with pytest.raises(AlllError) as ei:
            parse_dimacs(text)
        assert ei.value.code == code, text
    with pytest.raises(AlllError) as ei:
        read_dimacs(str(tmp_path / "missing.cnf"))
    assert ei.value.code == native.ALLL_ERR_IO


def test_product_dimacs_roundtrip_file(native, oracle_mod, tmp_path):
    from alllsatisfiabilitysolver_amd import read_dimacs

    o = oracle_mod
    offs, lits = o.generate_ksat(4, 300, 1200, 3)
    p = tmp_path / "x.cnf"
    p.write_text(o.to_dimacs(300, offs, lits, comments=["generated"]))
    v, offs2, lits2 = read_dimacs(str(p))
    assert v == 300
    np.testing.assert_array_equal(offs, offs2)
    np.testing.assert_array_equal(lits, lits2)
    rc, (v3, offs3, lits3) = o.dimacs_parse(p.read_bytes())
    assert rc == 0
    np.testing.assert_array_equal(lits, lits3)


def _messy_dimacs(rng, n_vars, n_clauses, bad=None):
    """DIMACS text exercising the loader's line rules: comments, blank lines, clauses split
    over lines and several clauses on one line, trailing words after a non-number, extra
    clauses past the header count, and optionally an out-of-range literal."""
    lines = ["c generated", "", "p cnf %d %d" % (n_vars, n_clauses)]
    cur = []
    for c in range(n_clauses + 5):
        k = int(rng.integers(0, 6))
        lits = [int(v) * (1 if rng.integers(0, 2) else -1) for v in rng.integers(1, n_vars + 1, k)]
        if bad is not None and c == bad:
            lits.append(n_vars + 3)
        toks = [str(x) for x in lits] + ["0"]
        r = rng.integers(0, 10)
        if r == 0:
            lines.append("c " + " ".join(toks))
        if r == 1:
            lines.append("   ")
        if r == 2 and len(toks) > 1:       # clause split over two lines
            cur += toks[:1]
            lines.append(" ".join(cur))
            cur = toks[1:]
        else:
            cur += toks
        if r != 3:                         # r == 3: next clause shares the line
            if r == 4:
                cur.append("x 7 0")        # a non-number word ends the line
            lines.append("  ".join(cur))
            cur = []
    lines.append(" ".join(cur + ["1", "0"]))
    return ("\n".join(lines) + "\n").encode()


@pytest.fixture
def force_parallel_loader(monkeypatch):
    monkeypatch.setenv("ALLL_DIMACS_MIN_PARALLEL", "0")


def test_parallel_dimacs_matches_reference_loader(native, force_parallel_loader):
    test_product_dimacs_matches_reference_loader(native)


def test_parallel_dimacs_errors(native, force_parallel_loader, tmp_path):
    test_product_dimacs_errors(native, tmp_path)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_parallel_dimacs_matches_oracle(native, oracle_mod, monkeypatch, seed):
    from alllsatisfiabilitysolver_amd import parse_dimacs

    rng = np.random.default_rng(seed)
    text = _messy_dimacs(rng, 500, 20000)
    rc, (v0, o0, l0) = oracle_mod.dimacs_parse(text)
    assert rc == 0
    for thresh in ["0", str(1 << 40)]:     # parallel, serial
        monkeypatch.setenv("ALLL_DIMACS_MIN_PARALLEL", thresh)
        v, offs, lits = parse_dimacs(text)
        assert v == v0
        np.testing.assert_array_equal(offs, o0)
        np.testing.assert_array_equal(lits, l0)


@pytest.mark.parametrize("text", [
    b"p cnf 3 1\n1 0\n2\n",                 # literals after the last zero
    b"p cnf 3 1\n1 0 2 3\n",
    b"p cnf 3 2\n1 0 2 0 3 0\n-1\n",        # clauses past the header's count
    b"p cnf 3 0\n1 2\n",
    b"p cnf 3 0\n",
    b"c x\n\n  \np cnf 3 2\n+1 2x 0 -3\n\n2\t0 -\n0\n",  # signs, trailing non-digits, tabs
])
def test_parallel_dimacs_edge_cases(native, oracle_mod, monkeypatch, text):
    from alllsatisfiabilitysolver_amd import parse_dimacs

    rc, (v0, o0, l0) = oracle_mod.dimacs_parse(text)
    assert rc == 0
    for nt in ["2", "3", "64"]:
        monkeypatch.setenv("ALLL_DIMACS_MIN_PARALLEL", "0")
        monkeypatch.setenv("ALLL_DIMACS_THREADS", nt)
        v, offs, lits = parse_dimacs(text)
        assert v == v0
        np.testing.assert_array_equal(offs, o0)
        np.testing.assert_array_equal(lits, l0)


def test_parallel_dimacs_literal_range(native, monkeypatch):
    """Out-of-range literals: same error code, clause index in the message and skipped
    literals as the serial loader."""
    L = native.lib()
    rng = np.random.default_rng(7)
    for bad in [0, 777, 19999, 20002]:    # 20002 is past the header count: not an error
        text = _messy_dimacs(rng, 300, 20000, bad=bad)
        res = []
        for thresh in ["0", str(1 << 40)]:
            monkeypatch.setenv("ALLL_DIMACS_MIN_PARALLEL", thresh)
            v, c, ln = ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_uint64()
            rc = L.alll_dimacs_parse(text, len(text), ctypes.byref(v), ctypes.byref(c), None, None,
                                     ctypes.byref(ln))
            msg = native.last_error()
            offs = np.zeros(c.value + 1, np.uint64)
            lits = np.zeros(max(1, ln.value), np.uint32)
            rc2 = L.alll_dimacs_parse(text, len(text), ctypes.byref(v), ctypes.byref(c),
                                      offs.ctypes.data_as(native._u64p), lits.ctypes.data_as(native._u32p),
                                      ctypes.byref(ln))
            res.append((rc, rc2, msg if rc else "", offs, lits))
        (p_rc, p_rc2, p_msg, p_o, p_l), (s_rc, s_rc2, s_msg, s_o, s_l) = res
        assert (p_rc, p_rc2) == (s_rc, s_rc2)
        assert p_rc == (native.ALLL_ERR_LITERAL_RANGE if bad < 20000 else native.ALLL_OK)
        assert p_msg == s_msg and (bad >= 20000 or f"clause {bad}" in p_msg)
        np.testing.assert_array_equal(p_o, s_o)
        np.testing.assert_array_equal(p_l, s_l)


@pytest.mark.parametrize("kind", [0, 1])
def test_product_generator_matches_oracle(native, oracle_mod, kind):
    from alllsatisfiabilitysolver_amd import generate_ksat

    for (n, m, k) in [(200, 800, 3), (4000, 6000, 8), (2500, 10000, 3)]:
        o1, l1 = oracle_mod.generate_ksat(1, n, m, k, kind)
        o2, l2 = generate_ksat(1, n, m, k, kind)
        np.testing.assert_array_equal(o1, o2)
        np.testing.assert_array_equal(l1, l2)
    # sub-range generation equals the slice of the full instance
    _, full = generate_ksat(7, 1000, 5000, 3, kind)
    _, part = generate_ksat(7, 1000, 5000, 3, kind, 1234, 4321)
    np.testing.assert_array_equal(full[1234 * 3:4321 * 3], part)


def test_product_generator_multithreaded_range(native, oracle_mod):
    from alllsatisfiabilitysolver_amd import generate_ksat

    _, big = generate_ksat(2, 1 << 20, 1 << 21, 3)  # threaded path (>= 2^20 clauses)
    _, ref = oracle_mod.generate_ksat(2, 1 << 20, 1 << 21, 3)
    np.testing.assert_array_equal(ref, big)
