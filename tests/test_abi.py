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
    assert ctypes.sizeof(native.Options) == 8 + 8 + 4 * 4 + 128 + 4 + 4 + 8
    assert ctypes.sizeof(native.Stats) == 5 * 8 + 8 + 8 + 64 * 8
    assert ctypes.sizeof(native.PhaseTimes) == 6 * 8


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
