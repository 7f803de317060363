"""Matrix Market reader (host part) against the reference's own data files and the fixtures made
from them (tests/golden/mm/*.mtx are copies of the reference's ReleaseTests / 3DSpGEMM files;
tests/golden/fixtures.npz holds the matrices the golden products were computed from)."""
import os

import numpy as np
import pytest

import helpers as H

MM = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mm")


def _host_dcsc(m, n, rows, cols, vals):
    return H.Dcsc.from_coo(m, n, list(rows), list(cols), np.asarray(vals, np.float64))


@pytest.mark.parametrize("name", ["sevenvertex", "small_nonsym"])
def test_mmread_general_matches_fixture(fixtures, name):
    from combblas_amd.mm import mmread

    m, n, r, c, v, field, sym = mmread(os.path.join(MM, f"{name}.mtx"))
    assert sym == "general"
    H.assert_dcsc_equal(_host_dcsc(m, n, r, c, v), fixtures[f"{name}_A"])


def test_mmread_symmetric_expands(fixtures):
    from combblas_amd.mm import mmread

    m, n, r, c, v, field, sym = mmread(os.path.join(MM, "bcsstk01.mtx"), expand_symmetric=False)
    assert (field, sym) == ("real", "symmetric")
    H.assert_dcsc_equal(_host_dcsc(m, n, r, c, v), fixtures["bcsstk01_A"])
    m, n, r2, c2, v2, _, _ = mmread(os.path.join(MM, "bcsstk01.mtx"))
    off = r != c
    assert r2.size == r.size + off.sum()
    full = _host_dcsc(m, n, r2, c2, v2)
    # ParallelReadMM mirrors (i, j) -> (j, i): the expanded matrix is symmetric
    dense = np.zeros((m, n))
    for j in range(full.nzc):
        for p in range(full.cp[j], full.cp[j + 1]):
            dense[full.ir[p], full.jc[j]] = full.num[p]
    assert np.array_equal(dense, dense.T)


def test_mmread_pattern_and_integer(tmp_path):
    from combblas_amd.mm import mmread

    p = tmp_path / "p.mtx"
    p.write_text("%%MatrixMarket matrix coordinate pattern general\n% c\n3 4 3\n1 1\n3 4\n2 2\n")
    m, n, r, c, v, field, _ = mmread(str(p))
    assert (m, n, field) == (3, 4, "pattern") and list(r) == [0, 2, 1] and list(c) == [0, 3, 1]
    assert np.array_equal(v, np.ones(3))
    q = tmp_path / "i.mtx"
    q.write_text("%%MatrixMarket matrix coordinate integer general\n2 2 2\n1 2 7\n2 1 -3\n")
    _, _, r, c, v, field, _ = mmread(str(q))
    assert field == "integer" and v.dtype == np.int64 and list(v) == [7, -3]


def test_mmread_rejects_out_of_range(tmp_path):
    from combblas_amd.mm import mmread

    p = tmp_path / "bad.mtx"
    p.write_text("%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1.0\n")
    with pytest.raises(ValueError):
        mmread(str(p))
