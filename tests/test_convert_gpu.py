"""Device format conversions on the GPU: tuples -> DCSC (cbh_tuples_to_dcsc),
DCSC -> tuples (cbh_dcsc_to_tuples) and Matrix Market files through them.

Pins: the R-MAT edge list of the reference's packed Graph500 generator converts to exactly the
matrix `SpParMat(DistEdgeList, removeloops)` builds (the host conversion pinned to the reference
in test_oracle.py); the reference's own .mtx files read onto the device multiply to the
reference's products (tests/golden/fixtures.npz, made by oracle/_ref from the reference sources).
Other cases compare with a numpy restatement of SortColBased + duplicate summation (dyadic values,
so sums are exact in any order).
"""
import os

import numpy as np
import pytest
import torch

import helpers as H

pytestmark = pytest.mark.gpu
MM = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mm")
DEV = torch.device("cuda", 0)


def _expect(m, n, rows, cols, vals, drop_loops=False, op=np.add):
    order = np.lexsort((rows, cols))  # column-major, stable
    r, c, v = rows[order], cols[order], vals[order]
    key = c * m + r
    head = np.ones(len(key), bool)
    head[1:] = key[1:] != key[:-1]
    starts = np.nonzero(head)[0]
    s = op.reduceat(v, starts) if len(v) else v
    r, c = r[starts], c[starts]
    if drop_loops:
        keep = r != c
        r, c, s = r[keep], c[keep], s[keep]
    return H.Dcsc.from_coo(m, n, list(r), list(c), s)


def _host(M):
    h = M.to_host()
    return H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num)


@pytest.mark.parametrize("dt", [np.float64, np.int64, np.float32, np.int32, np.bool_])
@pytest.mark.parametrize("drop", [False, True])
def test_tuples_to_dcsc_random(ctx, dt, drop):
    import combblas_amd as cb

    rng = np.random.default_rng(11)
    m, n, k = 300, 217, 5000  # ~7 % duplicates, unsorted, diagonal entries present
    rows = rng.integers(0, m, k)
    cols = rng.integers(0, n, k)
    vals = (rng.integers(-8, 9, k) * 0.25).astype(dt) if dt != np.bool_ else rng.integers(0, 2, k).astype(bool)
    M = cb.SpDCCols.from_tuples(ctx, m, n, torch.from_numpy(rows).to(DEV), torch.from_numpy(cols).to(DEV),
                                torch.from_numpy(vals).to(DEV), removeloops=drop)
    exp = _expect(m, n, rows, cols, vals.astype(np.uint8) if dt == np.bool_ else vals, drop,
                  np.bitwise_or if dt == np.bool_ else np.add)
    H.assert_dcsc_equal(_host(M), exp)


def test_tuples_to_dcsc_rmat_edges_match_reference_build(ctx):
    """the reference generator's edge list -> the same A as SpParMat(DistEdgeList) (multiplicities)"""
    import combblas_amd as cb

    src, dst = cb.rmat_edges(12)
    A = cb.rmat(12)
    M = cb.SpDCCols.from_tuples(ctx, A.m, A.n, torch.from_numpy(src).to(DEV), torch.from_numpy(dst).to(DEV),
                                torch.ones(src.size, dtype=torch.int64, device=DEV))
    H.assert_dcsc_equal(_host(M), H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))


def test_dcsc_to_tuples_roundtrip(ctx):
    import combblas_amd as cb

    A = cb.rmat(10, dtype=np.float64)
    dA = cb.SpDCCols.from_host(ctx, A)
    r, c, v = dA.to_tuples()
    assert r.dtype == torch.int32 and c.dtype == torch.int64 and r.numel() == A.nnz
    cols = np.repeat(A.jc, np.diff(A.cp))
    assert np.array_equal(c.cpu().numpy(), cols) and np.array_equal(r.cpu().numpy(), A.ir)
    assert np.array_equal(v.cpu().numpy(), A.num)
    back = cb.SpDCCols.from_tuples(ctx, A.m, A.n, r, c, v)
    H.assert_dcsc_equal(_host(back), H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))


def test_tuples_edge_cases(ctx):
    import combblas_amd as cb
    from combblas_amd._lib import CombBLASHipError

    e = torch.empty(0, dtype=torch.int64, device=DEV)
    M = cb.SpDCCols.from_tuples(ctx, 5, 7, e.to(torch.int32), e, torch.empty(0, dtype=torch.float64, device=DEV))
    assert (M.m, M.n, M.nnz, M.nzc) == (5, 7, 0, 0)
    only_loops = torch.tensor([1, 2], device=DEV)
    M = cb.SpDCCols.from_tuples(ctx, 4, 4, only_loops, only_loops, torch.ones(2, dtype=torch.float64, device=DEV),
                                removeloops=True)
    assert M.nnz == 0
    with pytest.raises(CombBLASHipError):
        cb.SpDCCols.from_tuples(ctx, 4, 4, torch.tensor([4], device=DEV), torch.tensor([0], device=DEV),
                                torch.ones(1, dtype=torch.float64, device=DEV))


@pytest.mark.parametrize("name", ["sevenvertex", "small_nonsym"])
def test_readmm_to_device_and_multiply_matches_reference(ctx, fixtures, name):
    import combblas_amd as cb
    from combblas_amd.mm import ReadMM

    A = ReadMM(ctx, os.path.join(MM, f"{name}.mtx"))
    H.assert_dcsc_equal(_host(A), fixtures[f"{name}_A"])
    B = ReadMM(ctx, os.path.join(MM, f"{name}.mtx"))
    C = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, A, B)
    H.assert_dcsc_equal(_host(C), fixtures[f"{name}_C"], rtol=1e-12)


def test_readmm_symmetric_and_writemm_roundtrip(ctx, fixtures, tmp_path):
    from combblas_amd.mm import ReadMM, WriteMM, mmread

    lower = ReadMM(ctx, os.path.join(MM, "bcsstk01.mtx"), expand_symmetric=False)
    H.assert_dcsc_equal(_host(lower), fixtures["bcsstk01_A"])
    full = ReadMM(ctx, os.path.join(MM, "bcsstk01.mtx"))
    f = _host(full)
    dense = np.zeros((f.m, f.n))
    for j in range(f.nzc):
        dense[f.ir[f.cp[j]:f.cp[j + 1]], f.jc[j]] = f.num[f.cp[j]:f.cp[j + 1]]
    assert np.array_equal(dense, dense.T)
    p = str(tmp_path / "out.mtx")
    WriteMM(p, full)
    again = ReadMM(ctx, p)
    H.assert_dcsc_equal(_host(again), f)
    m, n, r, c, v, field, sym = mmread(p)
    assert (m, n, field, sym) == (48, 48, "real", "general") and r.size == f.nnz
