"""CPU checks of the application-level oracle (oracle/apps_oracle.py) and of the host input
generators against the reference's own outputs (tests/golden/apps.npz, made by
tests/golden/make_golden_apps.py from oracle/_ref/ref_harness):

  C4 TC        Applications/TC.cpp:62-121   L with explicit zeros, C = (L*L) .* L, triangles
  C5 MCL       ParFriends.h:185-353          MCLPruneRecoverySelect on the expanded matrix
  C3 Galerkin  GalerkinNew.cpp:100-106       SAT = T' * (A * T)
"""
import os
import sys

import numpy as np
import pytest

import helpers as H

sys.path.insert(0, os.path.join(H.REPO, "oracle"))
import apps_oracle as AO  # noqa: E402


def tc_lower(scale):
    """TC.cpp:98-104 on the host: RemoveLoops, A += A', values 1, upper entries kept as zeros"""
    import combblas_amd as cb

    A = cb.rmat(scale)
    d = H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num)
    r, c = d.ir.astype(np.int64), d.cols()
    keep = r != c
    r, c = r[keep], c[keep]
    key = np.unique(np.concatenate([c * d.m + r, r * d.m + c]))
    rows, cols = key % d.m, key // d.m
    vals = (rows > cols).astype(np.int64)
    return H.Dcsc.from_coo(d.m, d.n, rows, cols, vals)


@pytest.mark.parametrize("scale", [8, 10])
def test_tc_oracle_vs_reference(apps, apps_meta, oracle, scale):
    L = tc_lower(scale)
    H.assert_dcsc_equal(L, apps[f"tc{scale}_L"], msg="L")
    C = AO.ewise_mult(oracle.spgemm(L, L, "plus_times", "hybrid"), L)
    H.assert_dcsc_equal(C, apps[f"tc{scale}_C"], msg="(L*L).*L")
    assert int(C.num.sum()) == apps_meta["tc"][str(scale)]["triangles"]


def test_tc_known_answer(apps_meta):
    assert apps_meta["tc"]["10"]["triangles"] == 78452  # TC.cpp at scale 10, 1 rank


def test_mcl_generator_deterministic(apps, apps_meta):
    from combblas_amd.mclgen import planted_partition

    inp = apps_meta["mcl"]["input"]
    h = planted_partition(inp["n"], inp["avg_deg"], inp["seed"])
    H.assert_dcsc_equal(H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num), apps["mcl_A"], msg="generator")
    colsum = np.bincount(apps["mcl_A"].cols(), weights=apps["mcl_A"].num)
    np.testing.assert_allclose(colsum, 1.0, rtol=1e-12)


def test_mcl_expansion_oracle(apps, oracle):
    A = apps["mcl_A"]
    C = oracle.spgemm(A, A, "plus_times", "hybrid")
    R = apps["mcl_A2"]
    assert np.array_equal(C.jc, R.jc) and np.array_equal(C.cp, R.cp) and np.array_equal(C.ir, R.ir)
    np.testing.assert_allclose(C.num, R.num, rtol=1e-12, atol=0)


@pytest.mark.parametrize("i", [0, 1])
def test_mcl_prune_oracle_vs_reference(apps, apps_meta, i):
    p = apps_meta["mcl"][str(i)]
    out = AO.mcl_prune_recovery_select(apps["mcl_A2"], p["hard"], p["select"], p["recover"], p["pct"])
    H.assert_dcsc_equal(out, apps[f"mcl_out{i}"], msg=f"mcl params {i}")


def test_kselect1_contract():
    assert AO.kselect1(np.array([3.0, 1.0, 2.0]), 2) == 2.0
    assert AO.kselect1(np.array([3.0, 1.0]), 5) == 1.0  # fewer than k: the smallest
    assert AO.kselect1(np.array([]), 5) == np.finfo(np.float64).tiny  # empty: numeric_limits::min()


def test_galerkin_inputs_and_oracle(apps, oracle):
    from combblas_amd.galerkin import poisson27, prolongation, transpose

    d = lambda h: H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num)  # noqa: E731
    A, T = d(poisson27(8)), d(prolongation(8))
    S = d(transpose(prolongation(8)))
    H.assert_dcsc_equal(A, apps["gal_A"], msg="A")
    H.assert_dcsc_equal(T, apps["gal_T"], msg="T")
    H.assert_dcsc_equal(S, apps["gal_S"], msg="S")
    AT = oracle.spgemm(A, T, "plus_times", "hybrid")
    SAT = oracle.spgemm(S, AT, "plus_times", "hybrid")
    H.assert_dcsc_equal(SAT, apps["gal_SAT"], msg="SAT")  # dyadic values: exact


@pytest.mark.parametrize("nx", [4, 8, 16])
def test_galerkin_column_order_generators(nx):
    """the sort-free generators bench_galerkin.py uses at 256^3 build exactly the pinned operators"""
    from combblas_amd.galerkin import poisson27, poisson27_csc, prolongation, prolongation_csc

    for slow, fast in ((poisson27(nx), poisson27_csc(nx)), (prolongation(nx), prolongation_csc(nx))):
        H.assert_dcsc_equal(H.Dcsc(fast.m, fast.n, fast.jc, fast.cp, fast.ir, fast.num),
                            H.Dcsc(slow.m, slow.n, slow.jc, slow.cp, slow.ir, slow.num), msg=f"nx {nx}")


def test_galerkin_closed_form_sum(oracle):
    """sum(R^T A R) = (R 1)^T A (R 1): the size-independent check of the C3 bench line"""
    from bench_galerkin import closed_form_sum
    from combblas_amd.galerkin import poisson27_csc, prolongation_csc, transpose

    A, R = poisson27_csc(8), prolongation_csc(8)
    S = transpose(R)
    d = lambda h: H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num)  # noqa: E731
    SAT = oracle.spgemm(d(S), oracle.spgemm(d(A), d(R), "plus_times", "hybrid"), "plus_times", "hybrid")
    assert float(SAT.num.sum()) == closed_form_sum(A, R)
