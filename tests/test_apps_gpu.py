"""gfx950 parity of the callers around the SpGEMM hot path (combblas_amd/csrc/apps.h through the
C-ABI), against the reference's own outputs (tests/golden/apps.npz, made by
tests/golden/make_golden_apps.py from oracle/_ref/ref_harness) and the numpy restatements of
oracle/apps_oracle.py:

  C4 TC        MaskedSpGEMM(L, L, mask L) == the reference's (L*L).*L, triangles bit-exact
               (Applications/TC.cpp:108-115)
  EWiseMult    Friends.h:834-887 on random operands with disjoint / shared column sets
  C5 MCL       column stats, radix Kselect (SpParMat.cpp:1413-1700), PruneColumn and the whole
               MCLPruneRecoverySelect (ParFriends.h:185-353) on the reference's expanded matrix
               -> the reference's pruned matrix bit for bit
  C3 Galerkin  T'(A T) with two LocalHybridSpGEMM -> the reference's SAT bit for bit (dyadic)
"""
import os
import sys

import numpy as np
import pytest

import helpers as H

sys.path.insert(0, os.path.join(H.REPO, "oracle"))
import apps_oracle as AO  # noqa: E402

pytestmark = pytest.mark.gpu


def _dev(ctx, d, dtype=None):
    import combblas_amd as cb

    return cb.SpDCCols.from_host(ctx, cb.HostDcsc(d.m, d.n, d.jc, d.cp, d.ir, d.num), dtype)


def _host(S):
    h = S.to_host()
    return H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num)


@pytest.mark.parametrize("method", ["expand", "dot"])
@pytest.mark.parametrize("scale", [8, 10])
def test_tc_masked_vs_reference(ctx, apps, apps_meta, scale, method):
    from combblas_amd.apps import MaskedSpGEMM, TriangleCount
    from combblas_amd.semirings import PlusTimesSRing

    L = apps[f"tc{scale}_L"]  # the reference's L: upper entries kept as explicit zeros (TC.cpp:98-104)
    dL, dL2 = _dev(ctx, L), _dev(ctx, L)
    C = MaskedSpGEMM(PlusTimesSRing, dL, dL2, dL, method=method)
    H.assert_dcsc_equal(_host(C), apps[f"tc{scale}_C"], msg=f"(L*L).*L scale {scale} {method}")
    assert TriangleCount(dL, dL2, method=method) == apps_meta["tc"][str(scale)]["triangles"]
    for S in (C, dL, dL2):
        S.free()


@pytest.mark.parametrize("scale,method", [(12, "expand"), (12, "dot"), (14, "dot"), (16, "dot")])
def test_tc_device_lower_vs_reference_digest(ctx, scale, method):
    """TC.cpp's whole flow on the device (TCLower: R-MAT -> L; masked (L*L).*L) against the
    reference's C at scales 12-16 (tests/golden/tc.json: nnz, nonzero columns, value sum =
    triangles, order-sensitive digest)"""
    import json

    from combblas_amd.apps import MaskedSpGEMM, TCLower
    from combblas_amd.semirings import PlusTimesSRing

    with open(os.path.join(H.GOLDEN, "tc.json")) as f:
        ref = json.load(f)["scales"][str(scale)]
    L = TCLower(ctx, scale)
    assert L.nnz == ref["nnzL"]
    L2 = TCLower(ctx, scale)
    C = MaskedSpGEMM(PlusTimesSRing, L, L2, L, method=method)
    c = _host(C)
    vs, dg = H.digest(c)
    assert (c.nnz, c.nzc) == (ref["nnzC"], ref["nzcC"])
    assert int(c.num.sum()) == ref["triangles"] and vs == ref["sumC"] and dg == int(ref["digestC"])
    for S in (C, L, L2):
        S.free()


@pytest.mark.parametrize("tag", ["pt_i64", "pt_f64", "max_i64", "min_i64", "bool"])
@pytest.mark.parametrize("pattern", [False, True])
@pytest.mark.parametrize("hub", [None, "0", "1"])
def test_masked_dot_vs_oracle(ctx, oracle, tag, pattern, hub, monkeypatch):
    """the dot form on a rectangular product with long rows of A and long columns of B (pieces of
    the wave kernel), every semiring, explicit zeros, empty mask columns; hub: the entries of the
    binary-search branch grouped by their longer list (apps.h hub groups: B's dense column 11 and A's
    dense rows 7 and 123) at the default group size (None: groups of 20-30 entries stay on the
    binary search), never ("0"), always ("1")"""
    from combblas_amd.apps import MaskedSpGEMM
    from combblas_amd.semirings import ALL

    if hub is not None:
        monkeypatch.setenv("CBH_DOT_HUB_MIN", hub)

    rng = np.random.default_rng(17)

    def vals(n):
        v = rng.integers(-3, 4, n)
        return {"pt_f64": v / 4.0, "bool": (v != 0).astype(np.uint8)}.get(tag, v.astype(np.int64))

    def with_lines(d, rows, cols):
        c0, r0, _ = d.to_coo_sorted()
        key = np.unique(np.concatenate([c0, cols]) * d.m + np.concatenate([r0, rows]))
        return H.Dcsc.from_coo(d.m, d.n, key % d.m, key // d.m, vals(key.size))

    # two dense rows of A and a dense column of B: shorter lists above the 2048-element piece
    a = with_lines(H.random_dcsc(rng, 300, 9000, 0.02), np.r_[np.full(9000, 7), np.full(9000, 123)],
                   np.r_[np.arange(9000), np.arange(9000)])
    b = with_lines(H.random_dcsc(rng, 9000, 200, 0.02), np.arange(0, 9000, 2), np.full(4500, 11))
    M = H.with_explicit_zeros(H.random_dcsc(rng, a.m, b.n, 0.1, dtype=a.num.dtype, empty_cols=0.3))
    sr = {"pt_i64": "plus_times", "pt_f64": "plus_times", "max_i64": "select_max", "min_i64": "min_plus",
          "bool": "or_and"}[tag]
    SR = ALL[{"pt_i64": "PlusTimesSRing", "pt_f64": "PlusTimesSRing", "max_i64": "SelectMaxSRing",
              "min_i64": "MinPlusSRing", "bool": "OrAndSRing"}[tag]]
    mask = H.Dcsc(M.m, M.n, M.jc, M.cp, M.ir, np.ones(M.nnz, a.num.dtype)) if pattern else M
    exp = AO.ewise_mult(oracle.spgemm(a, b, sr, "hybrid"), mask)
    dA, dB, dM = _dev(ctx, a), _dev(ctx, b), _dev(ctx, M)
    C = MaskedSpGEMM(SR, dA, dB, dM, pattern=pattern, method="dot")
    H.assert_dcsc_equal(_host(C), exp, rtol=1e-12 if tag == "pt_f64" else 0.0, msg=f"masked dot {tag}")
    for S in (C, dA, dB, dM):
        S.free()


def test_transpose_vs_host(ctx):
    from combblas_amd.apps import Transpose

    rng = np.random.default_rng(4)
    a = H.random_dcsc(rng, 333, 217, 0.05, dtype=np.float64, empty_cols=0.2)
    T = _host(Transpose(_dev(ctx, a)))
    c, r, v = a.to_coo_sorted()
    H.assert_dcsc_equal(T, H.Dcsc.from_coo(a.n, a.m, c, r, v), msg="transpose")


def test_tc_known_answer_scale10(ctx, apps):
    from combblas_amd.apps import TriangleCount

    dL = _dev(ctx, apps["tc10_L"])
    assert TriangleCount(dL) == 78452  # TC.cpp at scale 10
    dL.free()


@pytest.mark.parametrize("tag", ["pt_i64", "pt_f64", "max_i64", "min_i64", "bool"])
@pytest.mark.parametrize("pattern", [False, True])
def test_masked_semirings_vs_oracle(ctx, oracle, tag, pattern):
    """(A*B) .* M over every semiring, with a random mask holding explicit zeros, whole empty
    columns and columns of M absent from B; pattern=True keeps the semiring sums."""
    import combblas_amd as cb
    from combblas_amd.apps import MaskedSpGEMM
    from combblas_amd.semirings import ALL

    A = cb.rmat(9)
    a = H.values_for(tag, H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))
    rng = np.random.default_rng(11)
    M = H.random_dcsc(rng, a.m, a.n, 0.05, dtype=a.num.dtype, empty_cols=0.3)
    M = H.with_explicit_zeros(M)
    sr = {"pt_i64": "plus_times", "pt_f64": "plus_times", "max_i64": "select_max", "min_i64": "min_plus",
          "bool": "or_and"}[tag]
    SR = ALL[{"pt_i64": "PlusTimesSRing", "pt_f64": "PlusTimesSRing", "max_i64": "SelectMaxSRing",
              "min_i64": "MinPlusSRing", "bool": "OrAndSRing"}[tag]]
    full = oracle.spgemm(a, a, sr, "hybrid")
    mask = H.Dcsc(M.m, M.n, M.jc, M.cp, M.ir, np.ones(M.nnz, a.num.dtype)) if pattern else M
    exp = AO.ewise_mult(full, mask)
    dA, dB, dM = _dev(ctx, a), _dev(ctx, a), _dev(ctx, M)
    C = MaskedSpGEMM(SR, dA, dB, dM, pattern=pattern)
    H.assert_dcsc_equal(_host(C), exp, rtol=1e-12 if tag == "pt_f64" else 0.0, msg=f"masked {tag}")
    for S in (C, dA, dB, dM):
        S.free()


def test_masked_long_mask_columns(ctx, oracle):
    """mask columns longer than the kernel's LDS chunk (MCAP=2048): a dense-ish mask on a tall A"""
    from combblas_amd.apps import MaskedSpGEMM
    from combblas_amd.semirings import PlusTimesSRing

    rng = np.random.default_rng(5)
    a = H.random_dcsc(rng, 20000, 300, 0.02, dtype=np.int64)
    b = H.random_dcsc(rng, 300, 40, 0.3, dtype=np.int64)
    M = H.random_dcsc(rng, 20000, 40, 0.4, dtype=np.int64, empty_cols=0.1)
    exp = AO.ewise_mult(oracle.spgemm(a, b, "plus_times", "hybrid"), M)
    dA, dB, dM = _dev(ctx, a), _dev(ctx, b), _dev(ctx, M)
    C = MaskedSpGEMM(PlusTimesSRing, dA, dB, dM)
    H.assert_dcsc_equal(_host(C), exp, msg="masked, long mask columns")
    for S in (C, dA, dB, dM):
        S.free()


def test_masked_empty_operands(ctx):
    from combblas_amd.apps import MaskedSpGEMM
    from combblas_amd.semirings import PlusTimesSRing

    rng = np.random.default_rng(2)
    a = H.random_dcsc(rng, 50, 50, 0.1)
    z = H.Dcsc(50, 50, np.zeros(0, np.int64), np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0))
    for x, y, m in ((a, a, z), (z, a, a), (a, z, a)):
        C = MaskedSpGEMM(PlusTimesSRing, _dev(ctx, x), _dev(ctx, y), _dev(ctx, m))
        assert C.nnz == 0 and (C.m, C.n) == (50, 50)


@pytest.mark.parametrize("dt", [np.float64, np.int64, np.float32, np.int32])
def test_ewise_mult_vs_oracle(ctx, dt):
    from combblas_amd.apps import EWiseMult

    rng = np.random.default_rng(3)
    a = H.random_dcsc(rng, 700, 500, 0.03, dtype=dt, empty_cols=0.4)
    b = H.random_dcsc(rng, 700, 500, 0.03, dtype=dt, empty_cols=0.4)
    # make the intersection non-trivial: b shares half of a's entries
    keep = rng.random(a.nnz) < 0.5
    rows = np.concatenate([b.to_coo_sorted()[0], a.ir[keep].astype(np.int64)])
    cols = np.concatenate([b.to_coo_sorted()[1], a.cols()[keep]])
    vals = np.concatenate([b.to_coo_sorted()[2], a.num[keep] + 1]).astype(dt)
    key, first = np.unique(cols * a.m + rows, return_index=True)
    b = H.Dcsc.from_coo(a.m, a.n, key % a.m, key // a.m, vals[first])
    dA, dB = _dev(ctx, a), _dev(ctx, b)
    C = EWiseMult(dA, dB)
    H.assert_dcsc_equal(_host(C), AO.ewise_mult(a, b), msg=f"ewise {dt.__name__}")


def test_column_stats_vs_oracle(ctx, apps):
    from combblas_amd.apps import ColumnStats

    A2 = apps["mcl_A2"]
    for hard in (0.0, 0.005, 0.05, float("-inf")):
        got = [t.cpu().numpy() for t in ColumnStats(_dev(ctx, A2), hard)]
        exp = AO.column_stats(A2, hard)
        np.testing.assert_array_equal(got[0], exp[0])
        np.testing.assert_array_equal(got[1], exp[1])
        np.testing.assert_allclose(got[2], exp[2], rtol=1e-12, atol=0)  # summation order differs


def test_kselect_edge_cases(ctx):
    """k-th largest per column: ties, negatives, signed zeros, columns shorter than k (-> smallest),
    empty active columns (-> numeric_limits<double>::min()), inactive columns (NaN)"""
    import torch

    from combblas_amd import parfriends as pf
    from combblas_amd.backend import HipBackend

    rng = np.random.default_rng(1)
    cols = [[3.0, 1.0, 2.0], [5.0, 5.0, 5.0, 1.0], [-1.0, -7.5, 0.0, -0.0, 2.5], [4.0], [], [9.0, 8.0],
            list(rng.standard_normal(3000)), list(rng.standard_normal(5000)),  # LDS-staged / re-read from HBM
            list(np.round(rng.standard_normal(6000), 1)),  # many ties
            list(rng.uniform(0.001, 0.01, 2500)),  # common sign/exponent bits (the digits start below them)
            [1.0, np.nextafter(1.0, 2.0), 1.0, np.nextafter(1.0, 2.0), np.nextafter(1.0, 0.0)],  # last-bit keys
            list(rng.uniform(0.0, 1.0, 9000)),  # 1024-thread workgroup
            list(np.round(rng.uniform(0.0, 1.0, 40000), 3))]  # chunked over workgroups (ties too)
    rows, cc, vv = [], [], []
    for j, c in enumerate(cols):
        rows += list(range(len(c)))
        cc += [j] * len(c)
        vv += c
    d = H.Dcsc.from_coo(40000, len(cols), np.array(rows), np.array(cc), np.array(vv, np.float64))
    dA = _dev(ctx, d)

    class MultiPass:  # the backend without the one-launch select: the per-pass histogram path
        def __init__(self, be):
            self.be = be

        def __getattr__(self, name):
            if name == "kselect_cols":
                raise AttributeError(name)
            return getattr(self.be, name)

    for be in (HipBackend(ctx), MultiPass(HipBackend(ctx))):
        for k in (1, 2, 3, 5, 100, 4500, 7000, 8500, 39000):
            active = torch.tensor([True, True, True, True, True, False, True, True, True, True, True, True, True],
                                  device=ctx.tdevice)
            got = pf.Kselect(be, dA, active, k).cpu().numpy()
            for j, c in enumerate(cols):
                if not bool(active[j]):
                    assert np.isnan(got[j])
                else:
                    assert got[j] == AO.kselect1(np.array(c, np.float64), k), (type(be).__name__, k, j)


def test_column_stats_kept_vs_oracle(ctx, apps):
    """count / sum of what PruneColumn keeps, without forming it = the stats of the pruned matrix"""
    import torch

    from combblas_amd.apps import ColumnStatsKept

    A2 = apps["mcl_A2"]
    rng = np.random.default_rng(3)
    for t in (np.full(A2.n, 0.01), rng.uniform(0.0, 0.05, A2.n), np.full(A2.n, -np.inf)):
        got = [x.cpu().numpy() for x in ColumnStatsKept(_dev(ctx, A2), torch.tensor(t, device=ctx.tdevice))]
        _, cnt, sm = AO.column_stats(AO.prune_column(A2, t), -np.inf)
        np.testing.assert_array_equal(got[0], cnt)
        np.testing.assert_allclose(got[1], sm, rtol=1e-12, atol=0)


@pytest.mark.parametrize("i", [0, 1])
def test_mcl_prune_vs_reference(ctx, apps, apps_meta, i):
    """MCLPruneRecoverySelect of the reference's expanded matrix, on device -> the reference's
    pruned matrix, bit for bit (hard threshold, select and both recovery steps exercised)"""
    from combblas_amd import parfriends as pf
    from combblas_amd.backend import HipBackend

    p = apps_meta["mcl"][str(i)]
    be = HipBackend(ctx)
    out = pf._mcl_block(be, _dev(ctx, apps["mcl_A2"]), None, p["hard"], p["select"], p["recover"], p["pct"])
    H.assert_dcsc_equal(_host(out), apps[f"mcl_out{i}"], msg=f"MCL prune params {i}")


def test_mcl_expand_and_prune_vs_reference(ctx, apps, apps_meta):
    """the expansion on the hot path then the prune: A^2 within 1e-12 of the reference's and the
    pruned pattern identical to the oracle prune of the device A^2"""
    import combblas_amd as cb
    from combblas_amd import parfriends as pf
    from combblas_amd.backend import HipBackend

    A = apps["mcl_A"]
    C = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, _dev(ctx, A), _dev(ctx, A))
    got = _host(C)
    ref = apps["mcl_A2"]
    assert np.array_equal(got.jc, ref.jc) and np.array_equal(got.cp, ref.cp) and np.array_equal(got.ir, ref.ir)
    np.testing.assert_allclose(got.num, ref.num, rtol=1e-12, atol=0)
    p = apps_meta["mcl"]["0"]
    out = pf._mcl_block(HipBackend(ctx), C, None, p["hard"], p["select"], p["recover"], p["pct"])
    H.assert_dcsc_equal(_host(out), AO.mcl_prune_recovery_select(got, p["hard"], p["select"], p["recover"],
                                                                  p["pct"]), msg="MCL expand+prune")


def test_prune_columns_vs_oracle(ctx, apps):
    import torch

    from combblas_amd.apps import PruneColumn

    A2 = apps["mcl_A2"]
    th = np.random.default_rng(4).uniform(0, 0.05, A2.n)
    th[::7] = -np.inf  # keep everything
    th[::11] = np.inf  # drop everything
    out = PruneColumn(_dev(ctx, A2), torch.from_numpy(th).to(ctx.tdevice))
    H.assert_dcsc_equal(_host(out), AO.prune_column(A2, th), msg="PruneColumn")


def test_galerkin_vs_reference(ctx, apps):
    import combblas_amd as cb

    AT = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, _dev(ctx, apps["gal_A"]), _dev(ctx, apps["gal_T"]))
    H.assert_dcsc_equal(_host(AT), apps["gal_AT"], msg="A*T")
    SAT = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, _dev(ctx, apps["gal_S"]), AT)
    H.assert_dcsc_equal(_host(SAT), apps["gal_SAT"], msg="T'*(A*T)")
