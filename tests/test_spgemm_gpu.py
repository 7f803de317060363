"""GPU parity: the gfx950 SpGEMM / merge kernels (through the C-ABI) against
  * fixtures produced by the reference itself (tests/golden, exact structure + bit-exact values),
  * digests of reference outputs at larger R-MAT scales (golden.json),
  * the CPU oracle on seeded random / adversarial inputs (empty, ragged, wide, clustered).
Integer and boolean semirings must be bit-exact; f64 PlusTimes inputs here are dyadic, so they
are bit-exact too; the one genuinely rounding case (largeseq) uses rtol 1e-12 (north star)."""
import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu

SEMIRING_TAGS = ["pt_f64", "pt_i64", "max_i64", "min_i64", "bool"]
RTOL_F64 = 1e-12  # BASELINE.json north star: within 1e-12 relative for double PlusTimes


def SR(tag_or_name):
    import combblas_amd as cb

    name = H.SR_OF_TAG.get(tag_or_name, tag_or_name)
    return {"plus_times": cb.PlusTimesSRing, "select_max": cb.SelectMaxSRing, "min_plus": cb.MinPlusSRing,
            "or_and": cb.OrAndSRing}[name]


def dev(ctx, d: H.Dcsc):
    import combblas_amd as cb

    return cb.SpDCCols.from_host(ctx, cb.HostDcsc(d.m, d.n, d.jc, d.cp, d.ir, d.num))


def host(C) -> H.Dcsc:
    h = C.to_host()
    return H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num)


def gpu_mult(ctx, A, B, sr="plus_times"):
    import combblas_amd as cb

    dA, dB = dev(ctx, A), dev(ctx, B)
    C = cb.LocalHybridSpGEMM(SR(sr), dA, dB)
    return host(C)


@pytest.mark.parametrize("scale", [6, 8])
@pytest.mark.parametrize("tag", SEMIRING_TAGS)
def test_rmat_vs_reference(ctx, fixtures, scale, tag):
    A = fixtures[f"rmat{scale}_{tag}_A"]
    C = gpu_mult(ctx, A, A, tag)
    H.assert_dcsc_equal(C, fixtures[f"rmat{scale}_{tag}_C"], msg=f"rmat{scale} {tag}")


@pytest.mark.parametrize("kernel", ["hash", "hashu", "heap"])
def test_kernel_variants_vs_reference(ctx, fixtures, kernel):
    import combblas_amd as cb

    A = fixtures["rmat8_pt_i64_A"]
    f = {"hash": lambda a, b: cb.LocalSpGEMMHash(cb.PlusTimesSRing, a, b, sort=True),
         "hashu": lambda a, b: cb.LocalSpGEMMHash(cb.PlusTimesSRing, a, b, sort=False),
         "heap": lambda a, b: cb.LocalSpGEMM(cb.PlusTimesSRing, a, b)}[kernel]
    C = host(f(dev(ctx, A), dev(ctx, A)))
    H.assert_dcsc_equal(C, fixtures[f"rmat8_pt_i64_{kernel}_C"], sorted_rows=(kernel != "hashu"), msg=kernel)


@pytest.mark.parametrize("case", ["zeros8", "rect8", "sevenvertex", "small_nonsym", "bcsstk01"])
def test_reference_inputs(ctx, fixtures, case):
    A = fixtures[f"{case}_A"]
    B = fixtures.get(f"{case}_B", A)
    C = gpu_mult(ctx, A, B)
    H.assert_dcsc_equal(C, fixtures[f"{case}_C"], rtol=0.0 if case in ("zeros8", "rect8") else RTOL_F64, msg=case)
    if case == "zeros8":
        assert np.count_nonzero(C.num == 0) > 0


def test_largeseq_signed_doubles(ctx, fixtures):
    # genuine f64 rounding: summation order may differ from the reference's -> 1e-12 relative
    C = gpu_mult(ctx, fixtures["largeseq_A"], fixtures["largeseq_B"])
    H.assert_dcsc_equal(C, fixtures["largeseq_C"], rtol=RTOL_F64, msg="largeseq")


@pytest.mark.parametrize("parts", [2, 3])
@pytest.mark.parametrize("tag", ["pt_i64", "pt_f64", "max_i64"])
def test_multiway_merge_vs_reference(ctx, fixtures, parts, tag):
    import combblas_amd as cb

    P = [dev(ctx, fixtures[f"merge{parts}_{tag}_P{i}"]) for i in range(parts)]
    M = host(cb.MultiwayMerge(SR(tag), P, P[0].m, P[0].n))
    H.assert_dcsc_equal(M, fixtures[f"merge{parts}_{tag}_M"], msg=f"merge{parts} {tag}")


def test_merge_single_list_is_copy(ctx, fixtures):
    import combblas_amd as cb

    P = dev(ctx, fixtures["merge2_pt_i64_P0"])
    M = host(cb.MultiwayMerge(cb.PlusTimesSRing, [P]))
    H.assert_dcsc_equal(M, fixtures["merge2_pt_i64_P0"])


def _gen(scale):
    import combblas_amd as cb

    A = cb.rmat(scale)
    return H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num)


@pytest.mark.parametrize("scale", [10, 12])
@pytest.mark.parametrize("tag", SEMIRING_TAGS)
def test_rmat_digest_vs_reference(ctx, golden, scale, tag):
    A = H.values_for(tag, _gen(scale))
    C = gpu_mult(ctx, A, A, tag)
    g = golden["digests"][f"rmat{scale}_{tag}"]
    assert (C.nnz, C.nzc) == (g["nnz"], g["nzc"])
    vs, dg = H.digest(C)
    assert vs == g["sum"] and dg == int(g["digest"])


@pytest.mark.parametrize("scale", [14, 16])
def test_rmat_large_digest_vs_reference(ctx, golden, scale):
    # scale-16 A^2 is the reference's C1 config: nnz 53,638,834, sum 334,648,807
    A = _gen(scale)
    C = gpu_mult(ctx, A, A, "plus_times")
    g = golden["digests"][f"rmat{scale}_pt_i64"]
    assert (C.nnz, C.nzc) == (g["nnz"], g["nzc"])
    vs, dg = H.digest(C)
    assert vs == g["sum"] and dg == int(g["digest"])


def test_symbolic_known_answer(ctx):
    import combblas_amd as cb

    A = dev(ctx, _gen(14))
    B = dev(ctx, _gen(14))
    assert cb.estimateFLOPandNNZ(A, B) == (18786149, 6471508)


# ------------------------------------------------------------------ oracle-checked edge cases
def test_empty_operands(ctx):
    import combblas_amd as cb

    A = H.random_dcsc(np.random.default_rng(1), 50, 40, 0.1)
    Z = H.Dcsc(40, 30, [], [0], [], np.zeros(0))
    C = host(cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dev(ctx, A), dev(ctx, Z)))
    assert (C.m, C.n, C.nnz, C.nzc) == (50, 30, 0, 0)
    Z2 = H.Dcsc(50, 50, [], [0], [], np.zeros(0))
    C = host(cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dev(ctx, Z2), dev(ctx, A)))
    assert (C.m, C.n, C.nnz) == (50, 40, 0)


def test_dimension_mismatch_raises(ctx):
    import combblas_amd as cb
    from combblas_amd._lib import CombBLASHipError

    A = H.random_dcsc(np.random.default_rng(2), 20, 30, 0.2)
    with pytest.raises(CombBLASHipError) as e:
        cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dev(ctx, A), dev(ctx, A))
    assert e.value.code == 3002


@pytest.mark.parametrize("seed,m,k,n,dens", [(3, 1, 1, 1, 1.0), (4, 300, 200, 150, 0.02), (5, 2000, 1000, 300, 0.01),
                                              (6, 5000, 5000, 50, 0.002), (7, 64, 3000, 64, 0.05)])
@pytest.mark.parametrize("tag", ["pt_f64", "pt_i64", "max_i64", "min_i64", "bool"])
def test_random_vs_oracle(ctx, oracle, seed, m, k, n, dens, tag):
    rng = np.random.default_rng(seed)
    dt = {"pt_f64": np.float64, "bool": np.uint8}.get(tag, np.int64)
    A = H.random_dcsc(rng, m, k, dens, dt, empty_cols=0.2)
    B = H.random_dcsc(rng, k, n, dens * 2, dt, empty_cols=0.2)
    sr = H.SR_OF_TAG[tag]
    H.assert_dcsc_equal(gpu_mult(ctx, A, B, sr), oracle.spgemm(A, B, sr), msg=f"{tag} {m}x{k}x{n}")


def test_wide_column_chunked_entries(ctx, oracle):
    # B columns with thousands of entries (> EMAX=512 entries per LDS chunk) and many row tiles
    rng = np.random.default_rng(11)
    m = k = 20000
    A = H.random_dcsc(rng, m, k, 0.0008, np.int64)
    rows = rng.choice(k, 6000, replace=False)
    B = H.Dcsc.from_coo(k, 3, np.concatenate([rows, rows[:100], [5]]), np.concatenate(
        [np.zeros(6000, int), np.ones(100, int), [2]]), np.ones(6101, np.int64))
    B = H.Dcsc.from_coo(B.m, B.n, *[x for x in (B.ir, B.cols(), B.num)])
    H.assert_dcsc_equal(gpu_mult(ctx, A, B), oracle.spgemm(A, B, "plus_times"), msg="wide")


def test_clustered_rows_force_tile_splits(ctx, oracle):
    # banded / clustered rows: the order-preserving hash sees long runs -> tiles are halved
    m = 100000
    rows, cols = [], []
    for j in range(40):
        base = (j * 977) % (m - 5000)
        r = base + np.arange(0, 3000 * (1 + j % 3), 1 + j % 3)
        r = r[r < m]
        rows.append(r)
        cols.append(np.full(r.size, j))
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    A = H.Dcsc.from_coo(m, 40, rows, cols, (rows % 7 + 1).astype(np.int64))
    B = H.Dcsc.from_coo(40, 8, np.arange(40), np.arange(40) % 8, np.ones(40, np.int64))
    H.assert_dcsc_equal(gpu_mult(ctx, A, B), oracle.spgemm(A, B, "plus_times"), msg="clustered")


def test_dense_band_heavy_column(ctx, oracle):
    # a column whose output fills a contiguous row range densely (worst case for clustering)
    m = 30000
    A = H.Dcsc.from_coo(m, 2, np.concatenate([np.arange(10000, 30000), np.arange(0, 30000, 3)]),
                        np.concatenate([np.zeros(20000, int), np.ones(10000, int)]), np.ones(30000, np.int64))
    B = H.Dcsc.from_coo(2, 1, [0, 1], [0, 0], np.array([2, 3], np.int64))
    H.assert_dcsc_equal(gpu_mult(ctx, A, B), oracle.spgemm(A, B, "plus_times"), msg="band")


def test_phased_matches_oracle_digest(ctx, oracle):
    import combblas_amd as cb

    A = H.values_for("pt_i64", _gen(12))
    exp = oracle.spgemm(A, A, "plus_times", threads=4)
    vs, dg = H.digest(exp)
    dA, dB = dev(ctx, A), dev(ctx, A)
    for budget in (None, 64 * 1024, 1 << 20):  # force many phases
        st = cb.PhasedSpGEMM(cb.PlusTimesSRing, dA, dB, checksum=True, budget_bytes=budget or 0)
        assert st["nnz"] == exp.nnz and st["value_sum"] == vs and st["digest"] == dg, (budget, st)
        if budget == 64 * 1024:
            assert st["phases"] > 10


def test_torch_tensors_view_results(ctx, fixtures):
    import torch
    import combblas_amd as cb

    A = fixtures["rmat8_pt_i64_A"]
    C = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dev(ctx, A), dev(ctx, A))
    cp, jc, ir, num = C.tensors()
    assert cp.device.type == "cuda" and num.dtype == torch.int64
    exp = fixtures["rmat8_pt_i64_C"]
    np.testing.assert_array_equal(ir.cpu().numpy(), exp.ir)
    C2 = cb.SpDCCols.from_tensors(ctx, C.m, C.n, cp.clone(), jc.clone(), ir.clone(), num.clone())
    H.assert_dcsc_equal(host(C2), exp)


def test_plan_phase_slices_match_column_products(ctx):
    """SpGEMMPlan (cbh_plan_col_nnz / cbh_plan_spgemm_slots): one symbolic pass, then C = A*B(:, c0:c1)
    per phase equals cbh_spgemm on the column slice, with and without CBH_KEEP_EMPTY_COLS, and the
    per-slot nnz equals the symbolic pass's."""
    import combblas_amd as cb
    from combblas_amd._lib import CBH_KEEP_EMPTY_COLS
    from combblas_amd.backend import HipBackend
    from combblas_amd.parfriends import _colslice

    A = H.values_for("pt_i64", _gen(11))
    dA, dB = dev(ctx, A), dev(ctx, A)
    be = HipBackend(ctx)
    plan = cb.SpGEMMPlan(dA, dB)
    try:
        ref_nnz = cb.estimateFLOPandNNZ(dA, dB, per_column=True)[3]
        assert bool((plan.col_nnz() == ref_nnz).all().item())
        n = A.n
        cuts = [0, 1, 700, 701, n // 2, n // 2 + 333, n]
        for c0, c1 in zip(cuts[:-1], cuts[1:]):
            got = plan.multiply(cb.PlusTimesSRing, c0, c1)
            exp = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dA, _colslice(be, dB, c0, c1))
            H.assert_dcsc_equal(host(got), host(exp), msg=f"cols [{c0},{c1})")
        s1 = dB.nzc // 3
        keep = plan.multiply_slots(cb.PlusTimesSRing, 0, s1, flags=CBH_KEEP_EMPTY_COLS)
        assert keep.nzc == s1
        empty = plan.multiply_slots(cb.PlusTimesSRing, 5, 5)
        assert empty.nnz == 0
    finally:
        plan.close()
