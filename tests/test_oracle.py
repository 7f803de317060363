"""CPU: pin the oracle (our C++ restatement) against fixtures produced by the reference itself
(tests/golden/make_golden.py -> oracle/_ref/ref_harness), and pin the R-MAT generator."""
import numpy as np
import pytest

import helpers as H

SEMIRING_TAGS = ["pt_f64", "pt_i64", "max_i64", "min_i64", "bool"]


@pytest.mark.parametrize("scale", [6, 8])
@pytest.mark.parametrize("tag", SEMIRING_TAGS)
def test_oracle_rmat_full(oracle, fixtures, scale, tag):
    A = fixtures[f"rmat{scale}_{tag}_A"]
    C = oracle.spgemm(A, A, H.SR_OF_TAG[tag], "hybrid")
    H.assert_dcsc_equal(C, fixtures[f"rmat{scale}_{tag}_C"], msg=f"rmat{scale} {tag}")


@pytest.mark.parametrize("kernel", ["hash", "hashu", "heap"])
def test_oracle_kernel_variants(oracle, fixtures, kernel):
    A = fixtures["rmat8_pt_i64_A"]
    C = oracle.spgemm(A, A, "plus_times", kernel)
    # hashu keeps the reference's hash-slot row order: compare exactly, unsorted
    H.assert_dcsc_equal(C, fixtures[f"rmat8_pt_i64_{kernel}_C"], msg=kernel)


@pytest.mark.parametrize("case", ["zeros8", "rect8", "largeseq", "sevenvertex", "small_nonsym", "bcsstk01"])
def test_oracle_reference_inputs(oracle, fixtures, case):
    A = fixtures[f"{case}_A"]
    B = fixtures.get(f"{case}_B", A)
    sr = "plus_times"
    C = oracle.spgemm(A, B, sr, "hybrid")
    H.assert_dcsc_equal(C, fixtures[f"{case}_C"], msg=case)
    if case == "zeros8":
        assert np.count_nonzero(C.num == 0) > 0, "explicit zeros must be kept"


@pytest.mark.parametrize("parts", [2, 3])
@pytest.mark.parametrize("tag", ["pt_i64", "pt_f64", "max_i64"])
def test_oracle_merge(oracle, fixtures, parts, tag):
    P = [fixtures[f"merge{parts}_{tag}_P{i}"] for i in range(parts)]
    M = oracle.merge(P, H.SR_OF_TAG[tag])
    H.assert_dcsc_equal(M, fixtures[f"merge{parts}_{tag}_M"], msg=f"merge{parts} {tag}")


def test_merge_equals_full_product(oracle, fixtures):
    # SUMMA identity the merge fixtures are built on: sum_k A(:,Kk) B(Kk,:) = A B
    M = fixtures["merge3_pt_i64_M"]
    A = fixtures["rmat8_pt_i64_A"]
    H.assert_dcsc_equal(M, oracle.spgemm(A, A, "plus_times"), msg="merge vs product")


def _gen(scale):
    import combblas_amd as cb

    A = cb.rmat(scale)
    return H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num)


@pytest.mark.parametrize("scale", [8, 10, 12, 14])
def test_generator_matches_reference(golden, scale):
    A = _gen(scale)
    g = golden["generator"][str(scale)]
    assert (A.nnz, A.nzc) == (g["nnz"], g["nzc"])
    vs, dg = H.digest(A)
    assert vs == g["sum"] and dg == int(g["digest"])


@pytest.mark.parametrize("scale", [10, 12])
@pytest.mark.parametrize("tag", SEMIRING_TAGS)
def test_oracle_digests(oracle, golden, scale, tag):
    A = H.values_for(tag, _gen(scale))
    C = oracle.spgemm(A, A, H.SR_OF_TAG[tag], "hybrid", threads=4)
    g = golden["digests"][f"rmat{scale}_{tag}"]
    vs, dg = H.digest(C)
    assert (C.nnz, C.nzc) == (g["nnz"], g["nzc"])
    assert vs == g["sum"] and dg == int(g["digest"])


def test_oracle_symbolic_known_answer(oracle, golden):
    # scale-14 A^2: exact nnz 6,471,508 (reference estimateNNZ_Hash)
    A = _gen(14)
    flops, nnz, _, _ = oracle.symbolic(A, A, threads=4)
    assert flops == 18786149
    assert nnz == golden["digests"]["rmat14_pt_i64"]["nnz"] == 6471508
