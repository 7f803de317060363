"""GPU parity at BASELINE config C2's FULL size: R-MAT scale-22 A^2 (24,766,243,778 outputs, more
than HBM, so phased) against the reference itself.

tests/golden/scale22.json holds the reference's own LocalHybridSpGEMM (mtSpGEMM.h:212-460) over the
whole product, run block by block in this container by tests/golden/make_golden_s22.py: nnz, value
sum and the order-sensitive digest of (global index, column, row, value bits) over all 24.8 G
entries in C order, for PlusTimes<int64> and PlusTimes<double> (multiplicity values, so the f64
sums are exact and bit-exactness is the bar for both). The device side computes the same digest
inside cbh_spgemm_phased (CBH_PHASE_CHECKSUM) as every phase is materialised in HBM. A second,
size-independent check: sum(C) = sum_k colsum_k(A) * rowsum_k(A)."""
import json
import os

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu

GOLD = os.path.join(H.GOLDEN, "scale22.json")


@pytest.fixture(scope="module")
def s22():
    import combblas_amd as cb

    with open(GOLD) as f:
        g = json.load(f)
    A = cb.rmat(22, 16, dtype=np.int64)
    return g, A


@pytest.mark.parametrize("tag", ["pt_i64", "pt_f64"])
def test_scale22_whole_product_bit_exact(ctx, s22, tag):
    import combblas_amd as cb

    g, A = s22
    dt = np.int64 if tag == "pt_i64" else np.float64
    dA = cb.SpDCCols.from_host(ctx, A, dtype=dt)
    dB = cb.SpDCCols.from_host(ctx, A, dtype=dt)
    st = cb.PhasedSpGEMM(cb.PlusTimesSRing, dA, dB, checksum=True, budget_bytes=0)
    dA.free()
    dB.free()
    tot = g[tag]["total"]
    assert st["nnz"] == tot["nnz"] == 24766243778
    assert st["flops"] == 57556482116
    closed = H.product_value_sum(H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))
    assert st["value_sum"] == tot["sum"] == float(closed)
    assert st["digest"] == int(tot["digest"]), f"{tag}: digest {st['digest']} != reference {tot['digest']}"


def test_scale22_first_block_bit_exact(ctx, s22):
    """C(:, 0:65536) = A * A(:, 0:65536): the CPU-baseline sample, pinned block-wise"""
    import combblas_amd as cb

    g, A = s22
    blk = g["pt_i64"]["blocks"][0]
    c0, c1 = blk["block"]
    keep = (A.jc >= c0) & (A.jc < c1)
    idx = np.nonzero(keep)[0]
    lens = np.diff(A.cp)[idx]
    starts = A.cp[idx]
    ent = np.concatenate([np.arange(s, s + l) for s, l in zip(starts, lens)]) if idx.size else np.zeros(0, np.int64)
    B = cb.HostDcsc(A.m, A.n, A.jc[idx], np.concatenate([[0], np.cumsum(lens)]), A.ir[ent], A.num[ent])
    dA, dB = cb.SpDCCols.from_host(ctx, A), cb.SpDCCols.from_host(ctx, B)
    st = cb.PhasedSpGEMM(cb.PlusTimesSRing, dA, dB, checksum=True, budget_bytes=0)
    assert blk["gbase"] == 0
    assert (st["nnz"], st["value_sum"], st["digest"]) == (blk["nnz"], blk["sum"], int(blk["digest"]))
