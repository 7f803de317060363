"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference's callers around the SpGEMM hot
path, used as the checker of the device kernels in combblas_amd/csrc/apps.h.
Nothing in the product imports this module. Pinned against the reference itself: the fixtures in
tests/golden/apps.npz come from oracle/_ref/ref_harness (tc / mcl / synch modes) built from the
reference sources (tests/golden/make_golden_apps.py), and tests/test_apps_oracle.py checks this
restatement against them.

  ewise_mult(A, B)                    Friends.h:834-887 EWiseMult(exclude=false): pattern
                                      intersection, values A*B, empty columns dropped
  column_stats(A, hard)               ParFriends.h:196-200: A.Reduce(Column, plus, 0, v->1),
                                      Prune(v <= hard) then Reduce(Column, plus) / count
  kselect1(values, k)                 SpParMat.cpp:1541-1687 (Kselect1): k-th largest, the
                                      smallest when fewer than k, numeric_limits<double>::min()
                                      for an empty column
  prune_column(A, thresh)             dcsc.cpp:699-760 PruneColumn(pvals, less): keep !(v < t)
  mcl_prune_recovery_select(A, ...)   ParFriends.h:185-353 (kselectVersion 1)

Operates on tests/helpers.Dcsc objects (host DCSC: m, n, jc, cp, ir, num).
"""
from __future__ import annotations

import numpy as np

DBL_MIN = np.finfo(np.float64).tiny  # std::numeric_limits<double>::min()


def _dcsc(m, n, cols, rows, vals):
    import helpers as H  # tests/ is on sys.path wherever this checker runs

    return H.Dcsc.from_coo(m, n, rows, cols, vals)


def ewise_mult(A, B):
    """C = A .* B: entries present in both, value A(i,j)*B(i,j) (Friends.h:871)."""
    ca, cb = A.cols(), B.cols()
    ka = ca.astype(np.int64) * A.m + A.ir
    kb = cb.astype(np.int64) * B.m + B.ir
    common, ia, ib = np.intersect1d(ka, kb, assume_unique=True, return_indices=True)
    vals = (A.num[ia] * B.num[ib]).astype(A.num.dtype)
    return _dcsc(A.m, A.n, common // A.m, common % A.m, vals)


def column_stats(A, hard):
    """(nnz, nnz of v > hard, sum of v > hard) per column, summed serially in storage order."""
    cols = A.cols()
    keep = A.num > hard
    cnt = np.bincount(cols, minlength=A.n).astype(np.float64)
    cntp = np.bincount(cols[keep], minlength=A.n).astype(np.float64)
    sump = np.bincount(cols[keep], weights=A.num[keep], minlength=A.n).astype(np.float64)
    return cnt, cntp, sump


def kselect1(values, k):
    if values.size == 0:
        return DBL_MIN
    s = np.sort(values)[::-1]
    return s[k - 1] if values.size >= k else s[-1]


def _kselect(A, mask, k, out):
    for j in np.nonzero(mask)[0]:
        i = np.searchsorted(A.jc, j)
        vals = A.num[A.cp[i]:A.cp[i + 1]] if i < A.nzc and A.jc[i] == j else A.num[:0]
        out[j] = kselect1(vals, k)


def prune_column(A, thresh):
    cols = A.cols()
    keep = ~(A.num < thresh[cols])
    return _dcsc(A.m, A.n, cols[keep], A.ir[keep], A.num[keep])


def mcl_prune_recovery_select(A, hardThreshold, selectNum, recoverNum, recoverPct):
    cnt, cntp, sump = column_stats(A, hardThreshold)  # nnzPerColumnUnpruned, nnzPerColumn, colSums
    prune = np.full(A.n, hardThreshold, np.float64)
    rec = (cntp < recoverNum) & (cnt > cntp) & (sump < recoverPct)
    if rec.any():
        _kselect(A, rec, recoverNum, prune)
    if selectNum > 0:
        sel = ~rec & (cntp > selectNum)
        if sel.any():
            _kselect(A, sel, selectNum, prune)
            if recoverNum > 0:
                S = prune_column(A, prune)
                _, cnt1, sum1 = column_stats(S, -np.inf)
                s2 = sel & (cnt1 < recoverNum) & (sum1 < recoverPct)
                if s2.any():
                    _kselect(A, s2, recoverNum, prune)
    return prune_column(A, prune)
