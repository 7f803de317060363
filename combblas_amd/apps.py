"""Host mirror of the callers around the SpGEMM hot path, all on the gfx950
kernels of combblas_amd/csrc/apps.h behind the C-ABI (no CPU path):

  MaskedSpGEMM(SR, A, B, M)   C = (A*B) .* M in one pass -- TC.cpp:108-110 (Mult_AnXBn_Synch then
                              EWiseMult(L, false)) fused; pattern=True keeps the semiring sums
  EWiseMult(A, B)             SpParMat::EWiseMult(B, false) -> Friends.h:834-887
  TriangleCount(L)            TC.cpp:108-115 on one block: sum of (L*L) .* L
  ColumnStats / Kselect /     the column operations of MCLPruneRecoverySelect (ParFriends.h:185-353),
  PruneColumn                 SpParMat::Kselect1 (SpParMat.cpp:1413-1700), Dcsc::PruneColumn
                              (dcsc.cpp:699-760)
The distributed MCLPruneRecoverySelect (process-column reductions) is in parfriends.py.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import CBH_MASK_DOT, CBH_MASK_EXPAND, CBH_MASK_PATTERN, check, lib
from .semirings import Semiring
from .spdccols import SpDCCols

DBL_MIN = 2.2250738585072014e-308  # std::numeric_limits<double>::min() (Kselect1, empty column)


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def MaskedSpGEMM(SR: Semiring, A: SpDCCols, B: SpDCCols, M: SpDCCols, pattern=False, method="auto") -> SpDCCols:
    """method: "expand" (products of A*B looked up in the mask column), "dot" (row i of A
    intersected with column j of B per mask entry), "auto" (dot from nnz(A) >= 65536)"""
    flags = (CBH_MASK_PATTERN if pattern else 0) | {"auto": 0, "expand": CBH_MASK_EXPAND, "dot": CBH_MASK_DOT}[method]
    h = ctypes.c_void_p()
    check(lib().cbh_spgemm_masked(A.ctx.h, SR.code, A.h, B.h, M.h, flags, ctypes.byref(h)), A.ctx.h)
    return SpDCCols(A.ctx, h)


def Transpose(A: SpDCCols) -> SpDCCols:
    """A' as a new device block (SpDCCols::Transpose), rows ascending in every column"""
    h = ctypes.c_void_p()
    check(lib().cbh_transpose(A.ctx.h, A.h, ctypes.byref(h)), A.ctx.h)
    return SpDCCols(A.ctx, h)


def EWiseMult(A: SpDCCols, B: SpDCCols) -> SpDCCols:
    h = ctypes.c_void_p()
    check(lib().cbh_ewise_mult(A.ctx.h, A.h, B.h, ctypes.byref(h)), A.ctx.h)
    return SpDCCols(A.ctx, h)


def TriangleCount(L: SpDCCols, L2: SpDCCols = None, method="auto") -> int:
    """TC.cpp:108-115: C = (L*L) .* L, triangles = sum(C). L2 is a second copy of L (the
    product's operands must not alias, ParFriends.h:172-179)."""
    from .semirings import PlusTimesSRing
    own = L2 is None
    if own:
        L2 = SpDCCols.from_tensors(L.ctx, L.m, L.n, *[t.clone() for t in L.tensors()])
    C = MaskedSpGEMM(PlusTimesSRing, L, L2, L, method=method)
    tri = int(C.tensors()[3].sum().item()) if C.nnz else 0
    C.free()
    if own:
        L2.free()
    return tri


def ColumnStats(A: SpDCCols, hard: float):
    """(nnz, nnz of v > hard, sum of v > hard) per column as f64 device vectors over A's columns"""
    dev = A.ctx.tdevice
    out = [torch.empty(A.n, dtype=torch.float64, device=dev) for _ in range(3)]
    check(lib().cbh_col_stats(A.ctx.h, A.h, ctypes.c_double(hard), *[_p(t) for t in out]), A.ctx.h)
    return tuple(out)


def ColumnStatsKept(A: SpDCCols, thresh):
    """(count, sum) per column of the entries PruneColumn(thresh) keeps (!(v < thresh[col])), as
    f64 device vectors -- the statistics of the pruned matrix without forming it"""
    dev = A.ctx.tdevice
    out = [torch.empty(A.n, dtype=torch.float64, device=dev) for _ in range(2)]
    check(lib().cbh_col_stats_kept(A.ctx.h, A.h, _p(thresh.contiguous()), *[_p(t) for t in out]), A.ctx.h)
    return tuple(out)


def kselect_cols(A: SpDCCols, aidx, nact, k):
    """Kselect1 of whole local columns, one launch: f64 per active index, DBL_MIN where the active
    column has no entries"""
    out = torch.full((nact,), 2.2250738585072014e-308, dtype=torch.float64, device=A.ctx.tdevice)
    check(lib().cbh_kselect_cols(A.ctx.h, A.h, _p(aidx), nact, int(k), _p(out)), A.ctx.h)
    return out


def kselect_hist(A: SpDCCols, aidx, nact, prefix, shift):
    hist = torch.empty(nact * 256, dtype=torch.int32, device=A.ctx.tdevice)
    check(lib().cbh_kselect_hist(A.ctx.h, A.h, _p(aidx), nact, _p(prefix), shift, _p(hist)), A.ctx.h)
    return hist


def kselect_pick(ctx, nact, hist, prefix, rank, shift):
    check(lib().cbh_kselect_pick(ctx.h, nact, _p(hist), _p(prefix), _p(rank), shift), ctx.h)


def kselect_value(ctx, nact, prefix):
    out = torch.empty(nact, dtype=torch.float64, device=ctx.tdevice)
    check(lib().cbh_kselect_value(ctx.h, nact, _p(prefix), _p(out)), ctx.h)
    return out


def PruneColumn(A: SpDCCols, thresh) -> SpDCCols:
    """entries with !(v < thresh[col]) kept (SpParMat::PruneColumn(pvals, std::less))"""
    h = ctypes.c_void_p()
    check(lib().cbh_prune_columns(A.ctx.h, A.h, _p(thresh.contiguous()), ctypes.byref(h)), A.ctx.h)
    return SpDCCols(A.ctx, h)


def MCLPruneBlock(A: SpDCCols, hard, selectNum, recoverNum, recoverPct) -> SpDCCols:
    """MCLPruneRecoverySelect (ParFriends.h:185-353) of a block holding its columns whole, in one
    C-ABI call (cbh_mcl_prune_recovery_select): statistics, Kselect1 of the recovery / selection
    columns, the recovery check after selection and PruneColumn on the device; A is kept"""
    h = ctypes.c_void_p()
    check(lib().cbh_mcl_prune_recovery_select(A.ctx.h, A.h, float(hard), int(selectNum), int(recoverNum),
                                              float(recoverPct), None, None, ctypes.byref(h)), A.ctx.h)
    return SpDCCols(A.ctx, h)


def TCLower(ctx, scale: int, edgefactor: int = 16, seed=None) -> SpDCCols:
    """Applications/TC.cpp:98-104,139-150 on the device: the packed Graph500 R-MAT edges (bit-identical
    to DEL->GenGraph500Data), RemoveLoops, Symmetricize (A += A'), Apply(1) and
    GetLowerTriangular -- L keeps every entry of the symmetric pattern, value 1 below the
    diagonal and an explicit 0 above it. The tuples are combined on the device
    (cbh_tuples_to_dcsc; duplicates OR'ed as bools, so every kept entry is exactly 0 or 1)."""
    from .rmat import DEFAULT_SEED, rmat_edges
    from .spdccols import _torch

    torch = _torch()
    src, dst = rmat_edges(scale, edgefactor, DEFAULT_SEED if seed is None else seed)
    dev = ctx.tdevice
    s, d = torch.from_numpy(src).to(dev), torch.from_numpy(dst).to(dev)
    del src, dst
    rows, cols = torch.cat([s, d]), torch.cat([d, s])
    del s, d
    n = 1 << scale
    P = SpDCCols.from_tuples(ctx, n, n, rows.to(torch.int32), cols, rows > cols, removeloops=True)
    del rows, cols
    cp, jc, ir, num = P.tensors()
    L = SpDCCols.from_tensors(ctx, n, n, cp.clone(), jc.clone(), ir.clone(), num.to(torch.int64))
    P.free()
    return L
