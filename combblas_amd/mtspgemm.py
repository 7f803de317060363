"""Host mirror of the reference's local SpGEMM interface (include/CombBLAS/mtSpGEMM.h,
include/CombBLAS/MultiwayMerge.h). Same names, argument meaning and ownership rules; every call
runs on the gfx950 kernels behind the C-ABI (no CPU path).

Differences that follow from the device layout (documented in DESIGN.md §1):
  * results are device DCSC blocks (SpDCCols) instead of SpTuples: the reference converts its
    SpTuples to SpDCCols right after the call (ParFriends.h:1100-1102), here that is fused;
  * LocalSpGEMMHash(sort=False) still returns rows ascending (a valid order of the unsorted
    contract; the reference's slot order depends on a sequential insertion order);
  * LocalSpGEMM (heap) and the hybrid share one numeric kernel: the result contract is identical.
"""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import check, lib
from .semirings import Semiring
from .spdccols import SpDCCols


def _spgemm(SR: Semiring, A: SpDCCols, B: SpDCCols, clearA, clearB, flags=0) -> SpDCCols:
    if A.ctx is not B.ctx:
        raise ValueError("A and B live in different contexts")
    h = ctypes.c_void_p()
    check(lib().cbh_spgemm(A.ctx.h, SR.code, A.h, B.h, flags, ctypes.byref(h)), A.ctx.h)
    C = SpDCCols(A.ctx, h)
    if clearA:
        A.free()
    if clearB:
        B.free()
    return C


# cbh_spgemm's reference-order flags (combblas_hip.h): every output re-folded in the named kernel's order
CBH_ORDER_HYBRID, CBH_ORDER_HEAP, CBH_ORDER_HASH = 0x200, 0x400, 0x800


def _order(order, flag):
    if order in (None, "arrival"):
        return 0
    if order == "reference":
        return flag
    raise ValueError(f"order must be None, 'arrival' or 'reference', not {order!r}")


def LocalHybridSpGEMM(SR: Semiring, A: SpDCCols, B: SpDCCols, clearA=False, clearB=False, aux=None,
                      order=None) -> SpDCCols:
    """mtSpGEMM.h:213-460 -- C = A*B, rows ascending within each column. order="reference": every
    output folded in the reference's own order (heap branch for cr < 2, hash branch otherwise), so
    floating-point sums are bit-identical to the stock kernel's; default: arrival order."""
    return _spgemm(SR, A, B, clearA, clearB, _order(order, CBH_ORDER_HYBRID))


def LocalSpGEMMHash(SR: Semiring, A: SpDCCols, B: SpDCCols, clearA=False, clearB=False, sort=True,
                    order=None) -> SpDCCols:
    """mtSpGEMM.h:463-656 (sort=False is satisfied by the sorted result); order="reference": the
    hash kernel's fold order (products in B-entry order, add(new, old))."""
    return _spgemm(SR, A, B, clearA, clearB, _order(order, CBH_ORDER_HASH))


def LocalSpGEMM(SR: Semiring, A: SpDCCols, B: SpDCCols, clearA=False, clearB=False, order=None) -> SpDCCols:
    """mtSpGEMM.h:74-202 (heap SpGEMM) -- same numeric contract as the hybrid; order="reference":
    the heap kernel's pop order (libstdc++ heap, add(old, new))."""
    return _spgemm(SR, A, B, clearA, clearB, _order(order, CBH_ORDER_HEAP))


def estimateFLOPandNNZ(A: SpDCCols, B: SpDCCols, per_column=False):
    """estimateFLOP (mtSpGEMM.h:1057-1134) + estimateNNZ_Hash (:806-933).
    Returns (flops, nnzC) or, with per_column, (flops, nnzC, colflop, colnnz) as torch tensors."""
    f, z = ctypes.c_int64(), ctypes.c_int64()
    cf = cz = None
    pf = pz = None
    if per_column:
        import torch
        cf = torch.empty(B.nzc, dtype=torch.int64, device=A.ctx.tdevice)
        cz = torch.empty(B.nzc, dtype=torch.int64, device=A.ctx.tdevice)
        pf, pz = ctypes.c_void_p(cf.data_ptr()), ctypes.c_void_p(cz.data_ptr())
    check(lib().cbh_spgemm_symbolic(A.ctx.h, A.h, B.h, ctypes.byref(f), ctypes.byref(z), pf, pz), A.ctx.h)
    return (f.value, z.value, cf, cz) if per_column else (f.value, z.value)


class SpGEMMPlan:
    """The symbolic pass of C = A*B kept for a phase loop (cbh_plan_create): the exact nnz of every
    nonzero column of B, and C = A * B(:, c0:c1) per phase without re-running the symbolic pass --
    the phased drivers (MemEfficientSpGEMM, ParFriends.h:449-730, and its 3D form) multiply each
    stage pair once per phase on a column slice of B. A and B must stay alive until close()."""

    def __init__(self, A: SpDCCols, B: SpDCCols):
        if A.ctx is not B.ctx:
            raise ValueError("A and B live in different contexts")
        self.ctx, self.A, self.B = A.ctx, A, B
        h = ctypes.c_void_p()
        check(lib().cbh_plan_create(A.ctx.h, A.h, B.h, ctypes.byref(h)), A.ctx.h)
        self.h = h
        self._jc = None

    def col_nnz(self):
        """exact nnz of A*B per nonzero column slot of B (device int64 tensor, length B.nzc)"""
        import torch

        out = torch.empty(self.B.nzc, dtype=torch.int64, device=self.ctx.tdevice)
        check(lib().cbh_plan_col_nnz(self.h, ctypes.c_void_p(out.data_ptr())), self.ctx.h)
        return out

    def info(self):
        f, z = ctypes.c_int64(), ctypes.c_int64()
        check(lib().cbh_plan_info(self.h, ctypes.byref(f), ctypes.byref(z)), self.ctx.h)
        return f.value, z.value

    def multiply_slots(self, SR: Semiring, s0: int, s1: int, flags=0) -> SpDCCols:
        h = ctypes.c_void_p()
        check(lib().cbh_plan_spgemm_slots(self.h, SR.code, int(s0), int(s1), flags, ctypes.byref(h)), self.ctx.h)
        return SpDCCols(self.ctx, h)

    def multiply(self, SR: Semiring, c0: int, c1: int) -> SpDCCols:
        """C = A * B(:, c0:c1) as an m x B.n block (columns of B in [c0, c1))"""
        import torch

        if self.B.nzc == 0:
            return self.multiply_slots(SR, 0, 0)
        if self._jc is None:
            self._jc = self.B.tensors()[1]
        s0, s1 = (int(x) for x in torch.searchsorted(
            self._jc, torch.tensor([c0, c1], dtype=torch.int64, device=self._jc.device)).cpu())
        return self.multiply_slots(SR, s0, s1)

    def close(self):
        if self.h:
            lib().cbh_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def EstimateLocalFLOP(SR: Semiring, A: SpDCCols, B: SpDCCols, clearA=False, clearB=False) -> int:
    """mtSpGEMM.h:662-689"""
    return estimateFLOPandNNZ(A, B)[0]


def MultiwayMerge(SR: Semiring, lists, mdim=0, ndim=0, delarrs=False) -> SpDCCols:
    """MultiwayMerge.h:411-526 -- merge column-sorted partials, SR::add on duplicates."""
    if len(lists) == 0:
        raise ValueError("MultiwayMerge of zero lists")
    ctx = lists[0].ctx
    for L in lists:
        if (mdim or ndim) and (L.m != mdim or L.n != ndim):
            raise _lib.CombBLASHipError(3002, "Dimensions of SpTuples do not match on multiwayMerge()")
    cur = list(lists)
    first = True
    # the kernel merges up to 16 lists at once; larger fan-in is merged hierarchically
    while len(cur) > 1 or first:
        nxt = []
        for i in range(0, len(cur), 16):
            grp = cur[i:i + 16]
            arr = (ctypes.c_void_p * len(grp))(*[g.h.value for g in grp])
            h = ctypes.c_void_p()
            check(lib().cbh_merge(ctx.h, SR.code, len(grp), arr, ctypes.byref(h)), ctx.h)
            nxt.append(SpDCCols(ctx, h))
        if not first:  # intermediate results of the hierarchy (the inputs are the caller's)
            for g in cur:
                g.free()
        first = False
        cur = nxt
    if delarrs:
        for L in lists:
            L.free()
    return cur[0]


def PhasedSpGEMM(SR: Semiring, A: SpDCCols, B: SpDCCols, checksum=False, budget_bytes=None, on_phase=None):
    """MemEfficientSpGEMM's phase loop (ParFriends.h:449-730) for one block: B's columns are
    processed in phases sized from the exact symbolic pass; each phase's C block is materialised
    in HBM then its buffer reused. Returns {flops, nnz, phases, value_sum, digest}.

    on_phase(phase, slot0, slot1, Cphase): the per-phase consumer (MemEfficientSpGEMM's
    MCLPruneRecoverySelect + ColConcatenate, :694-721). Cphase is a borrowed m x B.n SpDCCols of
    C(:, B's column slots [slot0, slot1)) with the phase's empty columns kept; it is valid only
    during the call (clone() keeps a copy)."""
    if budget_bytes is not None:
        A.ctx.set_phase_budget(budget_bytes)
    st = _lib.cbh_phase_stats()
    flags = _lib.CBH_PHASE_CHECKSUM if checksum else 0
    cb = None
    errors = []
    if on_phase is not None:
        def _consume(user, phase, s0, s1, view):
            v = SpDCCols(A.ctx, ctypes.c_void_p(view), borrowed=True)
            try:
                on_phase(int(phase), int(s0), int(s1), v)
            except Exception as e:  # reported after the C call returns
                errors.append(e)
                return _lib.ERR_CALLBACK
            finally:
                v.h = None
            return 0
        cb = _lib.PHASE_FN(_consume)
        check(lib().cbh_ctx_set_phase_consumer(A.ctx.h, cb, None), A.ctx.h)
    try:
        rc = lib().cbh_spgemm_phased(A.ctx.h, SR.code, A.h, B.h, flags, ctypes.byref(st))
    finally:
        if cb is not None:
            lib().cbh_ctx_set_phase_consumer(A.ctx.h, _lib.PHASE_FN(), None)
    if errors:
        raise errors[0]
    check(rc, A.ctx.h)
    return {"flops": st.flops, "nnz": st.nnz, "phases": st.phases, "value_sum": st.value_sum,
            "digest": st.digest}
