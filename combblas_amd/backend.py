"""Local-block operations the distributed drivers (parfriends.py) call on every rank.

`HipBackend` is the product: every multiply / merge / symbolic pass runs in the gfx950 kernels
behind the C-ABI (LocalHybridSpGEMM, MultiwayMerge, estimateNNZ_Hash), and blocks are
device-resident SpDCCols whose arrays are torch tensors in HBM, so RCCL broadcasts and
alltoalls move them without host copies. The drivers only see this interface; the CPU
multi-process tests substitute a checker backend for it (tests/dist_util.py), which is how the
grid logic is exercised without a GPU.
"""
from __future__ import annotations

import numpy as np
import torch

from .mtspgemm import LocalHybridSpGEMM, MultiwayMerge, estimateFLOPandNNZ
from .spdccols import Context, HostDcsc, SpDCCols

TORCH_OF_NP = {np.dtype(np.float64): torch.float64, np.dtype(np.int64): torch.int64,
               np.dtype(np.uint8): torch.uint8, np.dtype(np.float32): torch.float32,
               np.dtype(np.int32): torch.int32}


class HipBackend:
    def __init__(self, ctx: Context):
        if getattr(ctx, "tdevice", None) is None or ctx._alloc_cb is None:
            raise ValueError("the distributed drivers need a Context created with torch_allocator=True")
        self.ctx = ctx
        self.device = ctx.tdevice

    # ------------------------------------------------------------------ blocks
    def from_host(self, h: HostDcsc) -> SpDCCols:
        return SpDCCols.from_host(self.ctx, h)

    def wrap(self, m, n, cp, jc, ir, num) -> SpDCCols:
        return SpDCCols.from_tensors(self.ctx, int(m), int(n), cp, jc, ir, num)

    @staticmethod
    def dims(b: SpDCCols):
        return b.m, b.n, b.nnz, b.nzc

    @staticmethod
    def arrays(b: SpDCCols):
        return b.tensors()

    @staticmethod
    def value_dtype(b: SpDCCols):
        return TORCH_OF_NP[b.np_dtype]

    @staticmethod
    def to_host(b: SpDCCols) -> HostDcsc:
        return b.to_host()

    @staticmethod
    def free(b: SpDCCols):
        b.free()

    # ------------------------------------------------------------------ kernels
    @staticmethod
    def multiply(SR, A: SpDCCols, B: SpDCCols) -> SpDCCols:
        return LocalHybridSpGEMM(SR, A, B)

    @staticmethod
    def merge(SR, blocks, m, n) -> SpDCCols:
        return MultiwayMerge(SR, blocks, m, n)

    @staticmethod
    def plan(A: SpDCCols, B: SpDCCols):
        """one symbolic pass of A*B for a phase loop: .col_nnz(), .multiply(SR, c0, c1), .close()"""
        from .mtspgemm import SpGEMMPlan

        return SpGEMMPlan(A, B)

    @staticmethod
    def col_nnz(A: SpDCCols, B: SpDCCols):
        """exact nnz of A*B per nonzero column slot of B (device int64, length B.nzc)"""
        if A.nnz == 0 or B.nnz == 0:
            return torch.zeros(B.nzc, dtype=torch.int64, device=A.ctx.tdevice)
        return estimateFLOPandNNZ(A, B, per_column=True)[3]

    def synchronize(self):
        self.ctx.synchronize()

    # ------------------------------------------------------------------ callers around the hot path
    # (C-ABI entry points of combblas_amd/csrc/apps.h; vectors are device tensors)
    def masked(self, SR, A: SpDCCols, B: SpDCCols, M: SpDCCols, pattern=False) -> SpDCCols:
        from .apps import MaskedSpGEMM
        return MaskedSpGEMM(SR, A, B, M, pattern=pattern)

    def ewise_mult(self, A: SpDCCols, B: SpDCCols) -> SpDCCols:
        from .apps import EWiseMult
        return EWiseMult(A, B)

    def col_stats(self, A: SpDCCols, hard):
        from .apps import ColumnStats
        return ColumnStats(A, hard)

    def col_stats_kept(self, A: SpDCCols, thresh):
        from .apps import ColumnStatsKept
        return ColumnStatsKept(A, thresh)

    def kselect_cols(self, A: SpDCCols, aidx, nact, k):
        from .apps import kselect_cols
        return kselect_cols(A, aidx, nact, k)

    def kselect_hist(self, A: SpDCCols, aidx, nact, prefix, shift):
        from .apps import kselect_hist
        return kselect_hist(A, aidx, nact, prefix, shift)

    def kselect_pick(self, nact, hist, prefix, rank, shift):
        from .apps import kselect_pick
        kselect_pick(self.ctx, nact, hist, prefix, rank, shift)

    def kselect_value(self, nact, prefix):
        from .apps import kselect_value
        return kselect_value(self.ctx, nact, prefix)

    def prune_columns(self, A: SpDCCols, thresh) -> SpDCCols:
        from .apps import PruneColumn
        return PruneColumn(A, thresh)

    def mcl_prune_block(self, A: SpDCCols, hard, selectNum, recoverNum, recoverPct) -> SpDCCols:
        from .apps import MCLPruneBlock
        return MCLPruneBlock(A, hard, selectNum, recoverNum, recoverPct)
