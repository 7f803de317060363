"""Distributed sparse matrices: one local block per rank, device-resident.

SpParMat   (SpParMat.h / SpParMat.cpp)     2D block distribution on a CommGrid.
SpParMat3D (SpParMat3D.h / SpParMat3D.cpp) nlayers 2D layers; A is column-split and B row-split
                                           across layers (non-special layout).

Block distribution (SpParMat::Owner, SpParMat.cpp:5076-5104): rows are cut into gr blocks of
m/gr rows, the last block taking the remainder (all rows go to the last block when m < gr);
columns likewise. 3D (SpParMat3D::Owner, SpParMat3D.cpp:337-402): the layer-0 block is then cut
into nlayers column chunks (colsplit) or row chunks (rowsplit) of width/nlayers, the last chunk
taking the remainder. Local ids are 0-based within the block, as in the reference.

`distribute` builds each rank's block straight from the global matrix (every rank holds the
deterministic generator's output), which lands the same entries on the same ranks as the
reference's SparseCommon / ExchangeData redistribution.
"""
from __future__ import annotations

import numpy as np
import torch.distributed as dist

from .commgrid import CommGrid, CommGrid3D
from .spdccols import HostDcsc


def block_range(total, nprocs, idx):
    """[lo, hi) of block idx (Owner: total//nprocs per block, remainder to the last)"""
    per = total // nprocs
    lo = idx * per
    hi = total if idx == nprocs - 1 else lo + per
    return lo, hi


def split_range(lo, hi, nparts, idx):
    """chunk idx of [lo, hi) cut into nparts (SpParMat3D::Owner's n_perproc = width / nlayers)"""
    a, b = block_range(hi - lo, nparts, idx)
    return lo + a, lo + b


def host_block(G: HostDcsc, r0, r1, c0, c1) -> HostDcsc:
    """G[r0:r1, c0:c1] with block-local ids (entries keep their (col,row) order)"""
    s, e = np.searchsorted(G.jc, [c0, c1])
    jc, cp = G.jc[s:e], G.cp[s:e + 1]
    if jc.size == 0:
        return HostDcsc(r1 - r0, c1 - c0, [], [0], [], G.num[:0])
    ir, num = G.ir[cp[0]:cp[-1]], G.num[cp[0]:cp[-1]]
    cols = np.repeat(jc - c0, np.diff(cp))
    keep = (ir >= r0) & (ir < r1)
    cols, ir, num = cols[keep], ir[keep] - r0, num[keep]
    counts = np.bincount(cols, minlength=c1 - c0)
    njc = np.nonzero(counts)[0]
    ncp = np.concatenate([[0], np.cumsum(counts[njc])])
    return HostDcsc(r1 - r0, c1 - c0, njc, ncp, ir, num)


class SpParMat:
    """A 2D-distributed matrix: this rank's block `seq` (a backend block) of the global m x n."""

    def __init__(self, seq, grid: CommGrid, backend, m, n, row_off=0, col_off=0):
        self.seq, self.commGrid, self.backend = seq, grid, backend
        self.m, self.n = int(m), int(n)
        self.row_off, self.col_off = int(row_off), int(col_off)

    @staticmethod
    def distribute(G: HostDcsc, grid: CommGrid, backend, dtype=None):
        r0, r1 = block_range(G.m, grid.grrows, grid.myprocrow)
        c0, c1 = block_range(G.n, grid.grcols, grid.myproccol)
        blk = host_block(G if dtype is None else G.astype(dtype), r0, r1, c0, c1)
        return SpParMat(backend.from_host(blk), grid, backend, G.m, G.n, r0, c0)

    def getnrow(self):
        return self.m

    def getncol(self):
        return self.n

    def seqptr(self):
        return self.seq

    def getcommgrid(self):
        return self.commGrid

    def getlocalnnz(self):
        return self.backend.dims(self.seq)[2]

    def getnnz(self):
        """SpParMat::getnnz (allreduce of the local counts)"""
        from .comm import allreduce_
        import torch

        t = torch.tensor([self.getlocalnnz()], dtype=torch.int64, device=self.backend.device)
        return int(allreduce_(t, self.commGrid.world).item())

    def gather_host(self) -> HostDcsc | None:
        """The whole matrix on rank 0 (verification / small matrices; None elsewhere)."""
        return _gather(self.backend, self.seq, self.row_off, self.col_off, self.m, self.n)


class SpParMat3D:
    """nlayers stacked layer matrices; `colsplit` says how the layer-0 block was cut."""

    def __init__(self, seq, grid3: CommGrid3D, backend, m, n, colsplit, row_off=0, col_off=0):
        self.seq, self.commGrid3D, self.backend, self.colsplit = seq, grid3, backend, colsplit
        self.m, self.n = int(m), int(n)
        self.row_off, self.col_off = int(row_off), int(col_off)

    @staticmethod
    def local_ranges(m, n, grid3: CommGrid3D, colsplit):
        g = grid3.commGridLayer
        r0, r1 = block_range(m, g.grrows, g.myprocrow)
        c0, c1 = block_range(n, g.grcols, g.myproccol)
        L, l = grid3.gridLayers, grid3.rankInFiber
        if colsplit:
            c0, c1 = split_range(c0, c1, L, l)
        else:
            r0, r1 = split_range(r0, r1, L, l)
        return r0, r1, c0, c1

    @staticmethod
    def distribute(G: HostDcsc, grid3: CommGrid3D, backend, colsplit, dtype=None):
        r0, r1, c0, c1 = SpParMat3D.local_ranges(G.m, G.n, grid3, colsplit)
        blk = host_block(G if dtype is None else G.astype(dtype), r0, r1, c0, c1)
        return SpParMat3D(backend.from_host(blk), grid3, backend, G.m, G.n, colsplit, r0, c0)

    def getnrow(self):
        return self.m

    def getncol(self):
        return self.n

    def GetLayerMat(self):
        return self

    def seqptr(self):
        return self.seq

    def getcommgrid3D(self):
        return self.commGrid3D

    def isColSplit(self):
        return self.colsplit

    def getlocalnnz(self):
        return self.backend.dims(self.seq)[2]

    def gather_host(self) -> HostDcsc | None:
        return _gather(self.backend, self.seq, self.row_off, self.col_off, self.m, self.n)


def _gather(backend, seq, row_off, col_off, m, n):
    h = backend.to_host(seq)
    cols = np.repeat(h.jc, np.diff(h.cp)) + col_off
    piece = (h.ir.astype(np.int64) + row_off, cols, h.num)
    if dist.is_initialized() and dist.get_world_size() > 1:
        out = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
        dist.gather_object(piece, out, dst=0)
        if dist.get_rank() != 0:
            return None
    else:
        out = [piece]
    rows = np.concatenate([p[0] for p in out])
    cols = np.concatenate([p[1] for p in out])
    num = np.concatenate([p[2] for p in out])
    o = np.lexsort((rows, cols))
    rows, cols, num = rows[o], cols[o], num[o]
    jc, first = np.unique(cols, return_index=True)
    cp = np.append(first, rows.size).astype(np.int64)
    return HostDcsc(m, n, jc, cp, rows.astype(np.int32), num)
