"""Process grids of the distributed SpGEMM (reference: CommGrid.cpp:37-75,164-180, CommGrid3D.h:21-107).

One process per GPU. A CommGrid arranges `ranks` row-major on a gr x gc grid
(myprocrow = r / gc, myproccol = r % gc, CommGrid.cpp:60-61); its row world holds the ranks of
one grid row, its column world those of one grid column. A CommGrid3D stacks `nlayers` such
grids: global rank = layer * (gr*gc) + row * gc + col (CommGrid3D.h:84-86, non-special layout);
the fiber world joins the ranks with the same position in every layer.

All communicators are created collectively: every rank builds every group in the same order
(torch.distributed.new_group, like MPI_Comm_split, needs every rank of the parent).
"""
from __future__ import annotations

import math

import torch.distributed as dist

from ._lib import CombBLASHipError
from .comm import Group

GRIDMISMATCH = 3001  # SpDefs.h
NOTSQUARE = 3003


def _world():
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class CommGrid:
    """CommGrid(world, nrowproc, ncolproc) over the ordered global ranks `ranks` (default: all)."""

    def __init__(self, grid_rows=0, grid_cols=0, ranks=None):
        me, world = _world()
        self.ranks = list(range(world)) if ranks is None else list(ranks)
        p = len(self.ranks)
        if grid_rows == 0 and grid_cols == 0:
            grid_rows = grid_cols = math.isqrt(p)
            if grid_rows * grid_cols != p:
                raise CombBLASHipError(NOTSQUARE, "This version of the Combinatorial BLAS only works on a square "
                                                  "logical processor grid")
        if grid_rows * grid_cols != p:
            raise CombBLASHipError(GRIDMISMATCH, f"{grid_rows}x{grid_cols} grid over {p} ranks")
        self.grrows, self.grcols = grid_rows, grid_cols
        self.member = me in self.ranks
        self.myrank = self.ranks.index(me) if self.member else -1
        self.myprocrow, self.myproccol = divmod(self.myrank, grid_cols) if self.member else (-1, -1)
        self.world = Group(self.ranks, me)
        rows = [Group([self.ranks[r * grid_cols + c] for c in range(grid_cols)], me) for r in range(grid_rows)]
        cols = [Group([self.ranks[r * grid_cols + c] for r in range(grid_rows)], me) for c in range(grid_cols)]
        self.rowWorld = rows[self.myprocrow] if self.member else None
        self.colWorld = cols[self.myproccol] if self.member else None

    # reference accessors
    def GetGridRows(self):
        return self.grrows

    def GetGridCols(self):
        return self.grcols

    def GetSize(self):
        return self.grrows * self.grcols

    def GetRank(self, rowrank=None, colrank=None):
        if rowrank is None:
            return self.myrank
        return rowrank * self.grcols + colrank

    def GetRankInProcRow(self):
        return self.myproccol

    def GetRankInProcCol(self):
        return self.myprocrow

    def GetRowWorld(self):
        return self.rowWorld

    def GetColWorld(self):
        return self.colWorld

    def __eq__(self, other):
        return isinstance(other, CommGrid) and self.ranks == other.ranks and \
            (self.grrows, self.grcols) == (other.grrows, other.grcols)

    __hash__ = object.__hash__


def ProductGrid(gridA: CommGrid, gridB: CommGrid):
    """CommGrid.cpp:164-180: C's grid and the number of SUMMA stages (= A's grid columns)."""
    if gridA.grcols != gridB.grrows:
        raise CombBLASHipError(GRIDMISMATCH, "Grids don't confirm for multiplication")
    if gridA != gridB:
        raise CombBLASHipError(GRIDMISMATCH, "A and B live on different process grids")
    return gridA, gridA.grcols


class CommGrid3D:
    """CommGrid3D(world, nlayers, 0, 0): nlayers square grids (non-special layout)."""

    def __init__(self, nlayers, ranks=None):
        me, world = _world()
        self.ranks = list(range(world)) if ranks is None else list(ranks)
        p = len(self.ranks)
        if nlayers < 1 or p % nlayers:
            raise CombBLASHipError(NOTSQUARE, "Number of processes is not divisible by number of layers")
        ppl = p // nlayers
        gr = math.isqrt(ppl)
        if gr * gr != ppl:
            raise CombBLASHipError(NOTSQUARE, "only square grids within a layer")
        self.gridLayers, self.gridRows, self.gridCols = nlayers, gr, gr
        self.myrank = self.ranks.index(me)
        self.rankInFiber, self.rankInLayer = divmod(self.myrank, ppl)
        self.world = Group(self.ranks, me)
        layers = [CommGrid(gr, gr, self.ranks[l * ppl:(l + 1) * ppl]) for l in range(nlayers)]
        fibers = [Group([self.ranks[l * ppl + q] for l in range(nlayers)], me) for q in range(ppl)]
        self.commGridLayer = layers[self.rankInFiber]
        self.fiberWorld = fibers[self.rankInLayer]
        self.layerWorld = self.commGridLayer.world

    def GetRank(self, layerrank, rowrank, colrank):
        return layerrank * self.gridRows * self.gridCols + rowrank * self.gridCols + colrank

    def GetGridLayers(self):
        return self.gridLayers

    def GetGridRows(self):
        return self.gridRows

    def GetGridCols(self):
        return self.gridCols

    def GetSize(self):
        return self.gridLayers * self.gridRows * self.gridCols

    def GetCommGridLayer(self):
        return self.commGridLayer

    def GetFiberWorld(self):
        return self.fiberWorld

    def GetLayerWorld(self):
        return self.layerWorld

    def GetRankInFiber(self):
        return self.rankInFiber

    def GetRankInLayer(self):
        return self.rankInLayer
