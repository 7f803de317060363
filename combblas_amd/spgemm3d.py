"""The standalone 3D SpGEMM layer (reference: 3DSpGEMM/CCGrid.h, SplitMatDist.h, SUMMALayer.h,
Reductions.h, Multiplier.h) -- the API `3DSpGEMM/mpipspgemm.cpp` drives, next to the library's
own 3D driver (parfriends.Mult_AnXBn_SUMMA3D).

  CCGrid                           CCGrid.h:6-45          c layers of a square gr x gr grid;
                                                          layer = rank % c, rank in layer = rank / c
  SplitMat                         SplitMatDist.h:143-213 layer 0's block cut into c column
                                                          (A) or row (B) pieces, piece l sent to
                                                          fiber rank l
  SUMMALayer                       SUMMALayer.h:24-97     the layer's SUMMA stages; returns the
                                                          unmerged stage products
  ParallelReduce_Alltoall_threaded Reductions.h:36-130    column chunk j of the layer product goes
                                                          to fiber rank j, received pieces merged
  ReduceAll_threaded               Reductions.h:133-155   MultiwayMerge of the stage list, then the
                                                          fiber reduce-scatter
  multiply                         Multiplier.h:10-61     SUMMALayer + ReduceAll_threaded

MI355X design: blocks stay device-resident (backend.HipBackend: gfx950 LocalSpGEMM / MultiwayMerge
kernels), SplitMat's point-to-point sends are one alltoallv over the fiber (RCCL), the stage
broadcasts are RCCL broadcasts on the row / column worlds and the reduce-scatter is one alltoallv
of the DCSC arrays (no tuple repacking: the reference's 24-B std::tuple stream becomes the 12-B
SoA arrays). Timers with the reference's names (comm_bcast, comm_reduce, comp_summa, comp_reduce,
comp_reduce_layer, comp_result, comp_split, comm_split) accumulate in `timers`.

One deliberate deviation: Reductions.h:99-102 shifts the received column ids of the LAST fiber
rank by fibrank * (its own, remainder-sized width); that equals the chunk start only when the
fiber size divides the column count (the reference's drivers use such sizes). Here every rank
shifts by its chunk's start i * (ndim / fprocs) -- the splitter findColSplitters cut it at
(MultiwayMerge.h:85-103) -- so uneven sizes give the correct product as well.
"""
from __future__ import annotations

import time

import torch

from . import parfriends as pf
from ._lib import CombBLASHipError
from .comm import Group, alltoallv
from .commgrid import GRIDMISMATCH, NOTSQUARE, CommGrid, _world
from .semirings import PlusTimesSRing

timers = dict(comm_bcast=0.0, comm_reduce=0.0, comp_summa=0.0, comp_reduce=0.0, comp_reduce_layer=0.0,
              comp_result=0.0, comp_split=0.0, comm_split=0.0)


def _sync(be):
    be.synchronize()
    return time.perf_counter()


class CCGrid:
    """CCGrid(c_factor, gr_cols) (CCGrid.h:9-30) over the ordered global ranks `ranks`. Besides
    the reference's members it holds `layerGrid`, the CommGrid over this rank's layer world
    (mpipspgemm.cpp builds it as CommGrid(CMG.layerWorld, 0, 0))."""

    def __init__(self, c_factor, gr_cols, ranks=None):
        me, world = _world()
        self.ranks = list(range(world)) if ranks is None else list(ranks)
        self.nprocs = len(self.ranks)
        c, g = int(c_factor), int(gr_cols)
        if c < 1 or g < 1:
            raise CombBLASHipError(GRIDMISMATCH, "CCGrid needs c_factor >= 1 and gr_cols >= 1")
        if g * g * c != self.nprocs:
            raise CombBLASHipError(NOTSQUARE, "The product of <GridRows> <GridCols> <Replicas> does not match the "
                                              "number of processes")
        self.GridLayers, self.GridRows, self.GridCols = c, g, g
        self.myrank = self.ranks.index(me)
        self.layer_grid = self.myrank % c  # = RankInFiber
        self.RankInLayer = self.myrank // c
        self.RankInCol = self.RankInLayer // g  # MYPROCROW
        self.RankInRow = self.RankInLayer % g  # MYPROCCOL
        ppl = g * g
        # MPI_Comm_split(WORLD, color, key): every group is built by every rank in the same order
        layer_ranks = [[self.ranks[q * c + l] for q in range(ppl)] for l in range(c)]  # key RankInLayer
        layers = [CommGrid(g, g, r) for r in layer_ranks]
        fibers = [Group([self.ranks[q * c + l] for l in range(c)], me) for q in range(ppl)]  # key layer_grid
        self.layerGrid = layers[self.layer_grid]
        self.layerWorld = self.layerGrid.world
        self.fiberWorld = fibers[self.RankInLayer]
        # rowWorld: color layer*GridRows + RankInLayer/GridRows, key RankInRow -- the layer grid's
        # row world; colWorld: color layer*GridCols + RankInLayer%GridRows, key RankInCol
        self.rowWorld = self.layerGrid.rowWorld
        self.colWorld = self.layerGrid.colWorld


def _colsplit_pieces(be, blk, nparts):
    """SpDCCols::ColSplit (SpDCCols.cpp:936-970): columns cut at (i+1)*(n/parts), the last piece
    takes the remainder; column ids rebased"""
    m, n, nnz, nzc = be.dims(blk)
    if n < nparts:
        raise CombBLASHipError(3002, "Matrix is too small to be splitted")
    w = n // nparts
    out = []
    for i in range(nparts):
        c0, c1 = i * w, (n if i == nparts - 1 else (i + 1) * w)
        s = pf._colslice(be, blk, c0, c1)
        cp, jc, ir, num = be.arrays(s)
        out.append(be.wrap(m, c1 - c0, cp, (jc - c0).contiguous(), ir, num))
    return out


def _rowsplit_pieces(be, blk, nparts):
    """SplitMat's row split: Transpose, ColSplit, Transpose back (SplitMatDist.h:153,208) = rows
    cut at (i+1)*(m/parts), row ids rebased, every column's rows still ascending"""
    m, n, nnz, nzc = be.dims(blk)
    if m < nparts:
        raise CombBLASHipError(3002, "Matrix is too small to be splitted")
    h = m // nparts
    out = []
    for i in range(nparts):
        r0, r1 = i * h, (m if i == nparts - 1 else (i + 1) * h)
        s = pf._rowrange(be, blk, r0, r1)
        cp, jc, ir, num = be.arrays(s)
        out.append(be.wrap(r1 - r0, n, cp, jc, (ir - r0).to(torch.int32).contiguous(), num))
    return out


def SplitMat(CMG: CCGrid, localmat, be, rowsplit=False, vdtype=None):
    """SplitMatDist.h:143-213: `localmat` is the layer-0 rank's block (ignored on other layers);
    returns this rank's piece. The essentials go out first (MPI_Scatter on the fiber), then the
    four arrays of every piece in one alltoallv each (the reference's MPI_Send/MPI_Recv pairs)."""
    t0 = time.perf_counter()
    L, root = CMG.GridLayers, CMG.layer_grid == 0
    fib = CMG.fiberWorld
    dev = be.device
    if root:
        vdtype = be.value_dtype(localmat)
        parts = (_rowsplit_pieces if rowsplit else _colsplit_pieces)(be, localmat, L) if L > 1 else [localmat]
        ess = [be.dims(p) for p in parts]
    elif vdtype is None:
        raise CombBLASHipError(3002, "SplitMat on a non-root layer needs the value dtype")
    timers["comp_split"] += time.perf_counter() - t0
    t1 = time.perf_counter()
    if L == 1:
        timers["comm_split"] += time.perf_counter() - t1
        return localmat
    none = [0] * L
    send_ess = torch.tensor([v for e in ess for v in e] if root else [], dtype=torch.int64, device=dev)
    mine = alltoallv(send_ess, [4] * L if root else none, [4] + [0] * (L - 1), fib).cpu().tolist()
    m, n, nnz, nzc = (int(x) for x in mine)

    def scatter(k, dtype, mine_count):
        """array k (0 cp, 1 jc, 2 ir, 3 num) of every piece from the root to its fiber rank"""
        if root:
            send = torch.cat([be.arrays(p)[k] for p in parts])
            sc = [(e[3] + 1, e[3], e[2], e[2])[k] for e in ess]
        else:
            send, sc = torch.empty(0, dtype=dtype, device=dev), none
        return alltoallv(send, sc, [mine_count] + [0] * (L - 1), fib)

    rcp = scatter(0, torch.int64, nzc + 1)
    rjc = scatter(1, torch.int64, nzc)
    rir = scatter(2, torch.int32, nnz)
    rnum = scatter(3, vdtype, nnz)
    timers["comm_split"] += time.perf_counter() - t1
    return be.wrap(m, n, rcp, rjc, rir, rnum)


def _transpose(be, blk):
    """local transpose of a block (SpDCCols::Transpose), rows ascending in every column"""
    m, n, nnz, nzc = be.dims(blk)
    cp, jc, ir, num = be.arrays(blk)
    if nnz == 0:
        return pf._empty(be, n, m, num.dtype)
    col = torch.repeat_interleave(jc, cp[1:] - cp[:-1])
    key = ir.to(torch.int64) * max(n, 1) + col
    o = torch.sort(key, stable=True).indices
    ncol = ir.to(torch.int64)[o]
    nrow = col[o].to(torch.int32)
    njc, cnt = torch.unique_consecutive(ncol, return_counts=True)
    ncp = torch.zeros(njc.numel() + 1, dtype=torch.int64, device=ir.device)
    torch.cumsum(cnt, 0, out=ncp[1:])
    return be.wrap(n, m, ncp, njc.contiguous(), nrow.contiguous(), num[o].contiguous())


def SUMMALayer(SplitA, SplitB, C: list, CMG: CCGrid, isBT, threaded, be, SR=PlusTimesSRing):
    """SUMMALayer.h:24-97: GridCols stages; at stage i the row world broadcasts A's piece of rank
    i and the column world B's piece of rank i, and their product is appended to C (unmerged).
    isBT: SplitB holds B's piece locally transposed (the reference's outer-product variant)."""
    stages = CMG.GridCols
    vdtype = be.value_dtype(SplitA)
    Aess = pf._essentials(be, SplitA, CMG.rowWorld)
    Bess = pf._essentials(be, SplitB, CMG.colWorld)
    Aself, Bself = CMG.RankInRow, CMG.RankInCol
    for i in range(stages):
        t0 = _sync(be)
        Ai = pf._bcast_block(be, SplitA, Aess, i, CMG.rowWorld, vdtype)
        Bi = pf._bcast_block(be, SplitB, Bess, i, CMG.colWorld, vdtype)
        t1 = _sync(be)
        timers["comm_bcast"] += t1 - t0
        Bm = _transpose(be, Bi) if isBT else Bi
        C.append(be.multiply(SR, Ai, Bm))
        if Bm is not Bi:
            be.free(Bm)
        if i != Aself:
            be.free(Ai)
        if i != Bself:
            be.free(Bi)
        timers["comp_summa"] += _sync(be) - t1
    return C


class _Fiber:
    """the three members of a 3D grid the fiber reduce-scatter reads"""

    def __init__(self, fibWorld):
        self.fiberWorld = fibWorld
        self.gridLayers = fibWorld.size
        self.rankInFiber = fibWorld.rank


def ParallelReduce_Alltoall_threaded(fibWorld: Group, localmerged, be, SR=PlusTimesSRing):
    """Reductions.h:36-130: the layer product's column chunk j (splitters at j*(ncol/fprocs),
    findColSplitters) goes to fiber rank j; the received pieces are merged into this rank's
    m x ncol_j chunk with chunk-local column ids. Returns (chunk, its first column)."""
    if fibWorld.size == 1:
        return localmerged, 0
    t0 = _sync(be)
    m, n, _, _ = be.dims(localmerged)
    C, c0 = pf._fiber_reduce_scatter(be, SR, localmerged, _Fiber(fibWorld), m, n, be.value_dtype(localmerged))
    t1 = _sync(be)
    timers["comm_reduce"] += t1 - t0
    if C is not localmerged:
        be.free(localmerged)
    return C, c0


def ReduceAll_threaded(unreducedC: list, CMG: CCGrid, be, SR=PlusTimesSRing):
    """Reductions.h:133-155: MultiwayMerge of the stage products (delarrs), then the fiber
    reduce-scatter; returns this rank's C chunk. The reference fixes PlusTimesSRing<double,double>
    here; SR is a parameter (default the same semiring)."""
    m, n = be.dims(unreducedC[0])[:2]
    vdtype = be.value_dtype(unreducedC[0])
    t0 = _sync(be)
    merged = pf._merge(be, SR, list(unreducedC), m, n, vdtype)
    for p in unreducedC:
        if p is not merged:
            be.free(p)
    unreducedC.clear()
    timers["comp_reduce"] += _sync(be) - t0
    C, _ = ParallelReduce_Alltoall_threaded(CMG.fiberWorld, merged, be, SR)
    return C


def multiply(splitA, splitB, CMG: CCGrid, isBT, threaded, be, SR=PlusTimesSRing):
    """Multiplier.h:10-61: C chunk of this rank = ReduceAll_threaded(SUMMALayer(...)). The timers
    are reset first, as the reference resets its globals; they hold the breakdown afterwards."""
    for k in timers:
        if k not in ("comp_split", "comm_split"):
            timers[k] = 0.0
    unreducedC = []
    SUMMALayer(splitA, splitB, unreducedC, CMG, isBT, threaded, be, SR)
    return ReduceAll_threaded(unreducedC, CMG, be, SR)
