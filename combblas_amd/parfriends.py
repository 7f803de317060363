"""Distributed SpGEMM drivers over RCCL (reference: include/CombBLAS/ParFriends.h).

  Mult_AnXBn_Synch     ParFriends.h:1004-1108  2D SUMMA: per stage i, A's block (r,i) is broadcast
                                               on the row world and B's block (i,c) on the column
                                               world, multiplied locally, and the stage partials
                                               are merged (MultiwayMerge).
  MemEfficientSpGEMM   ParFriends.h:449-730    the same product with B's columns cut into phases so
                                               that the partials of one phase fit the memory budget
                                               (the prune/select/recover steps of HipMCL are not on
                                               this path).
  Mult_AnXBn_SUMMA3D   ParFriends.h:2917-3190  per-layer SUMMA, then the fiber reduce-scatter: the
                                               layer partial is cut into nlayers column ranges
                                               (divisions3d), exchanged with an alltoallv and the
                                               received pieces merged.
  Mult_AnXBn_Overlap   ParFriends.h:1110-1235  Synch with the broadcasts of stage i+1 posted (non-blocking, on
                                               RCCL's stream) before stage i's local multiply.
  Mult_AnXBn_DoubleBuff ParFriends.h:798-997   A split by columns and B by rows into halves; each stage
                                               multiplies the halves in turn, so only half of A's and
                                               B's received blocks are resident at a time (overlapped
                                               like Overlap).
  PSpGEMM              SpParMat.h:454-467      dispatch on the operand type.

MI355X design: every block is device-resident and every collective moves HBM tensors
(torch.distributed "nccl" = RCCL over xGMI), the local multiply / merge / symbolic pass are the
gfx950 kernels (backend.HipBackend). In the phased drivers all stage blocks are broadcast once
up front and kept in HBM (a scale-22 R-MAT A is 0.8 GB; HBM is 288 GB), so the phase loop of
the 2D driver runs without any communication and phases are planned from the exact per-column
nnz of the partials (estimateNNZ_Hash), not from a sampled estimate.
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import CombBLASHipError
from .comm import allgather_i64, allreduce_, alltoallv, bcast, ibcast
from .commgrid import ProductGrid
from .spparmat import SpParMat, SpParMat3D, block_range

DIMMISMATCH = 3002


# ---------------------------------------------------------------------------------- block utils
def _empty(be, m, n, vdtype):
    dev = be.device
    return be.wrap(m, n, torch.zeros(1, dtype=torch.int64, device=dev), torch.zeros(0, dtype=torch.int64, device=dev),
                   torch.zeros(0, dtype=torch.int32, device=dev), torch.zeros(0, dtype=vdtype, device=dev))


def _colslice(be, blk, c0, c1):
    """columns [c0, c1) of a block, same column space (ir/num are views, cp is rebased)"""
    m, n, nnz, nzc = be.dims(blk)
    if c0 <= 0 and c1 >= n:
        return blk
    cp, jc, ir, num = be.arrays(blk)
    s, e = (int(x) for x in torch.searchsorted(jc, torch.tensor([c0, c1], dtype=torch.int64, device=jc.device)).cpu())
    p0, p1 = (int(x) for x in cp[[s, e]].cpu()) if nzc else (0, 0)
    return be.wrap(m, n, (cp[s:e + 1] - p0).contiguous(), jc[s:e], ir[p0:p1], num[p0:p1])


def _concat_cols(be, blocks, m, n, vdtype):
    """ColConcatenate of blocks over increasing, disjoint column ranges of one column space"""
    blocks = [b for b in blocks if be.dims(b)[3] > 0]
    if not blocks:
        return _empty(be, m, n, vdtype)
    if len(blocks) == 1:
        return blocks[0]
    arrs = [be.arrays(b) for b in blocks]
    off, cps = 0, []
    for i, (cp, jc, ir, num) in enumerate(arrs):
        cps.append((cp[:-1] if i + 1 < len(arrs) else cp) + off)
        off += ir.numel()
    return be.wrap(m, n, torch.cat(cps), torch.cat([a[1] for a in arrs]), torch.cat([a[2] for a in arrs]),
                   torch.cat([a[3] for a in arrs]))


def _merge(be, SR, parts, m, n, vdtype):
    parts = [p for p in parts if be.dims(p)[2] > 0]  # `if(!C_cont->isZero()) tomerge.push_back`
    if not parts:
        return _empty(be, m, n, vdtype)
    if len(parts) == 1:
        return parts[0]
    return be.merge(SR, parts, m, n)


def _essentials(be, blk, group):
    """SpParHelper::GetSetSizes: (m, n, nnz, nzc) of every rank of the group"""
    return allgather_i64(be.dims(blk), group, be.device).tolist()


def _bcast_block(be, blk, ess, root, group, vdtype):
    """SpParHelper::BCastMatrix: rank `root` of `group` sends its block's cp, jc, ir, num"""
    m, n, nnz, nzc = ess[root]
    if group.rank == root:
        cp, jc, ir, num = be.arrays(blk)
    else:
        dev = be.device
        cp = torch.empty(nzc + 1, dtype=torch.int64, device=dev)
        jc = torch.empty(nzc, dtype=torch.int64, device=dev)
        ir = torch.empty(nnz, dtype=torch.int32, device=dev)
        num = torch.empty(nnz, dtype=vdtype, device=dev)
    for t in (cp, jc, ir, num):
        bcast(t, root, group)
    return blk if group.rank == root else be.wrap(m, n, cp, jc, ir, num)


def _ibcast_block(be, blk, ess, root, group, vdtype):
    """SpParHelper::IBCastMatrix: the non-blocking form of _bcast_block -> (block, requests)"""
    m, n, nnz, nzc = ess[root]
    if group.rank == root:
        cp, jc, ir, num = be.arrays(blk)
    else:
        dev = be.device
        cp = torch.empty(nzc + 1, dtype=torch.int64, device=dev)
        jc = torch.empty(nzc, dtype=torch.int64, device=dev)
        ir = torch.empty(nnz, dtype=torch.int32, device=dev)
        num = torch.empty(nnz, dtype=vdtype, device=dev)
    reqs = [ibcast(t, root, group) for t in (cp, jc, ir, num)]
    return (blk if group.rank == root else be.wrap(m, n, cp, jc, ir, num)), reqs


def _rowrange(be, blk, r0, r1):
    """the entries of a block with rows in [r0, r1), same dimensions (Split of the transposed
    block in Mult_AnXBn_DoubleBuff, ParFriends.h:822-828, without the two transposes)"""
    m, n, nnz, nzc = be.dims(blk)
    cp, jc, ir, num = be.arrays(blk)
    if nnz == 0 or (r0 <= 0 and r1 >= m):
        return blk
    keep = (ir >= r0) & (ir < r1)
    col_of = torch.repeat_interleave(torch.arange(nzc, device=ir.device), cp[1:] - cp[:-1])
    cnt = torch.zeros(nzc, dtype=torch.int64, device=ir.device).index_add_(0, col_of, keep.to(torch.int64))
    nz = cnt > 0
    cpn = torch.zeros(int(nz.sum().item()) + 1, dtype=torch.int64, device=ir.device)
    cpn[1:] = torch.cumsum(cnt[nz], 0)
    return be.wrap(m, n, cpn, jc[nz].contiguous(), ir[keep].contiguous(), num[keep].contiguous())


def _hcat(be, blocks, m, vdtype):
    """[A_0 A_1 ...]: column concatenation of m x k_i blocks (column ids shifted by sum k_<i)"""
    dims = [be.dims(b) for b in blocks]
    kout = int(sum(d[1] for d in dims))
    live = [(b, off) for b, off, d in zip(blocks, np.cumsum([0] + [d[1] for d in dims])[:-1], dims) if d[3] > 0]
    if not live:
        return _empty(be, m, kout, vdtype)
    arrs = [be.arrays(b) for b, _ in live]
    cps, base = [], 0
    for i, (cp, jc, ir, num) in enumerate(arrs):
        cps.append((cp[:-1] if i + 1 < len(arrs) else cp) - cp[0] + base)
        base += int(ir.numel())
    return be.wrap(m, kout, torch.cat(cps), torch.cat([a[1] + int(off) for a, (_, off) in zip(arrs, live)]),
                   torch.cat([a[2] for a in arrs]), torch.cat([a[3] for a in arrs]))


def _vcat(be, blocks, n, vdtype):
    """[B_0; B_1; ...]: row concatenation of k_i x n blocks (row ids shifted by sum k_<i). A stable
    sort by column keeps every column's rows ascending (block i's rows all precede block i+1's)."""
    dims = [be.dims(b) for b in blocks]
    kout = int(sum(d[0] for d in dims))
    offs = np.cumsum([0] + [d[0] for d in dims])[:-1]
    cols, rows, vals = [], [], []
    for b, off, d in zip(blocks, offs, dims):
        if d[2] == 0:
            continue
        cp, jc, ir, num = be.arrays(b)
        cols.append(torch.repeat_interleave(jc, cp[1:] - cp[:-1]))
        rows.append(ir + int(off))
        vals.append(num)
    if not cols:
        return _empty(be, kout, n, vdtype)
    col = torch.cat(cols)
    key, perm = torch.sort(col, stable=True)
    jc, cnt = torch.unique_consecutive(key, return_counts=True)
    cp = torch.zeros(jc.numel() + 1, dtype=torch.int64, device=col.device)
    torch.cumsum(cnt, 0, out=cp[1:])
    return be.wrap(kout, n, cp, jc.contiguous(), torch.cat(rows)[perm].contiguous(), torch.cat(vals)[perm].contiguous())


def _stage_product_operands(be, A, B, grid, stages, Ab, Bb, vdtype):
    """The strips A(r, :) = [A_0 ... A_{s-1}] and B(:, c) = [B_0; ...; B_{s-1}] of this rank's C
    block. sum_i A_i B_i (the stage partials the reference merges, ParFriends.h:1064-1104) is then
    ONE local product over the inner dimension of all stages: the kernels accumulate every k, so
    no partial is materialised and no MultiwayMerge pass runs; C is the same matrix (integer and
    boolean semirings bit for bit; floating-point sums in another order). The received stage
    blocks are released once copied. One stage: the operands ARE A's and B's local blocks
    (_release_operands leaves those alone)."""
    m, n = be.dims(A.seq)[0], be.dims(B.seq)[1]
    if stages == 1:  # the rank's own blocks, used in place (no copy, no column sort of B)
        return Ab[0], Bb[0]
    Acat = _hcat(be, Ab, m, vdtype)
    Bcat = _vcat(be, Bb, n, vdtype)
    Aself, Bself = grid.GetRankInProcRow(), grid.GetRankInProcCol()
    for i in range(stages):
        if i != Aself and Ab[i] is not Acat:
            be.free(Ab[i])
        if i != Bself and Bb[i] is not Bcat:
            be.free(Bb[i])
    return Acat, Bcat


def _release_operands(be, A, B, Acat, Bcat):
    if Acat is not A.seq:
        be.free(Acat)
    if Bcat is not B.seq and Bcat is not Acat:
        be.free(Bcat)


def _check_dims(A, B):
    if A.getncol() != B.getnrow():
        raise CombBLASHipError(DIMMISMATCH, f"Can not multiply, dimensions does not match {A.getncol()} != {B.getnrow()}")
    if A.seq is B.seq:
        raise CombBLASHipError(3005, "A and B must not alias (ParFriends.h:172-179)")


def _stage_blocks(A, B, grid, stages):
    be = A.backend
    vdtype = be.value_dtype(A.seq)
    Aess = _essentials(be, A.seq, grid.rowWorld)
    Bess = _essentials(be, B.seq, grid.colWorld)
    Ab = [_bcast_block(be, A.seq, Aess, i, grid.rowWorld, vdtype) for i in range(stages)]
    Bb = [_bcast_block(be, B.seq, Bess, i, grid.colWorld, vdtype) for i in range(stages)]
    return Ab, Bb, vdtype


def _phase_cuts(be, plans, Bb, ncols, phases, budget_entries, groups=()):
    """Column ranges [c0, c1) of the local output block. With phases <= 0 they are planned from
    the exact per-column nnz of the stage partials, each phase's partials staying within
    budget_entries. The counts and the budget are reduced over every group in `groups` in turn
    (the ranks that share this block's column space: the processor column in 2D; the fiber, then
    the layer's processor column in 3D), so that every rank whose later collectives pair up
    (MCLPruneRecoverySelect's column reductions, the fiber reduce-scatter) cuts identically --
    the reference's equivalent is one global phase count (MPI_MAX over World, ParFriends.h:494)."""
    if phases and phases > 0:
        return [block_range(ncols, phases, p) for p in range(phases)]
    t = torch.tensor([budget_entries], dtype=torch.int64, device=be.device)
    for g in groups:
        allreduce_(t, g, torch.distributed.ReduceOp.MIN)
    budget_entries = int(t.item())
    col = torch.zeros(ncols + 1, dtype=torch.int64, device=be.device)
    for p, b in zip(plans, Bb):
        if be.dims(b)[3]:
            col.index_add_(0, be.arrays(b)[1], p.col_nnz())
    for g in groups:
        allreduce_(col, g)
    cum = np.concatenate([[0], np.cumsum(col[:ncols].cpu().numpy())])
    cuts, c0 = [], 0
    while c0 < ncols:
        c1 = int(np.searchsorted(cum, cum[c0] + budget_entries, side="right")) - 1
        c1 = min(max(c1, c0 + 1), ncols)
        cuts.append((c0, c1))
        c0 = c1
    return cuts or [(0, ncols)]


def _budget_entries(be, vdtype, perProcessMemory, copies):
    if perProcessMemory and perProcessMemory > 0:
        budget = perProcessMemory
    else:
        free, _ = torch.cuda.mem_get_info(be.device) if be.device.type == "cuda" else (1 << 34, 0)
        budget = int(free * 0.4)
    esz = 4 + torch.empty(0, dtype=vdtype).element_size()
    return max(1, budget // (esz * copies))


# ---------------------------------------------------------------------------------- 2D
def Mult_AnXBn_Synch(SR, A: SpParMat, B: SpParMat, clearA=False, clearB=False) -> SpParMat:
    """C = A*B by 2D SUMMA (ParFriends.h:1004-1108); received blocks are dropped after their stage."""
    _check_dims(A, B)
    grid, stages = ProductGrid(A.commGrid, B.commGrid)
    be = A.backend
    vdtype = be.value_dtype(A.seq)
    Aess = _essentials(be, A.seq, grid.rowWorld)
    Bess = _essentials(be, B.seq, grid.colWorld)
    Aself, Bself = grid.GetRankInProcRow(), grid.GetRankInProcCol()
    m, n = be.dims(A.seq)[0], be.dims(B.seq)[1]
    tomerge = []
    for i in range(stages):
        Ai = _bcast_block(be, A.seq, Aess, i, grid.rowWorld, vdtype)
        Bi = _bcast_block(be, B.seq, Bess, i, grid.colWorld, vdtype)
        tomerge.append(be.multiply(SR, Ai, Bi))
        if i != Aself:
            be.free(Ai)
        if i != Bself:
            be.free(Bi)
    C = _merge(be, SR, tomerge, m, n, vdtype)
    if clearA:
        be.free(A.seq)
    if clearB:
        be.free(B.seq)
    return SpParMat(C, grid, be, A.m, B.n, A.row_off, B.col_off)


def Mult_AnXBn_Overlap(SR, A: SpParMat, B: SpParMat, clearA=False, clearB=False) -> SpParMat:
    """2D SUMMA with communication overlapped (ParFriends.h:1110-1235): the broadcasts of stage
    i+1 are posted before stage i's local multiply, so RCCL moves the next blocks over xGMI while
    the gfx950 kernels run. Same result as Mult_AnXBn_Synch."""
    _check_dims(A, B)
    grid, stages = ProductGrid(A.commGrid, B.commGrid)
    be = A.backend
    vdtype = be.value_dtype(A.seq)
    Aess = _essentials(be, A.seq, grid.rowWorld)
    Bess = _essentials(be, B.seq, grid.colWorld)
    Aself, Bself = grid.GetRankInProcRow(), grid.GetRankInProcCol()
    m, n = be.dims(A.seq)[0], be.dims(B.seq)[1]

    def post(i):
        return (_ibcast_block(be, A.seq, Aess, i, grid.rowWorld, vdtype),
                _ibcast_block(be, B.seq, Bess, i, grid.colWorld, vdtype))

    tomerge = []
    nxt = post(0)
    for i in range(stages):
        (Ai, ra), (Bi, rb) = nxt
        for r in ra + rb:
            r.wait()
        if i + 1 < stages:
            nxt = post(i + 1)
        tomerge.append(be.multiply(SR, Ai, Bi))
        if i != Aself:
            be.free(Ai)
        if i != Bself:
            be.free(Bi)
    C = _merge(be, SR, tomerge, m, n, vdtype)
    if clearA:
        be.free(A.seq)
    if clearB:
        be.free(B.seq)
    return SpParMat(C, grid, be, A.m, B.n, A.row_off, B.col_off)


def Mult_AnXBn_DoubleBuff(SR, A: SpParMat, B: SpParMat, clearA=False, clearB=False) -> SpParMat:
    """ParFriends.h:798-997: A's local block is split by columns and B's by rows at the same
    point (A1*B1 + A2*B2 = A*B), and every stage multiplies the two halves in turn, so the
    received buffers hold half blocks. The 2*stages partials are merged once. The next half's
    broadcasts are posted before the current half is multiplied (as in Mult_AnXBn_Overlap)."""
    _check_dims(A, B)
    grid, stages = ProductGrid(A.commGrid, B.commGrid)
    be = A.backend
    vdtype = be.value_dtype(A.seq)
    m, n = be.dims(A.seq)[0], be.dims(B.seq)[1]
    # SpDCCols::Split at ncol/2 (SpDCCols.cpp): every rank splits its own A block's columns and
    # its own B block's rows; at stage i both come from blocks of inner dimension k_i, so the
    # halves broadcast in one step always pair up
    ka, kb = be.dims(A.seq)[1], be.dims(B.seq)[0]
    halves = [(_colslice(be, A.seq, 0, ka // 2), _rowrange(be, B.seq, 0, kb // 2)),
              (_colslice(be, A.seq, ka // 2, ka), _rowrange(be, B.seq, kb // 2, kb))]
    ess = [(_essentials(be, a, grid.rowWorld), _essentials(be, b, grid.colWorld)) for a, b in halves]
    Aself, Bself = grid.GetRankInProcRow(), grid.GetRankInProcCol()
    order = [(i, x) for i in range(stages) for x in range(2)]

    def post(j):
        i, x = order[j]
        (a, b), (ea, eb) = halves[x], ess[x]
        return (_ibcast_block(be, a, ea, i, grid.rowWorld, vdtype), _ibcast_block(be, b, eb, i, grid.colWorld, vdtype))

    tomerge = []
    nxt = post(0)
    for j, (i, x) in enumerate(order):
        (Ai, ra), (Bi, rb) = nxt
        for r in ra + rb:
            r.wait()
        if j + 1 < len(order):
            nxt = post(j + 1)
        tomerge.append(be.multiply(SR, Ai, Bi))
        if i != Aself:
            be.free(Ai)
        if i != Bself:
            be.free(Bi)
    C = _merge(be, SR, tomerge, m, n, vdtype)
    if clearA:
        be.free(A.seq)
    if clearB:
        be.free(B.seq)
    return SpParMat(C, grid, be, A.m, B.n, A.row_off, B.col_off)


def MemEfficientSpGEMM(SR, A: SpParMat, B: SpParMat, phases=0, hardThreshold=None, selectNum=0, recoverNum=0,
                       recoverPct=0.0, kselectVersion=1, computationKernel=1, perProcessMemory=0, on_phase=None):
    """Phased 2D SUMMA (ParFriends.h:449-730; same argument order). phases=0 plans the phases
    from the exact symbolic pass and `perProcessMemory` bytes (default 40 % of free HBM). With a
    hardThreshold every phase's block goes through MCLPruneRecoverySelect (:698) before it is
    kept. on_phase(C_block, c0, c1) consumes each phase's block of C (local columns [c0, c1));
    without it the phases are concatenated and the SpParMat C is returned. computationKernel
    (hash / heap) selects the same device kernel: both contracts are met by it."""
    _check_dims(A, B)
    grid, stages = ProductGrid(A.commGrid, B.commGrid)
    be = A.backend
    Ab, Bb, vdtype = _stage_blocks(A, B, grid, stages)
    m, n = be.dims(A.seq)[0], be.dims(B.seq)[1]
    Acat, Bcat = _stage_product_operands(be, A, B, grid, stages, Ab, Bb, vdtype)
    plans = [be.plan(Acat, Bcat)]  # one symbolic pass for every phase
    cuts = _phase_cuts(be, plans, [Bcat], n, phases, _budget_entries(be, vdtype, perProcessMemory, 1),
                       groups=(grid.colWorld,))
    out = []
    for c0, c1 in cuts:
        C = plans[0].multiply(SR, c0, c1)
        if hardThreshold is not None:
            C = _mcl_block(be, C, grid.colWorld, hardThreshold, selectNum, recoverNum, recoverPct)
        if on_phase is not None:
            on_phase(C, c0, c1)
        else:
            out.append(C)
    for p in plans:
        p.close()
    _release_operands(be, A, B, Acat, Bcat)
    if on_phase is not None:
        return len(cuts)
    return SpParMat(_concat_cols(be, out, m, n, vdtype), grid, be, A.m, B.n, A.row_off, B.col_off)


# ---------------------------------------------------------------------------------- 3D
def _divisions3d(ncols, nlayers):
    """SpParMat3D::CalculateColSplitDistributionOfLayer (non-special), SpParMat3D.cpp:592-605"""
    y = ncols // nlayers
    return [y] * (nlayers - 1) + [ncols - (nlayers - 1) * y]


def _fiber_reduce_scatter(be, SR, P, grid3, m, ncols, vdtype):
    """ParFriends.h:3097-3183: column chunk j of the layer partial P goes to fiber rank j; the
    received pieces of this rank's chunk are merged. Returns (block, chunk start)."""
    L, me = grid3.gridLayers, grid3.rankInFiber
    fib = grid3.fiberWorld
    div = _divisions3d(ncols, L)
    starts = np.concatenate([[0], np.cumsum(div)]).astype(np.int64)
    cp, jc, ir, num = be.arrays(P)
    dev = be.device
    bounds = torch.searchsorted(jc, torch.tensor(starts, dtype=torch.int64, device=dev))
    cpb = cp[bounds]
    slot_b, ent_b = bounds.cpu().tolist(), cpb.cpu().tolist()
    s_nzc = [slot_b[j + 1] - slot_b[j] for j in range(L)]
    s_nnz = [ent_b[j + 1] - ent_b[j] for j in range(L)]
    lo = ent_b[0]
    prof = torch.tensor([v for j in range(L) for v in (s_nzc[j], s_nnz[j])], dtype=torch.int64, device=dev)
    rprof = alltoallv(prof, [2] * L, [2] * L, fib).cpu().tolist()
    r_nzc, r_nnz = rprof[0::2], rprof[1::2]
    s0, s1 = slot_b[0], slot_b[L]
    collen = (cp[s0 + 1:s1 + 1] - cp[s0:s1]).contiguous()
    rjc = alltoallv(jc[s0:s1], s_nzc, r_nzc, fib)
    rlen = alltoallv(collen, s_nzc, r_nzc, fib)
    rir = alltoallv(ir[lo:ent_b[L]], s_nnz, r_nnz, fib)
    rnum = alltoallv(num[lo:ent_b[L]], s_nnz, r_nnz, fib)
    c0, w = int(starts[me]), int(div[me])
    pieces, a, b = [], 0, 0
    for j in range(L):
        if r_nzc[j]:
            cpj = torch.zeros(r_nzc[j] + 1, dtype=torch.int64, device=dev)
            torch.cumsum(rlen[a:a + r_nzc[j]], 0, out=cpj[1:])
            pieces.append(be.wrap(m, w, cpj, rjc[a:a + r_nzc[j]] - c0, rir[b:b + r_nnz[j]], rnum[b:b + r_nnz[j]]))
        a += r_nzc[j]
        b += r_nnz[j]
    return _merge(be, SR, pieces, m, w, vdtype), c0


def Mult_AnXBn_SUMMA3D(SR, A: SpParMat3D, B: SpParMat3D, phases=1, perProcessMemory=0, on_phase=None):
    """C = A*B on a 3D grid (A column-split, B row-split). Returns the column-split SpParMat3D C,
    or, with on_phase, feeds every phase's piece of this rank's C chunk to on_phase(C, c0, c1)
    (local columns of the chunk) and returns the number of phases. phases=0 plans them from the
    exact symbolic pass (the reference's MemEfficientSpGEMM3D phase loop, ParFriends.h:3200-3520)."""
    _check_dims(A, B)
    if not A.colsplit or B.colsplit:
        raise CombBLASHipError(DIMMISMATCH, "Mult_AnXBn_SUMMA3D needs a column-split A and a row-split B")
    g3 = A.commGrid3D
    grid, stages = ProductGrid(g3.commGridLayer, B.commGrid3D.commGridLayer)
    be = A.backend
    Ab, Bb, vdtype = _stage_blocks(A, B, grid, stages)
    m, n = be.dims(A.seq)[0], be.dims(B.seq)[1]
    Acat, Bcat = _stage_product_operands(be, A, B, grid, stages, Ab, Bb, vdtype)
    plans = [be.plan(Acat, Bcat)]  # one symbolic pass for every phase
    cuts = _phase_cuts(be, plans, [Bcat], n, phases, _budget_entries(be, vdtype, perProcessMemory, 2),
                       groups=(g3.fiberWorld, grid.colWorld))
    div = _divisions3d(n, g3.gridLayers)
    out, mine0 = [], 0
    for c0, c1 in cuts:
        P = plans[0].multiply(SR, c0, c1)
        C, mine0 = _fiber_reduce_scatter(be, SR, P, g3, m, n, vdtype)
        w = div[g3.rankInFiber]
        p0, p1 = min(max(c0 - mine0, 0), w), min(max(c1 - mine0, 0), w)
        if on_phase is not None:
            on_phase(C, p0, p1)
        else:
            out.append(C)
    for p in plans:
        p.close()
    _release_operands(be, A, B, Acat, Bcat)
    if on_phase is not None:
        return len(cuts)
    w = div[g3.rankInFiber]
    Cb = _concat_cols(be, out, m, w, vdtype)
    return SpParMat3D(Cb, g3, be, A.m, B.n, True, A.row_off, B.col_off + mine0)


def MemEfficientSpGEMM3D(SR, A: SpParMat3D, B: SpParMat3D, phases=1, hardThreshold=None, selectNum=0, recoverNum=0,
                         recoverPct=0.0, kselectVersion=1, computationKernel=1, perProcessMemory=0):
    """HipMCL's 3D expansion (ParFriends.h:3215-3700): per phase the layer SUMMA, the fiber
    reduce-scatter, then MCLPruneRecoverySelect on the phase's piece as a matrix of the layer's
    2D grid (:3683-3686: column statistics reduce over the layer's processor column)."""
    g3 = A.commGrid3D
    be = A.backend
    colgroup = g3.commGridLayer.colWorld
    got = []

    def keep(C, p0, p1):
        if hardThreshold is not None:
            C = _mcl_block(be, C, colgroup, hardThreshold, selectNum, recoverNum, recoverPct)
        got.append(C)

    Mult_AnXBn_SUMMA3D(SR, A, B, phases=phases, perProcessMemory=perProcessMemory, on_phase=keep)
    m, w = be.dims(got[0])[0], be.dims(got[0])[1]
    div = _divisions3d(be.dims(B.seq)[1], g3.gridLayers)
    mine0 = sum(div[:g3.rankInFiber])
    Cb = _concat_cols(be, got, m, w, be.value_dtype(A.seq))
    return SpParMat3D(Cb, g3, be, A.m, B.n, True, A.row_off, B.col_off + mine0)


# ---------------------------------------------------------------------------- TC / MCL callers
def EWiseMult(A: SpParMat, B: SpParMat, exclude=False) -> SpParMat:
    """SpParMat::EWiseMult(B, false) (SpParMat.cpp, Friends.h:834-887) on identically distributed
    matrices: the local blocks are intersected, values multiplied (TC.cpp:110)."""
    if exclude:
        raise NotImplementedError("EWiseMult(exclude=true) (SetDifference) is outside the hot-path scope")
    be = A.backend
    return SpParMat(be.ewise_mult(A.seq, B.seq), A.commGrid, be, A.m, A.n, A.row_off, A.col_off)


def ColumnStats(be, blk, hard, colgroup=None):
    """per-column (nnz, nnz of v > hard, sum of v > hard) of the distributed matrix's local
    columns, summed over the processor column (A.Reduce(Column, ...), ParFriends.h:196-200)"""
    cnt, cntp, sump = be.col_stats(blk, hard)
    if colgroup is not None:
        for t in (cnt, cntp, sump):
            allreduce_(t, colgroup)
    return cnt, cntp, sump


def Kselect(be, blk, active, k, colgroup=None, total=None):
    """k-th largest value of every active column (SpParMat::Kselect1, SpParMat.cpp:1413-1700):
    sorted descending, element k-1; the smallest when the column has fewer than k entries;
    numeric_limits<double>::min() when it is empty. Radix select over order-preserving keys, 8
    bits per pass, the digit histograms summed over the processor column (instead of gathering
    every rank's top-k list up the column as the reference does). Returns a dense f64 vector
    (NaN outside `active`)."""
    dev = be.device
    n = be.dims(blk)[1]
    kth = torch.full((n,), float("nan"), dtype=torch.float64, device=dev)
    act = torch.nonzero(active).flatten()
    nact = int(act.numel())
    if nact == 0:
        return kth
    if total is None:
        total = ColumnStats(be, blk, float("-inf"), colgroup)[0]
    aidx = torch.full((n,), -1, dtype=torch.int32, device=dev)
    aidx[act] = torch.arange(nact, dtype=torch.int32, device=dev)
    if _whole_columns(colgroup) and hasattr(be, "kselect_cols"):  # one launch, columns staged in LDS
        kth[act] = be.kselect_cols(blk, aidx, nact, k)
        return kth
    tot = total[act].to(torch.int64)
    rank = torch.where(tot >= k, torch.full_like(tot, k - 1), tot - 1).contiguous()
    prefix = torch.zeros(nact, dtype=torch.int64, device=dev)  # uint64 key bits
    for shift in range(56, -1, -8):
        hist = be.kselect_hist(blk, aidx, nact, prefix, shift)
        if colgroup is not None:
            allreduce_(hist, colgroup)
        be.kselect_pick(nact, hist, prefix, rank, shift)
    vals = be.kselect_value(nact, prefix)
    kth[act] = torch.where(tot > 0, vals, torch.full_like(vals, 2.2250738585072014e-308))
    return kth


def _whole_columns(colgroup):
    """the block holds its columns whole (no processor column to sum over)"""
    return colgroup is None or getattr(colgroup, "size", 1) == 1


def _kept_stats(be, A, prune, colgroup):
    """(count, sum) per column of PruneColumn(A, prune) -- the recovery check of ParFriends.h:318-329"""
    if _whole_columns(colgroup) and hasattr(be, "col_stats_kept"):
        return be.col_stats_kept(A, prune)  # without forming the pruned matrix
    S = be.prune_columns(A, prune)
    _, cnt1, sum1 = ColumnStats(be, S, float("-inf"), colgroup)
    be.free(S)
    return cnt1, sum1


def _mcl_block(be, A, colgroup, hardThreshold, selectNum, recoverNum, recoverPct):
    """ParFriends.h:185-353 on a local block whose columns may be split over `colgroup` (a block
    holding its columns whole: one device call, cbh_mcl_prune_recovery_select)"""
    if _whole_columns(colgroup) and hasattr(be, "mcl_prune_block"):
        out = be.mcl_prune_block(A, hardThreshold, selectNum, recoverNum, recoverPct)
        be.free(A)
        return out
    cnt, cntp, sump = ColumnStats(be, A, hardThreshold, colgroup)  # unpruned nnz, pruned nnz, pruned sums
    prune = torch.full_like(cnt, hardThreshold)
    rec = (cntp < recoverNum) & (cnt > cntp) & (sump < recoverPct)
    if bool(rec.any()):
        prune = torch.where(rec, Kselect(be, A, rec, recoverNum, colgroup, cnt), prune)
    if selectNum > 0:
        sel = ~rec & (cntp > selectNum)
        if bool(sel.any()):
            prune = torch.where(sel, Kselect(be, A, sel, selectNum, colgroup, cnt), prune)
            if recoverNum > 0:
                cnt1, sum1 = _kept_stats(be, A, prune, colgroup)
                s2 = sel & (cnt1 < recoverNum) & (sum1 < recoverPct)
                if bool(s2.any()):
                    prune = torch.where(s2, Kselect(be, A, s2, recoverNum, colgroup, cnt), prune)
    out = be.prune_columns(A, prune)
    be.free(A)
    return out


def MCLPruneRecoverySelect(A: SpParMat, hardThreshold, selectNum, recoverNum, recoverPct, kselectVersion=1):
    """ParFriends.h:185-353: prune entries below per-column thresholds -- hardThreshold, or the
    selectNum-th / recoverNum-th largest entry for columns needing selection / recovery. A is
    pruned in place (its local block replaced), as in the reference."""
    A.seq = _mcl_block(A.backend, A.seq, A.commGrid.colWorld, hardThreshold, selectNum, recoverNum, recoverPct)
    return A


def PSpGEMM(SR, A, B, **kw):
    """SpParMat.h:454-467 -- the product of two distributed matrices on their grid."""
    if isinstance(A, SpParMat3D):
        return Mult_AnXBn_SUMMA3D(SR, A, B, **kw)
    return Mult_AnXBn_Synch(SR, A, B, **kw)
