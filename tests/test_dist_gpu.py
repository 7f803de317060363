"""Distributed drivers on the GPU: several ranks share cuda:0 (one test box has one MI355X), the
local multiply / merge / symbolic run in the gfx950 kernels (HipBackend) and the collectives go
through gloo with host staging (RCCL refuses two ranks on one device; on a node every rank owns
its GPU and the same code runs over RCCL). The assembled C must match the single-block oracle
product and the reference's digests bit for bit.
"""
import numpy as np
import pytest

import helpers as H
from dist_util import run_world

pytestmark = pytest.mark.gpu


def _trace(rank, msg):
    """CBH_TRACE_DIR: each rank appends its progress (flushed) to rank<r>.log there"""
    import os
    import time

    d = os.environ.get("CBH_TRACE_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"rank{rank}.log"), "a") as f:
            f.write(f"{time.time():.3f} {msg}\n")


def _gpu_worker(rank, world, scale, tag, mode, phases, budget, layers):
    import torch

    import combblas_amd as cb
    from combblas_amd import parfriends as pf
    from combblas_amd.backend import HipBackend
    from combblas_amd.commgrid import CommGrid, CommGrid3D
    from combblas_amd.semirings import ALL
    from combblas_amd.spparmat import SpParMat, SpParMat3D

    _trace(rank, f"start {tag} {mode}")
    torch.cuda.set_device(0)
    ctx = cb.Context(0)
    be = HipBackend(ctx)
    _trace(rank, "context")
    A = cb.rmat(scale)
    d = H.values_for(tag, H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))
    h = cb.HostDcsc(d.m, d.n, d.jc, d.cp, d.ir, d.num)
    SR = ALL[{"pt_i64": "PlusTimesSRing", "pt_f64": "PlusTimesSRing", "max_i64": "SelectMaxSRing",
              "min_i64": "MinPlusSRing", "bool": "OrAndSRing"}[tag]]
    if mode == "3d":
        g3 = CommGrid3D(layers)
        dA = SpParMat3D.distribute(h, g3, be, colsplit=True)
        dB = SpParMat3D.distribute(h, g3, be, colsplit=False)
        C = pf.Mult_AnXBn_SUMMA3D(SR, dA, dB, phases=phases, perProcessMemory=budget)
    else:
        grid = CommGrid()
        dA = SpParMat.distribute(h, grid, be)
        dB = SpParMat.distribute(h, grid, be)
        if mode == "synch":
            _trace(rank, "distributed")
            C = pf.Mult_AnXBn_Synch(SR, dA, dB)
        elif mode == "overlap":
            C = pf.Mult_AnXBn_Overlap(SR, dA, dB)
        elif mode == "doublebuff":
            C = pf.Mult_AnXBn_DoubleBuff(SR, dA, dB)
        else:
            C = pf.MemEfficientSpGEMM(SR, dA, dB, phases=phases, perProcessMemory=budget)
    _trace(rank, "product")
    g = C.gather_host()
    torch.cuda.synchronize()
    _trace(rank, "gathered")
    ctx.close()
    if rank == 0:
        return (g.m, g.n, g.jc, g.cp, g.ir, g.num)
    return None


def _check(res, golden):
    m, n, jc, cp, ir, num = res
    got = H.Dcsc(m, n, jc, cp, ir, num)
    vs, dg = H.digest(got)
    assert (got.nnz, got.nzc) == (golden["nnz"], golden["nzc"])
    assert vs == golden["sum"] and dg == int(golden["digest"])


@pytest.mark.parametrize("tag", ["pt_i64", "max_i64"])
def test_gpu_summa2d_2x2(golden, tag):
    res = run_world(_gpu_worker, 4, 12, tag, "synch", 1, 0, 1, timeout=150)
    _check(res, golden["digests"][f"rmat12_{tag}"])


@pytest.mark.parametrize("mode", ["overlap", "doublebuff"])
def test_gpu_summa2d_overlap_doublebuff(golden, mode):
    """Mult_AnXBn_Overlap / Mult_AnXBn_DoubleBuff (non-blocking stage broadcasts) on the device"""
    res = run_world(_gpu_worker, 4, 12, "pt_i64", mode, 1, 0, 1, timeout=150)
    _check(res, golden["digests"]["rmat12_pt_i64"])


def test_gpu_summa2d_phased(golden):
    res = run_world(_gpu_worker, 4, 12, "pt_f64", "phased", 0, 12 * 2 * 60000, 1, timeout=150)
    _check(res, golden["digests"]["rmat12_pt_f64"])


def test_gpu_summa3d_1x1x2(golden):
    res = run_world(_gpu_worker, 2, 12, "bool", "3d", 0, 12 * 3 * 80000, 2, timeout=150)
    _check(res, golden["digests"]["rmat12_bool"])


def test_gpu_summa3d_2x2x2(golden):
    res = run_world(_gpu_worker, 8, 12, "pt_i64", "3d", 2, 0, 2, timeout=150)
    _check(res, golden["digests"]["rmat12_pt_i64"])


def _gpu_ccgrid_worker(rank, world, scale, tag, c, g):
    """the standalone 3D API (spgemm3d: CCGrid / SplitMat / multiply) on the device"""
    import torch

    import combblas_amd as cb
    from combblas_amd import spgemm3d as s3
    from combblas_amd.backend import HipBackend
    from combblas_amd.spparmat import SpParMat, _gather, block_range

    torch.cuda.set_device(0)
    ctx = cb.Context(0)
    be = HipBackend(ctx)
    A = cb.rmat(scale)
    d = H.values_for(tag, H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))
    h = cb.HostDcsc(d.m, d.n, d.jc, d.cp, d.ir, d.num)
    CMG = s3.CCGrid(c, g)
    vdt = {"pt_i64": torch.int64, "pt_f64": torch.float64}[tag]
    root = CMG.layer_grid == 0
    sA = s3.SplitMat(CMG, SpParMat.distribute(h, CMG.layerGrid, be).seq if root else None, be, False, vdt)
    sB = s3.SplitMat(CMG, SpParMat.distribute(h, CMG.layerGrid, be).seq if root else None, be, True, vdt)
    C = s3.multiply(sA, sB, CMG, False, True, be)
    r0 = block_range(d.m, g, CMG.RankInCol)[0]
    c0, c1 = block_range(d.n, g, CMG.RankInRow)
    G = _gather(be, C, r0, c0 + CMG.layer_grid * ((c1 - c0) // c), d.m, d.n)
    torch.cuda.synchronize()
    ctx.close()
    if rank == 0:
        return (G.m, G.n, G.jc, G.cp, G.ir, G.num)
    return None


def test_gpu_ccgrid_multiply_2x2x2(golden):
    res = run_world(_gpu_ccgrid_worker, 8, 12, "pt_i64", 2, 2, timeout=150)
    _check(res, golden["digests"]["rmat12_pt_i64"])
