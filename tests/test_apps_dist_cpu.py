"""Configs C3-C5 on CPU processes (gloo) through the distributed drivers of parfriends.py, the
local-block operations supplied by the oracle backend (tests/dist_util.OracleBackend):

  C3 Galerkin  SAT = T' (A T) with two Mult_AnXBn_Synch on 2x2 (GalerkinNew.cpp:100-106) -> the
               reference's own SAT, bit for bit (dyadic values)
  C4 TC        C = EWiseMult(Mult_AnXBn_Synch(L, L), L) on 2x2 (TC.cpp:108-110) -> the reference's C
               and triangle count
  C5 MCL       MemEfficientSpGEMM with MCLPruneRecoverySelect on 2x2 (phased) and
               MemEfficientSpGEMM3D on 2x2x2: column statistics and the Kselect radix histograms
               are reduced over the processor column; the result must equal the one-block oracle
               prune of the same expanded matrix, and that matrix the reference's (1e-12)
"""
import os
import sys

import numpy as np
import pytest

import helpers as H
from dist_util import OracleBackend, run_world

sys.path.insert(0, os.path.join(H.REPO, "oracle"))
import apps_oracle as AO  # noqa: E402


def _h(d):
    import combblas_amd as cb

    return cb.HostDcsc(d.m, d.n, d.jc, d.cp, d.ir, d.num)


def _out(g):
    return (g.m, g.n, g.jc, g.cp, g.ir, g.num)


def _dc(res):
    return H.Dcsc(*res[:2], *res[2:])


def _backend(kind):
    """local-block operations: the CPU oracle (this file) or the gfx950 kernels with every rank
    sharing cuda:0 (tests/test_apps_dist_gpu.py; the collectives stay on gloo)"""
    if kind == "oracle":
        return OracleBackend(), None
    import torch

    import combblas_amd as cb
    from combblas_amd.backend import HipBackend

    torch.cuda.set_device(0)
    ctx = cb.Context(0)
    return HipBackend(ctx), ctx


def _close(ctx):
    if ctx is not None:
        import torch

        torch.cuda.synchronize()
        ctx.close()


def _galerkin_worker(rank, world, kind="oracle"):
    from combblas_amd import parfriends as pf
    from combblas_amd.commgrid import CommGrid
    from combblas_amd.galerkin import poisson27, prolongation, transpose
    from combblas_amd.semirings import PlusTimesSRing
    from combblas_amd.spparmat import SpParMat

    (be, ctx), grid = _backend(kind), CommGrid()
    A = SpParMat.distribute(poisson27(8), grid, be)
    T = SpParMat.distribute(prolongation(8), grid, be)
    S = SpParMat.distribute(transpose(prolongation(8)), grid, be)
    AT = pf.PSpGEMM(PlusTimesSRing, A, T)
    SAT = pf.PSpGEMM(PlusTimesSRing, S, AT)
    g = SAT.gather_host()
    _close(ctx)
    return _out(g) if rank == 0 else None


def test_galerkin_2x2_vs_reference(apps):
    got = _dc(run_world(_galerkin_worker, 4))
    H.assert_dcsc_equal(got, apps["gal_SAT"], msg="Galerkin SAT on 2x2")


def _tc_worker(rank, world, scale):
    from test_apps_oracle import tc_lower

    from combblas_amd import parfriends as pf
    from combblas_amd.commgrid import CommGrid
    from combblas_amd.semirings import PlusTimesSRing
    from combblas_amd.spparmat import SpParMat

    be, grid = OracleBackend(), CommGrid()
    L = _h(tc_lower(scale))
    La, Lb = SpParMat.distribute(L, grid, be), SpParMat.distribute(L, grid, be)
    C = pf.EWiseMult(pf.Mult_AnXBn_Synch(PlusTimesSRing, La, Lb), La)
    g = C.gather_host()
    return _out(g) if rank == 0 else None


def test_tc_2x2_vs_reference(apps, apps_meta):
    got = _dc(run_world(_tc_worker, 4, 10))
    H.assert_dcsc_equal(got, apps["tc10_C"], msg="TC (L*L).*L on 2x2")
    assert int(got.num.sum()) == apps_meta["tc"]["10"]["triangles"] == 78452


def _mcl_worker(rank, world, mode, params, phases, ppm=0, kind="oracle"):
    from combblas_amd import parfriends as pf
    from combblas_amd.commgrid import CommGrid, CommGrid3D
    from combblas_amd.semirings import PlusTimesSRing
    from combblas_amd.spparmat import SpParMat, SpParMat3D

    be, ctx = _backend(kind)
    A = _h(H.load_npz(os.path.join(H.GOLDEN, "apps.npz"))["mcl_A"])
    hard, sel, rec, pct = params
    res = []
    for prune in (False, True):
        kw = dict(hardThreshold=hard, selectNum=sel, recoverNum=rec, recoverPct=pct) if prune else {}
        if mode == "3d":
            g3 = CommGrid3D(2)
            dA = SpParMat3D.distribute(A, g3, be, colsplit=True)
            dB = SpParMat3D.distribute(A, g3, be, colsplit=False)
            C = pf.MemEfficientSpGEMM3D(PlusTimesSRing, dA, dB, phases=phases, perProcessMemory=ppm, **kw)
        else:
            grid = CommGrid()
            dA, dB = SpParMat.distribute(A, grid, be), SpParMat.distribute(A, grid, be)
            C = pf.MemEfficientSpGEMM(PlusTimesSRing, dA, dB, phases=phases, perProcessMemory=ppm, **kw)
        res.append(C.gather_host())
    _close(ctx)
    return (_out(res[0]), _out(res[1])) if rank == 0 else None


# phases=0 plans the phases from the exact symbolic pass under a small per-process budget (many
# phases; every rank's local counts differ): the cuts must still agree across the ranks whose
# column reductions pair up, or the prune's collectives would hang or mix columns
@pytest.mark.parametrize("mode,world,phases,ppm", [("2d", 4, 3, 0), ("3d", 8, 2, 0), ("2d", 4, 0, 96 * 1024),
                                                    ("3d", 8, 0, 64 * 1024)])
def test_mcl_prune_distributed(apps, apps_meta, mode, world, phases, ppm):
    check_mcl(apps, apps_meta, mode, run_world(_mcl_worker, world, mode, mcl_params(apps_meta), phases, ppm))


def mcl_params(apps_meta):
    p = apps_meta["mcl"]["0"]
    return (p["hard"], p["select"], p["recover"], p["pct"])


def check_mcl(apps, apps_meta, mode, res, rtol=0.0):
    """rtol: the device accumulates non-dyadic f64 sums in LDS-atomic arrival order, so the pruned run
    and the unpruned run of the same product may differ in the last bits (north_star's 1e-12)"""
    params = mcl_params(apps_meta)
    raw, pruned = res
    A2, got = _dc(raw), _dc(pruned)
    ref = apps["mcl_A2"]
    assert np.array_equal(A2.jc, ref.jc) and np.array_equal(A2.cp, ref.cp) and np.array_equal(A2.ir, ref.ir)
    np.testing.assert_allclose(A2.num, ref.num, rtol=1e-12, atol=0)
    H.assert_dcsc_equal(got, AO.mcl_prune_recovery_select(A2, *params), rtol=rtol, msg=f"MCL prune {mode}")
    assert got.nnz == pytest.approx(apps["mcl_out0"].nnz, rel=0.01)
