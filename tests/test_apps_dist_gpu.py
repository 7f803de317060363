"""GPU: configs C3 and C5 through the distributed drivers of parfriends.py with the gfx950
kernels (HipBackend) doing every local multiply, merge, symbolic pass and MCL column operation.
Ranks share cuda:0 (one MI355X per test box) and exchange over gloo with host staging; on a node
every rank owns its GPU and the same driver code runs over RCCL.

  C3 Galerkin  SAT = T' (A T), two PSpGEMM on 2x2 (GalerkinNew.cpp:101-123) -> the reference's own
               SAT bit for bit (dyadic values)
  C5 MCL       MemEfficientSpGEMM + MCLPruneRecoverySelect on 2x2 and MemEfficientSpGEMM3D on
               2x2x2 (ParFriends.h:449-730, 3214-3705; prune :185-353), fixed phases and phases=0
               (planned from the exact symbolic pass under a small per-process budget) -> the
               reference's expanded matrix mcl_A2 (1e-12) and the oracle prune of it (structure exact,
               values 1e-12: the pruned and the unpruned device runs sum in LDS-atomic order)
(the CPU twin of this file, with the oracle backend: tests/test_apps_dist_cpu.py)
"""
import pytest

import helpers as H
from dist_util import run_world
from test_apps_dist_cpu import _dc, _galerkin_worker, _mcl_worker, check_mcl, mcl_params

pytestmark = pytest.mark.gpu


def test_gpu_galerkin_2x2_vs_reference(apps):
    got = _dc(run_world(_galerkin_worker, 4, "hip", timeout=150))
    H.assert_dcsc_equal(got, apps["gal_SAT"], msg="Galerkin SAT on 2x2 (HIP)")


@pytest.mark.parametrize("mode,world,phases,ppm", [("2d", 4, 3, 0), ("3d", 8, 2, 0), ("2d", 4, 0, 96 * 1024),
                                                    ("3d", 8, 0, 64 * 1024)])
def test_gpu_mcl_prune_distributed(apps, apps_meta, mode, world, phases, ppm):
    res = run_world(_mcl_worker, world, mode, mcl_params(apps_meta), phases, ppm, "hip", timeout=200)
    check_mcl(apps, apps_meta, mode, res, rtol=1e-12)
