"""The standalone 3D SpGEMM API (combblas_amd/spgemm3d.py: 3DSpGEMM/CCGrid.h, SplitMatDist.h,
SUMMALayer.h, Reductions.h, Multiplier.h) on CPU processes (gloo), driven the way
3DSpGEMM/mpipspgemm.cpp drives it: layer 0 holds A and B on its 2D grid, SplitMat column-splits A
and row-splits B over the layers, multiply() runs the layer SUMMA and the fiber reduce-scatter.
The local multiply / merge come from the CPU oracle (tests/dist_util.OracleBackend); the assembled
C must equal the single-block product bit for bit and, for R-MAT, the reference's digests.
"""
import numpy as np
import pytest

import helpers as H
from dist_util import OracleBackend, run_world
from test_dist_cpu import _h, _inputs


def _worker(rank, world, spec, sr_name, c, g, isBT):
    from combblas_amd import spgemm3d as s3
    from combblas_amd.semirings import ALL
    from combblas_amd.spparmat import SpParMat, _gather, block_range

    be = OracleBackend()
    dA, dB = _inputs(spec)
    SR = ALL[sr_name]
    CMG = s3.CCGrid(c, g)
    vdt = be.value_dtype(be.from_host(_h(dA)))
    A = SpParMat.distribute(_h(dA), CMG.layerGrid, be).seq if CMG.layer_grid == 0 else None
    B = SpParMat.distribute(_h(dB), CMG.layerGrid, be).seq if CMG.layer_grid == 0 else None
    splitA = s3.SplitMat(CMG, A, be, rowsplit=False, vdtype=vdt)
    splitB = s3.SplitMat(CMG, B, be, rowsplit=True, vdtype=vdt)
    if isBT:
        splitB = s3._transpose(be, splitB)  # mpipspgemm.cpp "outer": splitB.Transpose()
    C = s3.multiply(splitA, splitB, CMG, isBT, not isBT, be, SR)
    r0 = block_range(dA.m, g, CMG.RankInCol)[0]
    c0, c1 = block_range(dB.n, g, CMG.RankInRow)
    off = c0 + CMG.layer_grid * ((c1 - c0) // c)
    assert be.dims(C)[0] == block_range(dA.m, g, CMG.RankInCol)[1] - r0
    G = _gather(be, C, r0, off, dA.m, dB.n)
    if rank == 0:
        return (G.m, G.n, G.jc, G.cp, G.ir, G.num, sorted(s3.timers))
    return None


def _check(res, spec, sr_tag, golden=None):
    m, n, jc, cp, ir, num, timers = res
    assert "comm_bcast" in timers and "comp_reduce_layer" in timers
    got = H.Dcsc(m, n, jc, cp, ir, num)
    dA, dB = _inputs(spec)
    exp = H.Oracle().spgemm(dA, dB, H.SR_OF_TAG.get(sr_tag, sr_tag), "hybrid")
    H.assert_dcsc_equal(got, exp, msg=f"{spec}")
    if golden is not None:
        vs, dg = H.digest(got)
        assert (got.nnz, got.nzc) == (golden["nnz"], golden["nzc"])
        assert vs == golden["sum"] and dg == int(golden["digest"])


def test_multiply_2x2x2_rmat_vs_reference(golden):
    spec = ("rmat", 10, "pt_i64")
    res = run_world(_worker, 8, spec, "PlusTimesSRing", 2, 2, False)
    _check(res, spec, "pt_i64", golden["digests"]["rmat10_pt_i64"])


@pytest.mark.parametrize("isBT", [False, True])
def test_multiply_1x1x2_uneven(isBT):
    # 13 columns over 2 layers (chunks 6 / 7) and odd inner / row sizes
    spec = ("rand", 31, 27, 13, 0.2, 5, np.float64)
    res = run_world(_worker, 2, spec, "PlusTimesSRing", 2, 1, isBT)
    _check(res, spec, "plus_times")


def test_multiply_2x2x1_single_layer():
    # c = 1: SplitMat is the identity and ParallelReduce_Alltoall_threaded returns its input
    spec = ("rand", 29, 23, 19, 0.2, 9, np.int64)
    res = run_world(_worker, 4, spec, "SelectMaxSRing", 1, 2, False)
    _check(res, spec, "select_max")


def _grid_error_worker(rank, world):
    from combblas_amd import spgemm3d as s3
    from combblas_amd._lib import CombBLASHipError

    try:
        s3.CCGrid(2, 2)
    except CombBLASHipError as e:
        return e.code
    return 0


def test_ccgrid_size_mismatch_rejected():
    assert run_world(_grid_error_worker, 2) == 3003
