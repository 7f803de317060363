"""GPU: the reference's phased and 3D drivers on device-resident blocks (include/combblas_hip/ParFriendsDev.h).

oracle/_ref/devpath3d_harness (g++, the reference's headers) builds SpParMat / SpParMat3D operands
over SpDCColsDev and calls the reference's own driver names -- MemEfficientSpGEMM with
MCLPruneRecoverySelect (ParFriends.h:449-730, :185-353), Mult_AnXBn_SUMMA3D (:2918-3208),
MemEfficientSpGEMM3D (:3214-3705) -- which resolve to the device overloads (device SUMMA, fiber
reduce-scatter as device pieces over grouped send/recv, device MCL prune with processor-column
reductions), then compares every rank's block with the STOCK drivers on host blocks. Grids:
1 rank (RCCL transport), 2x2 (4 ranks), 1x1x2 (2 ranks) and 2x2x2 (8 ranks), the multi-rank runs
sharing the one GPU over the host-staged MPI transport (RCCL refuses two ranks on one device)."""
import os
import subprocess

import pytest

import helpers as H

pytestmark = pytest.mark.gpu

HARNESS = os.path.join(H.REPO, "oracle", "_ref", "devpath3d_harness")
ENV = dict(os.environ, LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:/opt/conda/lib", OMP_NUM_THREADS="1")


def _run(np_, scale, layers, expect, transport, **extra_env):
    assert os.path.exists(HARNESS), "oracle/_ref/devpath3d_harness missing: run __graft_entry__.build() with the reference"
    cmd = [HARNESS, str(scale), str(layers)]
    env = dict(ENV, **extra_env)
    if np_ > 1:
        cmd = ["/opt/conda/bin/mpirun", "-np", str(np_)] + cmd
        env["COMBBLAS_HIP_COMM"] = "mpi"
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=170, cwd="/tmp")
    lines = [l for l in r.stdout.splitlines() if l.startswith("DEVPATH3D")]
    assert r.returncode == 0 and len(lines) == expect, r.stdout + r.stderr
    assert all(" OK " in l and f"ranks={np_}" in l and f"transport={transport}" in l for l in lines), r.stdout


def test_devpath3d_one_rank_rccl():
    _run(1, 11, 1, 6, "rccl")  # 3 MemEfficientSpGEMM + SUMMA3D + 2 MemEfficientSpGEMM3D


def test_devpath3d_2x2_shared_gpu():
    _run(4, 11, 0, 3, "mpi")


def test_devpath3d_1x1x2_shared_gpu():
    _run(2, 11, 2, 3, "mpi")


def test_devpath3d_2x2x2_shared_gpu():
    _run(8, 10, 2, 3, "mpi")


def test_devpath3d_2x2_per_stage_plans():
    """the reference's per-stage form of the phased drivers (one plan per SUMMA stage pair, stage
    partials merged per phase; COMBBLAS_HIP_STAGE_PLANS=per-stage) against the stock drivers; the
    tests above run the default concatenated strips"""
    _run(4, 11, 0, 3, "mpi", COMBBLAS_HIP_STAGE_PLANS="per-stage")


def test_devpath3d_2x2x2_per_stage_plans():
    _run(8, 10, 2, 3, "mpi", COMBBLAS_HIP_STAGE_PLANS="per-stage")
