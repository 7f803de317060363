"""GPU: device-resident SUMMA behind the reference's own PSpGEMM (include/combblas_hip/SpParMatDev.h).

oracle/_ref/devpath_harness (g++, the reference's headers) builds SpParMat<IT, NT, SpDCColsDev>
operands, calls the UNCHANGED PSpGEMM<SR> (SpParMat.h:454-467) -- which resolves to the
device-resident Mult_AnXBn_Synch overload: RCCL (ncclBroadcast) stage broadcasts, device multiply
and merge, no host copy of any block -- and compares every rank's block of C with the stock
OpenMP Mult_AnXBn_Synch. 1 rank over RCCL; 4 ranks (2x2 grid) sharing the one GPU with the
host-staged MPI transport (RCCL refuses two ranks on one device)."""
import os
import subprocess

import pytest

import helpers as H

pytestmark = pytest.mark.gpu

HARNESS = os.path.join(H.REPO, "oracle", "_ref", "devpath_harness")
ENV = dict(os.environ, LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:/opt/conda/lib")


def _check(out, ranks):
    lines = [l for l in out.splitlines() if l.startswith("DEVPATH")]
    # PSpGEMM (Mult_AnXBn_Synch), Mult_AnXBn_Overlap and Mult_AnXBn_DoubleBuff, two semirings each
    assert len(lines) == 6 and all(" OK " in l and f"ranks={ranks}" in l for l in lines), out


@pytest.mark.parametrize("scale", [10, 14])
def test_devpath_one_rank_rccl(scale):
    assert os.path.exists(HARNESS), "oracle/_ref/devpath_harness missing: run __graft_entry__.build() with the reference"
    r = subprocess.run([HARNESS, str(scale), "1"], env=dict(ENV, OMP_NUM_THREADS="8"), capture_output=True, text=True,
                       timeout=120, cwd="/tmp")
    assert r.returncode == 0, r.stdout + r.stderr
    _check(r.stdout, 1)
    assert "transport=rccl" in r.stdout


def test_devpath_2x2_grid_shared_gpu():
    r = subprocess.run(["/opt/conda/bin/mpirun", "-np", "4", HARNESS, "12", "1"],
                       env=dict(ENV, OMP_NUM_THREADS="2", COMBBLAS_HIP_COMM="mpi"), capture_output=True, text=True,
                       timeout=150, cwd="/tmp")
    assert r.returncode == 0, r.stdout + r.stderr
    _check(r.stdout, 4)
