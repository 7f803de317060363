"""GPU: the reference's UNCHANGED phased and 3D drivers on the gfx950 kernels.

oracle/_ref/dropin3d_harness (tests/dropin/dropin3d_harness.cpp, g++ with the reference's headers)
instantiates MemEfficientSpGEMM (ParFriends.h:449-730, hash and heap kernels, with
MCLPruneRecoverySelect), Mult_AnXBn_SUMMA3D (:2918-3208) and MemEfficientSpGEMM3D (:3214-3705)
for PlusTimesSRing<double,double>, whose LocalSpGEMMHash / LocalSpGEMM / MultiwayMerge /
MultiwayMergeHash COMBBLAS_HIP_INSTANTIATE routes to the device, and compares every rank's block
of C with the same driver on the stock OpenMP kernels. Ranks share the one GPU of the test box
(mpirun, one HIP context per rank): 1 rank (2D 1x1), 2 (3D 1x1x2), 4 (2D 2x2 and 3D 1x1x4) and
8 (3D 2x2x2)."""
import os
import subprocess

import pytest

import helpers as H

pytestmark = pytest.mark.gpu

HARNESS = os.path.join(H.REPO, "oracle", "_ref", "dropin3d_harness")
ENV = dict(os.environ, LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:/opt/conda/lib", OMP_NUM_THREADS="1")


@pytest.mark.parametrize("ranks,layers,ncases", [(1, 0, 4), (2, 2, 3), (4, 4, 7), (8, 2, 3)])
def test_reference_phased_and_3d_drivers(ranks, layers, ncases):
    assert os.path.exists(HARNESS), "oracle/_ref/dropin3d_harness missing: run __graft_entry__.build() with the reference"
    r = subprocess.run(["/opt/conda/bin/mpirun", "-np", str(ranks), HARNESS, "11", str(layers)], env=ENV,
                       capture_output=True, text=True, timeout=170, cwd="/tmp")
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    lines = [l for l in out.splitlines() if l.startswith("DROPIN3D")]
    assert len(lines) == ncases and all(" OK " in l and f"ranks={ranks}" in l for l in lines), out
