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
# the ranks share the box's one GPU: an explicit rehearsal (HipSpGEMM.h context() refuses more local
# ranks than devices otherwise)
ENV = dict(os.environ, LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:/opt/conda/lib", OMP_NUM_THREADS="1",
           COMBBLAS_HIP_SHARE_DEVICE="1")


@pytest.mark.parametrize("ranks,layers,ncases", [(1, 0, 4), (2, 2, 3), (4, 4, 7), (8, 2, 3)])
def test_reference_phased_and_3d_drivers(ranks, layers, ncases):
    assert os.path.exists(HARNESS), "oracle/_ref/dropin3d_harness missing: run __graft_entry__.build() with the reference"
    r = subprocess.run(["/opt/conda/bin/mpirun", "-np", str(ranks), HARNESS, "11", str(layers)], env=ENV,
                       capture_output=True, text=True, timeout=170, cwd="/tmp")
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    lines = [l for l in out.splitlines() if l.startswith("DROPIN3D")]
    assert len(lines) == ncases and all(" OK " in l and f"ranks={ranks}" in l for l in lines), out


DEV3DS = os.path.join(H.REPO, "oracle", "_ref", "dropin3ds_harness")
STOCK3DS = os.path.join(H.REPO, "oracle", "_ref", "stock3ds_harness")


def _blocks(binary, ranks, layers, scale, mode=None, env=None):
    cmd = ["/opt/conda/bin/mpirun", "-np", str(ranks), binary, str(scale), str(layers)] + ([mode] if mode else [])
    r = subprocess.run(cmd, env=env or ENV, capture_output=True, text=True, timeout=170, cwd="/tmp")
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    blocks = sorted(l.split()[1:] for l in out.splitlines() if l.startswith("BLOCK3DS "))
    total = [l for l in out.splitlines() if l.startswith("TOTAL3DS ")]
    assert len(blocks) == ranks and len(total) == 1, out
    return blocks, total[0]


@pytest.mark.parametrize("ranks,layers", [(2, 2), (8, 2), (4, 1)])
def test_reference_standalone_3d_layer(ranks, layers):
    """The reference's standalone 3DSpGEMM/ layer (CCGrid -> SplitMat -> multiply = SUMMALayer +
    ReduceAll_threaded / ParallelReduce_Alltoall_threaded, Multiplier.h:10-61) with its LocalSpGEMM
    and MultiwayMerge calls routed to the gfx950 kernels (COMBBLAS_HIP_INSTANTIATE) gives every rank
    the same block of C -- structure, order and values -- as the same driver on the stock kernels."""
    for b in (DEV3DS, STOCK3DS):
        assert os.path.exists(b), f"{b} missing: run __graft_entry__.build() with the reference"
    dev, tot_dev = _blocks(DEV3DS, ranks, layers, 11)
    stock, tot_stock = _blocks(STOCK3DS, ranks, layers, 11)
    assert dev == stock, (dev, stock)
    assert tot_dev.split()[1:3] == tot_stock.split()[1:3]
    print(f"DROPIN3DSTANDALONE {tot_dev.split()[1]} OK {tot_dev.split()[2]} ranks={ranks}")


DEVPATH3DS = os.path.join(H.REPO, "oracle", "_ref", "devpath3ds_harness")


@pytest.mark.parametrize("ranks,layers", [(1, 1), (2, 2), (8, 2)])
def test_device_resident_standalone_3d_layer(ranks, layers):
    """The device overloads of the standalone layer (include/combblas_hip/Dev3DSpGEMM.h: SUMMALayer,
    ReduceAll_threaded, ParallelReduce_Alltoall_threaded, multiply over SpDCColsDev) give every rank
    the stock layer's block of C. One rank runs RCCL; ranks sharing the GPU stage the broadcasts and
    the fiber exchange through host MPI (COMBBLAS_HIP_COMM=mpi: RCCL refuses two ranks per device)."""
    for b in (DEVPATH3DS, STOCK3DS):
        assert os.path.exists(b), f"{b} missing: run __graft_entry__.build() with the reference"
    env = dict(ENV, COMBBLAS_HIP_COMM="mpi") if ranks > 1 else ENV
    r = subprocess.run(["/opt/conda/bin/mpirun", "-np", str(ranks), DEVPATH3DS, "11", str(layers)], env=env,
                       capture_output=True, text=True, timeout=170, cwd="/tmp")
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    dev = sorted(l.split()[1:] for l in out.splitlines() if l.startswith("BLOCK3DS "))
    stock, tot_stock = _blocks(STOCK3DS, ranks, layers, 11)
    assert dev == stock, (dev, stock)
    print(f"DEVPATH3DSTANDALONE {tot_stock.split()[1]} OK {tot_stock.split()[2]} ranks={ranks}")


@pytest.mark.parametrize("ranks,layers", [(1, 1), (2, 2), (4, 1)])
def test_device_resident_outer_product_mode(ranks, layers):
    """mpipspgemm.cpp's outer-product case (:176-179): splitB transposed locally and
    multiply(splitA, splitB, CMG, isBT = true, threaded = false). The device SUMMALayer transposes
    every received B block back on the device (cbh_transpose) where the reference calls
    MultiplyReturnTuples(..., isBT): every rank's block of C equals the stock layer's in the same
    mode (which equals the column-threaded mode's)."""
    for b in (DEVPATH3DS, STOCK3DS):
        assert os.path.exists(b), f"{b} missing: run __graft_entry__.build() with the reference"
    env = dict(ENV, COMBBLAS_HIP_COMM="mpi") if ranks > 1 else ENV
    dev, _ = _blocks(DEVPATH3DS, ranks, layers, 11, "bt", env)
    stock_bt, tot = _blocks(STOCK3DS, ranks, layers, 11, "bt")
    stock, _ = _blocks(STOCK3DS, ranks, layers, 11)
    assert stock_bt == stock
    assert dev == stock_bt, (dev, stock_bt)
    print(f"DEVPATH3DSBT {tot.split()[1]} OK {tot.split()[2]} ranks={ranks}")
