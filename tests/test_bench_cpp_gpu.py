"""GPU: bench.py's N-GPU line through the C++ host path (cxx/_build/bench_summa under mpirun,
started by rank 0 of a torch.distributed.run job whose ranks wait on a gloo barrier).

The ranks share the one GPU, so the exchanges go through the host-staged MPI transport
(--share-gpu sets COMBBLAS_HIP_COMM=mpi). Grids: 2x2 (4 ranks: PSpGEMM -> device Mult_AnXBn_Synch
with one phase, MemEfficientSpGEMM's StagePlans loop with 3) and 1x1x2 (2 ranks: layer SUMMA +
fiber reduce-scatter, 1 and 2 phases) and 2x2x2 (8 ranks: the driver's N = 8 command -- input on a
2x4 grid redistributed by SpParMat3D, layer SUMMA on 2x2 grids, fiber reduce-scatter -- with 1 and
2 phases). The check: nnz(C) equals the reference's count for the scale, sum(C) the closed form
sum_k colsum_k(A) * rowsum_k(A) (exact: integer multiplicities), and the order-sensitive digest of
the whole product, assembled from the ranks' pieces at their global positions, the reference's own
(tests/golden/scale14.json, make_golden_s22.py 14)."""
import json
import os
import subprocess
import sys

import pytest

import helpers as H
from dist_util import _free_port

pytestmark = pytest.mark.gpu

BENCH = os.path.join(H.REPO, "cxx", "_build", "bench_summa")


@pytest.mark.parametrize("ranks,phases,host", [(4, 0, "Mult_AnXBn_Synch"), (4, 3, "MemEfficientSpGEMM phase loop"),
                                               (2, 0, "MemEfficientSpGEMM3D"), (2, 2, "MemEfficientSpGEMM3D"),
                                               (8, 0, "MemEfficientSpGEMM3D"), (8, 2, "MemEfficientSpGEMM3D")])
def test_bench_cpp_driver(ranks, phases, host):
    assert os.path.exists(BENCH), "cxx/_build/bench_summa missing: run __graft_entry__.build() with the reference"
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.join(H.REPO, "bench.py"),
           "--gpus", str(ranks), "--steps", "1", "--warmup", "1", "--scale", "14", "--share-gpu",
           "--dist-backend", "gloo", "--driver", "cpp", "--phases", str(phases)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=200 if ranks == 8 else 170, cwd="/tmp")
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(lines) == 1, r.stdout[-3000:] + r.stderr[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == ranks and d["check"]["ok"], d
    assert d["check"]["nnzC"] == 6471508
    gold = json.load(open(os.path.join(H.REPO, "tests", "golden", "scale14.json")))["pt_f64"]["total"]["digest"]
    assert d["check"]["reference_digest"] == gold and d["check"]["digest"] == gold, d["check"]
    assert ("3x3" not in d["config"]["parallelism"]) and (ranks != 8 or "2x2x2" in d["config"]["parallelism"]), d
    assert host in d["config"]["host_path"], d["config"]
    assert phases == 0 or d["config"]["phases"] == phases
    assert d["value"] > 0 and d["roofline"] is not None
