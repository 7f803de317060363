"""CPU: bench.py's N-GPU launcher (the C++ host path) without a GPU. torch.distributed.run starts two
bench.py ranks on gloo; rank 0 runs a stand-in for `mpirun -np 2 cxx/_build/bench_summa` (a script
that records its argv and environment and prints bench_summa's JSON line) and the other rank waits
on the group. Checked: one JSON line from rank 0 with the stand-in's numbers turned into the
metric (value = 2 * flops / step time, flops and the closed-form sum from the same R-MAT), the
check against the reference's nnz, the launcher's variables removed from the child's environment,
and a failing child reported (driver cpp: exit 1; under auto the python drivers, which need the
GPU, would run instead)."""
import json
import os
import stat
import subprocess
import sys

import pytest

import helpers as H
from dist_util import _free_port

STUB = r'''#!/bin/bash
# stand-in for mpirun: $1 = -np, $2 = N, $3 = binary, then scale steps warmup phases
env > "{envfile}"
echo "$@" > "{argfile}"
[ "{fail}" = 1 ] && exit 3
echo '{{"ms_per_step": 2.0, "steps": 1, "warmup": 0, "ranks": '$2', "grid": "3D SUMMA 1x1x2", "driver": "stub", "phases": 1, "nnzC": {nnz}, "value_sum": {vsum}, "setup_s": 0.1, "transport": "rccl", "kernel_stats_rank0": {{"num_large": [1.0, 2, 4000000000.0]}}}}'
'''


def _closed_form(scale):
    import numpy as np

    import combblas_amd as cb

    sys.path.insert(0, H.REPO)
    import bench

    A = cb.rmat(scale, 16, dtype=np.float64)
    return bench.host_flops(A), bench.product_value_sum(A)


def _run(tmp_path, fail, driver, port):
    flops, vsum = _closed_form(10)
    envfile, argfile = tmp_path / "env.txt", tmp_path / "args.txt"
    stub = tmp_path / "mpirun"
    stub.write_text(STUB.format(envfile=envfile, argfile=argfile, fail=1 if fail else 0, nnz=86246, vsum=float(vsum)))
    stub.chmod(stub.stat().st_mode | stat.S_IEXEC)
    env = dict(os.environ, CBH_MPIRUN=str(stub), CBH_BENCH_SUMMA=str(stub), MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", f"--master-port={port}", os.path.join(H.REPO, "bench.py"), "--gpus", "2", "--steps", "1",
           "--warmup", "0", "--scale", "10", "--driver", driver]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=str(tmp_path), env=env)
    return r, flops, envfile, argfile


def test_launcher_runs_the_cpp_driver(tmp_path):
    r, flops, envfile, argfile = _run(tmp_path, False, "cpp", _free_port())
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["ms_per_step"] == 2.0
    assert abs(d["value"] - 2.0 * flops / 2e-3 / 1e9) < 1e-3 * d["value"]
    assert d["check"]["ok"] and d["check"]["nnzC"] == 86246
    assert d["config"]["host_path"].startswith("C++: stub")
    assert d["roofline"]["kernel"].startswith("cbh::task_kernel")
    args = argfile.read_text().split()
    assert args[:2] == ["-np", "2"] and args[3:] == ["10", "1", "0", "0"]
    child = dict(l.split("=", 1) for l in envfile.read_text().splitlines() if "=" in l)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT"):
        assert k not in child, k  # mpirun's ranks must not see the torch launcher's rendezvous


def test_launcher_reports_a_failed_cpp_run(tmp_path):
    r, _, _, _ = _run(tmp_path, True, "cpp", _free_port())
    assert r.returncode != 0
    assert "C++ driver failed" in r.stderr
