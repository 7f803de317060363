#!/usr/bin/env python3
"""bench_c1.py -- BASELINE.json config C1: R-MAT scale-16 ef-16 A*A with PlusTimes<double> on one
rank through the reference's own MultTest-style plumbing (ReleaseTests/MultTest.cpp:161-181:
`C = Mult_AnXBn_Synch<PTDOUBLEDOUBLE, double, PSpMat<double>::DCCols>(A, B)`), i.e. SpParMat over
the stock host SpDCCols, with COMBBLAS_HIP_INSTANTIATE routing the driver to the device
(include/combblas_hip/HipSpGEMM.h mult_synch_host: blocks uploaded through pinned chunks, the
product and the stage merge on the MI355X, C downloaded straight into the result's Dcsc arrays).

The harness (oracle/_ref/dropin_harness, built by `make -C oracle ref` from the reference's headers
with g++) times the first call (HIP context creation and code-object load included) and the median
of --reps warm calls, split into the adaptor's stages (upload / kernel / merge / download), and the
reference's stock OpenMP path on the same operands (first call, median of --reps) as the CPU
baseline ("reference": the reference's own LocalHybridSpGEMM + MultiwayMerge + SpDCCols build).
Both results must be identical (structure, row order, values).

value = 2 * flops / warm call time: the whole driver call on host-resident operands, so the
PCIe transfers are inside it (this line is the drop-in's cost as a user sees it; the device-resident
rate of the same product is the `kernel` stage).
    python bench_c1.py [--scale 16] [--reps 5] [--threads N]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=16)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--threads", type=int, default=0, help="OpenMP threads (0 = the host cores this process may use)")
    a = p.parse_args()
    harness = os.path.join(HERE, "oracle", "_ref", "dropin_harness")
    if not os.path.exists(harness):
        sys.exit("oracle/_ref/dropin_harness is missing: run __graft_entry__.build() where the reference exists")
    threads = a.threads or int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    env = dict(os.environ, OMP_NUM_THREADS=str(threads),
               LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:/opt/conda/lib")
    r = subprocess.run([harness, "bench", str(a.scale), str(a.reps)], env=env, cwd="/tmp", capture_output=True,
                       text=True, timeout=900)
    line = [l for l in r.stdout.splitlines() if l.startswith("BENCHC1 ")]
    if r.returncode != 0 or not line:
        sys.exit(f"harness failed (rc {r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
    d = json.loads(line[-1][len("BENCHC1 "):])
    gf = lambda s: round(2 * d["flops"] / s / 1e9, 4) if s > 0 else None  # noqa: E731
    out = {
        "metric": "semiring GFLOP/s of PSpGEMM<PlusTimes<double>> (Mult_AnXBn_Synch over host SpDCCols, drop-in)",
        "value": gf(d["warm_s"]), "unit": "GFLOP/s", "n_gpus": 1, "steps": d["reps"], "warmup": 1,
        "ms_per_step": round(d["warm_s"] * 1e3, 3), "higher_is_better": True, "dtype": "f64",
        "data": "synthetic: packed Graph500 R-MAT (reference generator, seed 0xDECAFBAD)",
        "config": {"workload": f"C1 rmat{a.scale}_ef16_AxA_PlusTimes_f64, 1 rank, MultTest plumbing",
                   "nnzA": d["nnzA"], "nnzC": d["nnzC"], "flops": d["flops"]},
        "first_call_ms": round(d["first_s"] * 1e3, 3),
        "stages_ms": {k: round(d[k + "_s"] * 1e3, 3) for k in ("upload", "kernel", "merge", "download")},
        "kernel_gflops": gf(d["kernel_s"]),
        "check": {"identical_to_stock_path": d["match"]},
        "cpu_baseline": {"value": gf(d["cpu_s"]), "unit": "GFLOP/s", "cores": int(d["cpu_threads"]) or threads,
                         "kind": "reference",
                         "sample": f"the same call on the reference's stock OpenMP path (value-identical unspecialized "
                                   f"semiring), 1 rank x {threads} threads, median of {d['reps']} after one untimed "
                                   f"first call ({d['cpu_first_s'] * 1e3:.1f} ms) = {d['cpu_s'] * 1e3:.1f} ms"},
        "vs_stock": round(d["cpu_s"] / d["warm_s"], 3) if d["warm_s"] > 0 else None,
    }
    print(json.dumps(out), flush=True)
    if not d["match"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
