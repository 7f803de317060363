#!/usr/bin/env python3
"""bench_galerkin.py -- BASELINE.json config C3: the Galerkin triple product Rᵀ(A R) of
ReleaseTests/GalerkinNew.cpp:100-106 on the 27-point Poisson operator of a 256³ grid with trilinear
full-weighting prolongation onto 128³, on one MI355X. (The config names a 2×2
grid on 4 GPUs; this line is the same product on one GPU -- the 2×2 path is bench.py's SUMMA.)

One step = AT = LocalHybridSpGEMM(A, R) and SAT = LocalHybridSpGEMM(S, AT) with S = Rᵀ (built on
the device before the timed region, as GalerkinNew forms S before its products), PlusTimes<double>.
Every value is dyadic, so every sum is exact in f64 and the result is bit-identical under any
summation order.

Check: the value sum of SAT against its closed form (R1)ᵀ A (R1) computed on the host, and, unless
--no-oracle, the whole SAT against the CPU oracle's product (tests-only restatement of the
reference's hybrid kernel, threads = host cores).

roofline: the task-kernel class with the most HIP-event time over the timed steps, its algorithmic
bytes (12 B per B entry, product and output, + 16 B per task) / its duration.
CPU baseline ("reference"): GalerkinNew.cpp's own two PSpGEMM calls (oracle/_ref/ref_harness
galerkin, built from the reference sources) on a column sample of R (every --cpu-stride-th coarse
column: SAT(:, J) = Rᵀ(A R(:, J)) exactly), one warm-up and the median of 5, 1 rank x host cores.
    python bench_galerkin.py [--nx 256] [--steps 3] [--warmup 1] [--cpu-stride 4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def log(msg):
    print(f"[bench_galerkin] {msg}", file=sys.stderr, flush=True)


def closed_form_sum(A, R):
    """sum of Rᵀ A R = (R 1)ᵀ A (R 1), exact for these dyadic operators"""
    s = np.bincount(R.ir, weights=R.num, minlength=R.m)
    cols = np.repeat(A.jc, np.diff(A.cp))
    t = np.bincount(A.ir, weights=A.num * s[cols], minlength=A.m)
    return float(np.dot(s, t))


def reference_baseline(A, R, stride, reps=5):
    """GalerkinNew.cpp:99-106 (S = R', AT = PSpGEMM(A, R_s), SAT = PSpGEMM(S, AT)) by the reference
    itself on R's columns c % stride == 0, 1 rank x host cores; None when oracle/_ref is absent"""
    import subprocess
    import tempfile

    ref = os.path.join(HERE, "oracle", "_ref", "ref_harness")
    if not os.path.exists(ref):
        return None
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import helpers as H

    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        fa, fr = os.path.join(td, "A.cbm"), os.path.join(td, "R.cbm")
        H.write_cbm(fa, H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))
        H.write_cbm(fr, H.Dcsc(R.m, R.n, R.jc, R.cp, R.ir, R.num))
        env = dict(os.environ, OMP_NUM_THREADS=str(cores), LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:/opt/conda/lib")
        r = subprocess.run([ref, "galerkin", fa, fr, str(stride), str(reps)], env=env, cwd="/tmp",
                           capture_output=True, text=True, timeout=900)
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not line:
        log(f"reference baseline failed rc={r.returncode}: {r.stderr[-300:]}")
        return None
    d = json.loads(line[-1])
    return {"value": round(d["gflops"], 6), "unit": "GFLOP/s", "cores": d["threads"], "kind": "reference",
            "sample": f"GalerkinNew.cpp's PSpGEMM(A, R_s) and PSpGEMM(R', A R_s) (oracle/_ref built from the "
                      f"reference sources, 1 rank x {d['threads']} threads) on R's {d['cols']} columns c % {stride} == 0 "
                      f"({d['flops']} multiplies): median of {d['reps']} after 1 warm-up = {d['median_s']:.3f} s"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--nx", type=int, default=256)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--no-oracle", action="store_true")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-stride", type=int, default=4, help="R column sample of the reference CPU baseline")
    args = p.parse_args()
    import torch

    import combblas_amd as cb
    from combblas_amd.apps import Transpose
    from combblas_amd.galerkin import poisson27_csc, prolongation_csc

    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    A = poisson27_csc(args.nx)
    R = prolongation_csc(args.nx)
    log(f"operators: A {A.m}x{A.n} nnz {A.nnz}, R {R.m}x{R.n} nnz {R.nnz} ({time.perf_counter() - t0:.1f} s)")
    expect_sum = closed_form_sum(A, R)
    ctx = cb.Context(0)
    dA, dR = cb.SpDCCols.from_host(ctx, A), cb.SpDCCols.from_host(ctx, R)
    dS = Transpose(dR)
    f1 = cb.estimateFLOPandNNZ(dA, dR)[0]
    SR = cb.PlusTimesSRing

    def step():
        AT = cb.LocalHybridSpGEMM(SR, dA, dR)
        SAT = cb.LocalHybridSpGEMM(SR, dS, AT)
        return AT, SAT

    AT, SAT = step()
    f2 = cb.estimateFLOPandNNZ(dS, AT)[0]
    nnz_at = AT.nnz
    AT.free()
    SAT.free()
    for _ in range(max(args.warmup - 1, 0)):
        for X in step():
            X.free()
    ctx.synchronize()
    torch.cuda.synchronize()
    ctx.reset_kernel_stats()
    ctx.enable_timing(True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        AT, SAT = step()
        AT.free()
        if i + 1 < args.steps:
            SAT.free()
    ctx.synchronize()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    ctx.enable_timing(False)
    from bench import kernel_roofline

    roofline = kernel_roofline(ctx.kernel_stats())
    flops = int(f1) + int(f2)
    vsum, dig = SAT.checksum()
    log(f"{args.steps} step(s): {dt * 1e3:.1f} ms/step, nnz(AT) {nnz_at}, nnz(SAT) {SAT.nnz}")
    check = {"nnzAT": int(nnz_at), "nnzSAT": int(SAT.nnz), "value_sum": vsum, "expected_value_sum": expect_sum,
             "digest": str(dig)}
    oracle_tc = None
    if not args.no_oracle:
        sys.path.insert(0, os.path.join(HERE, "tests"))
        import helpers as H

        O = H.Oracle()
        cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
        hA, hR = H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num), H.Dcsc(R.m, R.n, R.jc, R.cp, R.ir, R.num)
        S = dS.to_host()
        hS = H.Dcsc(S.m, S.n, S.jc, S.cp, S.ir, S.num)
        del A, R
        t1 = time.perf_counter()
        hAT = O.spgemm(hA, hR, "plus_times", "hybrid", threads=cores)
        hSAT = O.spgemm(hS, hAT, "plus_times", "hybrid", threads=cores)
        tc = time.perf_counter() - t1
        osum, odig = H.digest(hSAT)
        check.update(oracle_nnzSAT=int(hSAT.nnz), oracle_digest=str(odig))
        oracle_tc = {"s": round(tc, 3), "gflops": round(2.0 * flops / tc / 1e9, 6), "cores": cores,
                     "note": "CPU oracle restatement (port) on the whole product"}
        del hA, hR, hS, hAT, hSAT
    check["ok"] = bool(vsum == expect_sum and (oracle_tc is None or (check["oracle_digest"] == check["digest"]
                                                                      and check["oracle_nnzSAT"] == check["nnzSAT"])))
    base = None
    if not args.no_cpu_baseline:
        log("reference CPU baseline (GalerkinNew's products on a column sample)")
        base = reference_baseline(poisson27_csc(args.nx), prolongation_csc(args.nx), args.cpu_stride)
    out = {"metric": "Galerkin R^T A R (C3): semiring GFLOP/s of the two products",
           "value": round(2.0 * flops / dt / 1e9, 3), "unit": "GFLOP/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "f64",
           "data": f"synthetic: 27-point Poisson on {args.nx}^3, trilinear prolongation onto {args.nx // 2}^3 (dyadic)",
           "config": {"workload": f"galerkin{args.nx}_RtAR_PlusTimes_f64", "nx": args.nx, "flops": flops,
                      "flops_AR": int(f1), "flops_RtAR": int(f2), "parallelism": "1 GPU (config C3 names 2x2)"},
           "roofline": roofline, "cpu_baseline": base, "oracle_cpu": oracle_tc, "check": check}
    print(json.dumps(out), flush=True)
    SAT.free()
    ctx.close()


if __name__ == "__main__":
    main()
