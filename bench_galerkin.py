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
reference's hybrid kernel, threads = host cores), which also gives the CPU baseline ("port").
    python bench_galerkin.py [--nx 256] [--steps 3] [--warmup 1]
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--nx", type=int, default=256)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--no-oracle", action="store_true")
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
    t0 = time.perf_counter()
    for i in range(args.steps):
        AT, SAT = step()
        AT.free()
        if i + 1 < args.steps:
            SAT.free()
    ctx.synchronize()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    flops = int(f1) + int(f2)
    vsum, dig = SAT.checksum()
    log(f"{args.steps} step(s): {dt * 1e3:.1f} ms/step, nnz(AT) {nnz_at}, nnz(SAT) {SAT.nnz}")
    check = {"nnzAT": int(nnz_at), "nnzSAT": int(SAT.nnz), "value_sum": vsum, "expected_value_sum": expect_sum,
             "digest": str(dig)}
    base = None
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
        base = {"value": round(2.0 * flops / tc / 1e9, 6), "unit": "GFLOP/s", "cores": cores, "kind": "port",
                "sample": f"the whole product (both multiplies) by the CPU oracle (restatement of the reference's "
                          f"LocalHybridSpGEMM, OpenMP over {cores} threads), one run: {tc:.2f} s"}
    check["ok"] = bool(vsum == expect_sum and (base is None or (check["oracle_digest"] == check["digest"]
                                                                 and check["oracle_nnzSAT"] == check["nnzSAT"])))
    out = {"metric": "Galerkin R^T A R (C3): semiring GFLOP/s of the two products",
           "value": round(2.0 * flops / dt / 1e9, 3), "unit": "GFLOP/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "f64",
           "data": f"synthetic: 27-point Poisson on {args.nx}^3, trilinear prolongation onto {args.nx // 2}^3 (dyadic)",
           "config": {"workload": f"galerkin{args.nx}_RtAR_PlusTimes_f64", "nx": args.nx, "flops": flops,
                      "flops_AR": int(f1), "flops_RtAR": int(f2), "parallelism": "1 GPU (config C3 names 2x2)"},
           "cpu_baseline": base, "check": check}
    print(json.dumps(out), flush=True)
    SAT.free()
    ctx.close()


if __name__ == "__main__":
    main()
