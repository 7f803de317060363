#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: semiring GFLOP/s of R-MAT A^2 SpGEMM on MI355X, with the
HBM-roofline fraction of the dominant kernel and the reference's CPU time beside it.

Workload (N=1): config C2 = Graph500 R-MAT scale 22, edge factor 16, A*A with
PlusTimesSRing<double> (B is a separate copy of A, as Mult_AnXBn_Synch requires). One step = the
whole product: symbolic pass (estimateFLOP + exact nnz) and every numeric column phase; C
(24.8 G nonzeros, ~297 GB) exceeds HBM, so B's columns are processed in phases whose C blocks are
materialised in HBM one after another (MemEfficientSpGEMM's phase loop, ParFriends.h:449-730).
Inputs are resident in HBM before the timed region.

N>1 (launched by torch.distributed.run): the same fixed product is split into N column stripes
of B with equal flops; every rank holds A (generated locally, no data-path collective) and
computes its stripe -> "scaling": "strong". Timing: barrier + synchronize around exactly K steps,
max over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scale 22]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "semiring GFLOP/s for R-MAT A² SpGEMM at 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s (spec)
DOMINANT = "num_large"
DOMINANT_KERNEL = "cbh::tile_kernel<cbh::PlusTimesD<double>, 4096, 512, 512, 1>"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--scale", type=int, default=22)
    p.add_argument("--edgefactor", type=int, default=16)
    p.add_argument("--phase-budget-gb", type=float, default=0.0, help="0 = half of free HBM")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-cols-frac", type=float, default=1.0 / 64, help="column sample of the CPU baseline")
    p.add_argument("--no-verify", action="store_true")
    return p.parse_args()


def column_stripe(A, world, rank):
    """B's nonzero columns split into `world` contiguous stripes of equal flops."""
    if world == 1:
        return 0, A.nzc
    dense = np.zeros(A.n + 1, np.int64)
    dense[A.jc + 1] = np.diff(A.cp)
    lenA = dense[1:]
    flop = np.add.reduceat(lenA[A.ir].astype(np.int64), A.cp[:-1]) if A.nnz else np.zeros(0, np.int64)
    cum = np.concatenate([[0], np.cumsum(flop)])
    cuts = [int(np.searchsorted(cum, cum[-1] * r / world)) for r in range(world + 1)]
    cuts[0], cuts[-1] = 0, A.nzc
    return cuts[rank], cuts[rank + 1]


def slice_cols(A, i0, i1):
    import combblas_amd as cb

    s, e = A.cp[i0], A.cp[i1]
    return cb.HostDcsc(A.m, A.n, A.jc[i0:i1], A.cp[i0:i1 + 1] - s, A.ir[s:e], A.num[s:e])


def cpu_baseline(scale, ef, frac):
    """Reference Mult_AnXBn_Synch (MPI+OpenMP, 1 rank) on a bounded column sample of the same
    product, C = A * A(:, 0:n*frac), on this host's cores. Falls back to the oracle port."""
    n = 1 << scale
    c1 = max(1, int(n * frac))
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    ref = os.path.join(HERE, "oracle", "_ref", "ref_harness")
    sample = f"C = A*A(:,0:{c1}) of R-MAT scale {scale} ef {ef} (1/{round(1 / frac)} of B's columns), 1 run"
    if os.path.exists(ref):
        env = dict(os.environ, OMP_NUM_THREADS=str(cores))
        try:
            r = subprocess.run([ref, "slice", str(scale), str(ef), "0", str(c1), "1", "pt_f64"], env=env, cwd="/tmp",
                               capture_output=True, text=True, timeout=900)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")]
            if r.returncode == 0 and line:
                d = json.loads(line[-1])
                return {"value": round(d["gflops"], 6), "unit": "GFLOP/s", "cores": d["threads"], "kind": "reference",
                        "sample": sample + f": {d['flops']} flops in {d['median_s']:.3f} s (Mult_AnXBn_Synch, "
                                           "oracle/_ref built from the reference sources)"}
        except Exception as e:  # noqa: BLE001
            print(f"reference CPU baseline failed: {e}", file=sys.stderr)
    # port: the oracle restatement (tests-only code, used here only as the CPU baseline leg)
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import helpers as H
    import combblas_amd as cb

    A = cb.rmat(scale, ef, dtype=np.float64)
    d = H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num)
    B = d.col_slice(0, c1)
    O = H.Oracle()
    t0 = time.perf_counter()
    C = O.spgemm(d, B, "plus_times", "hybrid", threads=cores)
    dt = time.perf_counter() - t0
    flops = O.symbolic(d, B, threads=cores)[0]
    return {"value": round(2 * flops / dt / 1e9, 6), "unit": "GFLOP/s", "cores": cores, "kind": "port",
            "sample": sample + f": {flops} flops in {dt:.3f} s (oracle restatement), nnzC {C.nnz}"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import combblas_amd as cb

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    def barrier():
        if world > 1:
            dist.barrier()

    def allreduce(x, op):
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=op)
        return t.item()

    # ---------------------------------------------------------------- inputs (resident in HBM)
    A = cb.rmat(args.scale, args.edgefactor, dtype=np.float64)
    i0, i1 = column_stripe(A, world, rank)
    Bs = slice_cols(A, i0, i1)
    ctx = cb.Context(local, torch_allocator=False)
    if args.phase_budget_gb > 0:
        ctx.set_phase_budget(int(args.phase_budget_gb * 2**30))
    dA = cb.SpDCCols.from_host(ctx, A)
    dB = cb.SpDCCols.from_host(ctx, Bs)  # separate copy (aliasing is rejected, ParFriends.h:172)
    nnzA = A.nnz
    del A, Bs
    SR = cb.PlusTimesSRing

    for _ in range(args.warmup):
        st = cb.PhasedSpGEMM(SR, dA, dB)
    ctx.synchronize()
    ctx.enable_timing(True)
    ctx.reset_kernel_stats()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st = cb.PhasedSpGEMM(SR, dA, dB)
    ctx.synchronize()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    ctx.enable_timing(False)
    ks = ctx.kernel_stats()

    my_s = (t1 - t0) / max(args.steps, 1)
    step_s = allreduce(my_s, dist.ReduceOp.MAX if world > 1 else None)
    flops = allreduce(float(st["flops"]), dist.ReduceOp.SUM if world > 1 else None)
    nnzC = allreduce(float(st["nnz"]), dist.ReduceOp.SUM if world > 1 else None)
    value = 2.0 * flops / step_s / 1e9

    k = ks[DOMINANT]
    achieved = (k["alg_bytes"] / (k["ms"] / 1e3) / 1e9) if k["ms"] > 0 else 0.0
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": DOMINANT_KERNEL, "launches": k["launches"],
                "avg_launch_ms": round(k["ms"] / max(k["launches"], 1), 4),
                "alg_bytes_per_launch": round(k["alg_bytes"] / max(k["launches"], 1))}
    pmc = os.path.join(HERE, "profiles", "pmc_num_large.json")
    if os.path.exists(pmc):
        try:
            roofline["traffic"] = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:  # noqa: BLE001
            pass

    check = None
    if not args.no_verify:
        sv = cb.PhasedSpGEMM(SR, dA, dB, checksum=True)
        nnz_all = allreduce(float(sv["nnz"]), dist.ReduceOp.SUM if world > 1 else None)
        vsum = allreduce(sv["value_sum"], dist.ReduceOp.SUM if world > 1 else None)
        known = {22: 24766243778, 20: 3284757756, 18: 425342972, 16: 53638834, 14: 6471508}.get(args.scale)
        check = {"nnzC": int(nnz_all), "value_sum": vsum, "expected_nnzC": known,
                 "ok": (known is None or int(nnz_all) == known)}

    out = None
    if rank == 0:
        base = None
        if world == 1 and not args.no_cpu_baseline:
            base = cpu_baseline(args.scale, args.edgefactor, args.cpu_cols_frac)
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "GFLOP/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 3), "higher_is_better": True,
            "scaling": "strong" if world > 1 else "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: packed Graph500 R-MAT (seed 0xDECAFBAD), bit-identical to the reference generator",
            "config": {"workload": f"rmat{args.scale}_ef{args.edgefactor}_AxA_PlusTimes_f64", "scale": args.scale,
                       "edgefactor": args.edgefactor, "nnzA": nnzA, "flops": int(flops), "nnzC": int(nnzC),
                       "phases": st["phases"], "parallelism": f"B column stripes x{world}" if world > 1 else "1 GPU",
                       "kernel_ms": {n: round(v["ms"] / max(args.steps, 1), 3) for n, v in ks.items()}},
            "roofline": roofline, "cpu_baseline": base, "check": check,
        }
        print(json.dumps(out), flush=True)
    barrier()
    del dA, dB
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
