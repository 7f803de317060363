#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: semiring GFLOP/s of R-MAT A^2 SpGEMM on MI355X, with the
HBM-roofline fraction of the dominant kernel and the reference's CPU time beside it.

Workload (N=1): config C2 = Graph500 R-MAT scale 22, edge factor 16, A*A with
PlusTimesSRing<double> (B is a separate copy of A, as Mult_AnXBn_Synch requires). One step = the
whole product: symbolic pass (estimateFLOP + exact nnz) and every numeric column phase; C
(24.8 G nonzeros, ~297 GB) exceeds HBM, so B's columns are processed in phases whose C blocks are
materialised in HBM one after another (MemEfficientSpGEMM's phase loop, ParFriends.h:449-730).
Inputs are resident in HBM before the timed region.

N>1 (launched by torch.distributed.run): the same fixed product on a process grid, as the
reference distributes it (north_star): 2D SUMMA with RCCL row/column broadcasts of the DCSC
blocks on a square world (4 GPUs = 2x2), 3D SUMMA otherwise (2 GPUs = 1x1x2, 8 GPUs = 2x2x2:
per-layer SUMMA + the fiber reduce-scatter as an RCCL alltoall), every phase of C materialised in
HBM -> "scaling": "strong". Timing: barrier + synchronize around exactly K steps, max over ranks.

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
DOMINANT_KERNEL = "cbh::task_kernel<cbh::PlusTimesD<double>, 4096, 512, 512, 8, 1>"


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
    p.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on a node; gloo only for rehearsals")
    p.add_argument("--share-gpu", action="store_true", help="rehearsal: every rank on cuda:0 (needs gloo)")
    return p.parse_args()


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


def grid_shape(world):
    """2D SUMMA on a square world (1, 4, 9, ...); otherwise 3D with the fewest layers that leave a
    square layer grid (2 -> 1x1x2, 8 -> 2x2x2), as BASELINE.json's north_star lays out."""
    import math

    for layers in range(1, world + 1):
        if world % layers == 0 and math.isqrt(world // layers) ** 2 == world // layers:
            return layers
    return world


def host_flops(A):
    """flops(A*A) = sum_k nnz(A(:,k)) * nnz(A(k,:)) (EstimateFLOP, ParFriends.h:355-441)"""
    colnnz = np.zeros(A.n, np.int64)
    colnnz[A.jc] = np.diff(A.cp)
    rownnz = np.bincount(A.ir, minlength=A.m).astype(np.int64)
    return int(np.dot(colnnz, rownnz))


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import combblas_amd as cb

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.share_gpu:  # rehearsal of the N-rank path on a one-GPU box (gloo, ranks share cuda:0)
        local = 0
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    def barrier():
        if world > 1:
            dist.barrier()

    def allreduce(x, op):
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        if world > 1:
            if args.dist_backend == "gloo":
                t = t.cpu()
            dist.all_reduce(t, op=op)
        return t.item()

    SR = cb.PlusTimesSRing
    A = cb.rmat(args.scale, args.edgefactor, dtype=np.float64)
    nnzA = A.nnz
    if world == 1:
        # ------------------------------------------------------------ 1 GPU: device phase loop
        ctx = cb.Context(local, torch_allocator=False)
        if args.phase_budget_gb > 0:
            ctx.set_phase_budget(int(args.phase_budget_gb * 2**30))
        dA = cb.SpDCCols.from_host(ctx, A)
        dB = cb.SpDCCols.from_host(ctx, A)  # separate copy (aliasing is rejected, ParFriends.h:172)
        del A

        def step():
            return cb.PhasedSpGEMM(SR, dA, dB)

        def verify():
            sv = cb.PhasedSpGEMM(SR, dA, dB, checksum=True)
            return sv["nnz"], sv["value_sum"]
        parallelism = "1 GPU"
    else:
        # ------------------------------------------------------------ N GPUs: SUMMA over RCCL
        from combblas_amd import parfriends as pf
        from combblas_amd.backend import HipBackend
        from combblas_amd.commgrid import CommGrid, CommGrid3D
        from combblas_amd.spparmat import SpParMat, SpParMat3D

        ctx = cb.Context(local)
        be = HipBackend(ctx)
        layers = grid_shape(world)
        flops_total = host_flops(A)
        budget = int(args.phase_budget_gb * 2**30) if args.phase_budget_gb > 0 else 0
        if layers == 1:
            grid = CommGrid()
            dA, dB = SpParMat.distribute(A, grid, be), SpParMat.distribute(A, grid, be)
            parallelism = f"2D SUMMA {grid.grrows}x{grid.grcols} (RCCL broadcasts)"
        else:
            g3 = CommGrid3D(layers)
            dA = SpParMat3D.distribute(A, g3, be, colsplit=True)
            dB = SpParMat3D.distribute(A, g3, be, colsplit=False)
            parallelism = f"3D SUMMA {g3.gridRows}x{g3.gridCols}x{layers} (RCCL broadcasts + fiber alltoall)"
        del A
        acc = {}

        def consume(C, c0, c1):
            acc["nnz"] = acc.get("nnz", 0) + be.dims(C)[2]
            if acc.get("sum") is not None:
                acc["sum"] += float(be.arrays(C)[3].sum().item()) if be.dims(C)[2] else 0.0

        def run():
            if layers == 1:
                ph = pf.MemEfficientSpGEMM(SR, dA, dB, phases=0, perProcessMemory=budget, on_phase=consume)
            else:
                ph = pf.Mult_AnXBn_SUMMA3D(SR, dA, dB, phases=0, perProcessMemory=budget, on_phase=consume)
            return ph

        def step():
            acc.clear()
            ph = run()
            return {"flops": flops_total, "nnz": acc["nnz"], "phases": ph}

        def verify():
            acc.clear()
            acc["sum"] = 0.0
            run()
            return acc["nnz"], acc["sum"]

    for _ in range(args.warmup):
        st = step()
    ctx.synchronize()
    ctx.enable_timing(True)
    ctx.reset_kernel_stats()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st = step()
    ctx.synchronize()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    ctx.enable_timing(False)
    ks = ctx.kernel_stats()

    my_s = (t1 - t0) / max(args.steps, 1)
    step_s = allreduce(my_s, dist.ReduceOp.MAX if world > 1 else None)
    flops = float(st["flops"])  # the whole product's multiplies (every rank knows the total)
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
    if os.path.exists(pmc):  # PMC passes of the same kernel (tools/pmc_traffic.py); stale files are ignored
        try:
            p = json.load(open(pmc))
            if p.get("kernel") == DOMINANT_KERNEL:
                roofline["traffic"] = p.get("hbm_bytes_per_launch")
                roofline["traffic_note"] = (f"HBM bytes per launch from rocprofv3 PMC (2xFETCH_SIZE+WRITE_SIZE, gfx950 "
                                            f"correction; raw {p.get('hbm_bytes_per_launch_raw')}), {p.get('source')}")
        except Exception:  # noqa: BLE001
            pass

    check = None
    if not args.no_verify:
        nz, vs = verify()
        nnz_all = allreduce(float(nz), dist.ReduceOp.SUM if world > 1 else None)
        vsum = allreduce(vs, dist.ReduceOp.SUM if world > 1 else None)
        known = {22: 24766243778, 20: 3284757756, 18: 425342972, 16: 53638834, 14: 6471508}.get(args.scale)
        check = {"nnzC": int(nnz_all), "value_sum": vsum, "expected_nnzC": known,
                 "ok": (known is None or int(nnz_all) == known)}

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
                       "phases": st["phases"], "parallelism": parallelism,
                       "kernel_ms": {n: round(v["ms"] / max(args.steps, 1), 3) for n, v in ks.items()}},
            "roofline": roofline, "cpu_baseline": base, "check": check,
        }
        print(json.dumps(out), flush=True)
    barrier()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
