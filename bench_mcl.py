#!/usr/bin/env python3
"""bench_mcl.py -- BASELINE.json config C5 on one MI355X: HipMCL's expansion A² followed by
MCLPruneRecoverySelect (Applications/MCL.cpp:574-577 -> ParFriends.h:449-730 with the prune of
:185-353), on the protein-similarity-like planted-partition input (combblas_amd.mclgen,
column-stochastic, ~44 nonzeros per column after symmetrisation), generated on the GPU
(mclgen.planted_partition_device). The config names n = 2^24 on a 2×2×2 grid of 8 GPUs; this line
runs the same size and pipeline on one GPU (the 8-GPU path is MemEfficientSpGEMM3D).

One step = parfriends.MemEfficientSpGEMM(PlusTimes, A, A, phases = planned from the exact symbolic
pass, hardThreshold = 1e-4, selectNum = 1100, recoverNum = 1400, recoverPct = 0.9 -- MCL.cpp's
defaults) on a 1×1 grid: every phase's block of A² is pruned on the device before it is kept.

Check on a sample of columns: the device expansion of those columns against the CPU oracle's
(structure exact, values within 1e-12), and the device's pruned columns against the oracle prune
(oracle/apps_oracle.py, pinned to the reference's MCLPruneRecoverySelect) of the device's own
unpruned columns (rows exact, values within 1e-12: the phased product and the sampled product may
split long columns into different chunk sums).

roofline: the task-kernel class with the most HIP-event time over the timed steps (bench.py's
kernel_roofline). CPU baseline ("reference"): MCL.cpp's own expansion call MemEfficientSpGEMM
with MCLPruneRecoverySelect (oracle/_ref/ref_harness mclexp, built from the reference sources) on
every --cpu-stride-th column of the right operand, 1 rank x host cores, median of 5 after a warm-up.
    python bench_mcl.py [--log2n 24] [--deg 100] [--steps 2] [--warmup 1] [--host-gen]
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

HARD, SELECT, RECOVER, PCT = 1e-4, 1100, 1400, 0.9  # MCL.cpp defaults (prunelimit, select, recover)


def log(msg):
    print(f"[bench_mcl] {msg}", file=sys.stderr, flush=True)


def reference_baseline(A, flops, stride):
    """MCL.cpp:574-577's expansion MemEfficientSpGEMM(A, A_s) + MCLPruneRecoverySelect by the
    reference itself (oracle/_ref/ref_harness mclexp) on A's columns c % stride == 0 as the right
    operand, 1 rank x host cores; None when oracle/_ref is absent"""
    import subprocess
    import tempfile

    ref = os.path.join(HERE, "oracle", "_ref", "ref_harness")
    if not os.path.exists(ref):
        return None
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import helpers as H

    if stride <= 0:
        stride = max(1, int(flops // 3e8))
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        fa = os.path.join(td, "A.cbm")
        H.write_cbm(fa, H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))
        env = dict(os.environ, OMP_NUM_THREADS=str(cores), LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:/opt/conda/lib")
        r = subprocess.run([ref, "mclexp", fa, str(stride), "5", str(HARD), str(SELECT), str(RECOVER), str(PCT)],
                           env=env, cwd="/tmp", capture_output=True, text=True, timeout=900)
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not line:
        log(f"reference baseline failed rc={r.returncode}: {r.stderr[-300:]}")
        return None
    d = json.loads(line[-1])
    return {"value": round(d["gflops"], 6), "unit": "GFLOP/s", "cores": d["threads"], "kind": "reference",
            "sample": f"MCL.cpp's expansion MemEfficientSpGEMM(A, A_s) with MCLPruneRecoverySelect (hard {HARD}, "
                      f"select {SELECT}, recover {RECOVER}/{PCT}; oracle/_ref built from the reference sources, 1 rank x "
                      f"{d['threads']} threads) on A's {d['cols']} columns c % {stride} == 0 ({d['flops']} multiplies, "
                      f"{d['nnz_after_prune']} kept): median of {d['reps']} after 1 warm-up = {d['median_s']:.3f} s"}


def cpp_line(args):
    """config C5 through the C++ driver HipMCL calls: oracle/_ref/mclbench_harness runs the
    reference-API MemEfficientSpGEMM on SpParMat<SpDCColsDev> (include/combblas_hip/ParFriendsDev.h,
    the overload Applications/MCL.cpp:574-577 resolves to), checks sampled columns against the
    reference's stock driver and times the stock driver on a column sample (the CPU baseline)"""
    import subprocess

    from combblas_amd import _lib
    from bench import kernel_roofline

    harness = os.path.join(HERE, "oracle", "_ref", "mclbench_harness")
    if not os.path.exists(harness):
        sys.exit("oracle/_ref/mclbench_harness is missing: run __graft_entry__.build() where the reference exists")
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    env = dict(os.environ, OMP_NUM_THREADS=str(cores), LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:/opt/conda/lib")
    cmd = [harness, str(args.log2n), str(args.deg), str(args.steps), str(args.phases), str(args.check_cols),
           str(args.cpu_stride)]
    r = subprocess.run(cmd, env=env, cwd="/tmp", capture_output=True, text=True, timeout=1100)
    for l in r.stdout.splitlines():
        if l.startswith("[memdiag]"):
            print(l, file=sys.stderr)
    line = [l for l in r.stdout.splitlines() if l.startswith("BENCHC5CPP ")]
    if not line:
        sys.exit(f"harness failed (rc {r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-3000:]}")
    d = json.loads(line[-1][len("BENCHC5CPP "):])
    ks = {name: {"ms": v[0], "launches": v[1], "alg_bytes": v[2]} for name, v in zip(_lib.K_NAMES, d["kernel_stats"])}
    out = {"metric": "HipMCL expansion A^2 + MCLPruneRecoverySelect (C5): semiring GFLOP/s of the expansion",
           "value": round(2.0 * d["flops"] / d["step_s"] / 1e9, 3), "unit": "GFLOP/s", "n_gpus": 1,
           "steps": d["steps"], "warmup": 1, "ms_per_step": round(d["step_s"] * 1e3, 3), "higher_is_better": True,
           "dtype": "f64",
           "data": f"synthetic: planted-partition generated on the GPU (cbh_gen_planted_partition), column-stochastic, "
                   f"n = 2^{args.log2n}, {args.deg} draws/col",
           "config": {"workload": f"mcl_pp{args.log2n}_deg{args.deg}_A2_prune", "n": d["n"], "nnzA": d["nnzA"],
                      "flops": d["flops"], "nnzC_unpruned": d["nnzC_unpruned"],
                      "nnz_after_prune": d["nnz_after_prune"], "phases": d["phases"],
                      "prune": {"hard": HARD, "select": SELECT, "recover": RECOVER, "pct": PCT},
                      "driver": "C++: combblas::MemEfficientSpGEMM on SpParMat<int64_t, double, SpDCColsDev> "
                                "(ParFriendsDev.h; StagePlans: one symbolic pass, numeric per phase)",
                      "parallelism": "1 GPU (config C5 names 2x2x2)", "kernel_ms": {k: round(v["ms"] / d["steps"], 3)
                                                                                   for k, v in ks.items() if v["ms"]}},
           "roofline": kernel_roofline(ks),
           "cpu_baseline": {"value": round(2.0 * d["cpu_flops"] / d["cpu_s"] / 1e9, 6), "unit": "GFLOP/s",
                            "cores": int(d["cpu_threads"]) or cores, "kind": "reference",
                            "sample": f"the reference's stock MemEfficientSpGEMM + MCLPruneRecoverySelect (OpenMP "
                                      f"kernels, same harness, 1 rank) on B = A's {d['cpu_cols']} columns c % "
                                      f"{d['cpu_stride']} == 0 ({d['cpu_flops']} multiplies, {d['cpu_kept']} kept): "
                                      f"median of 5 after 1 warm-up = {d['cpu_s']:.3f} s"},
           "check": {"sample_columns": d["check_cols"], "reference": "stock MemEfficientSpGEMM + prune on the sampled "
                                                                       "columns (rows exact, values 1e-12 relative)",
                     "row_mismatches": d["row_mismatches"], "value_mismatches": d["value_mismatches"],
                     "max_rel": d["max_rel"], "ok": d["ok"]}}
    print(json.dumps(out), flush=True)
    if not d["ok"] or r.returncode != 0:
        sys.exit(1)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--driver", choices=["python", "cpp"], default="python",
                   help="python: the parfriends mirror; cpp: the C++ overload (oracle/_ref/mclbench_harness)")
    p.add_argument("--gen", choices=["lib", "torch"], default="lib",
                   help="lib: cbh_gen_planted_partition (the C++ harness's input); torch: mclgen.planted_partition_device")
    p.add_argument("--phases", type=int, default=0, help="cpp driver: MemEfficientSpGEMM's phases (0: C's phase "
                                                          "blocks within 0.4 of free HBM, as the Python mirror)")
    p.add_argument("--log2n", type=int, default=24)
    p.add_argument("--deg", type=int, default=100)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--check-cols", type=int, default=100)
    p.add_argument("--host-gen", action="store_true", help="numpy generator (mclgen.planted_partition)")
    p.add_argument("--cpu-stride", type=int, default=0, help="0: about 3e8 multiplies in the CPU sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    args = p.parse_args()
    if args.driver == "cpp":
        return cpp_line(args)
    import torch

    import combblas_amd as cb
    from combblas_amd import parfriends as pf
    from combblas_amd.backend import HipBackend
    from combblas_amd.commgrid import CommGrid
    from combblas_amd.mclgen import planted_partition, planted_partition_device, planted_partition_lib
    from combblas_amd.spparmat import SpParMat

    torch.cuda.set_device(0)
    n = 1 << args.log2n
    ctx = cb.Context(0)
    be = HipBackend(ctx)
    grid = CommGrid()
    t0 = time.perf_counter()
    if args.host_gen:
        A = planted_partition(n, args.deg, 7)
        dA, dB = SpParMat.distribute(A, grid, be), SpParMat.distribute(A, grid, be)
    else:
        gA = (planted_partition_lib if args.gen == "lib" else planted_partition_device)(ctx, n, args.deg, 7)
        dA, dB = SpParMat(gA, grid, be, n, n), SpParMat(gA.clone(), grid, be, n, n)
        A = gA.to_host()
    log(f"input: n {n}, nnz {A.nnz} ({time.perf_counter() - t0:.1f} s)")
    colnnz = np.zeros(n, np.int64)
    colnnz[A.jc] = np.diff(A.cp)
    flops = int((np.bincount(A.ir, minlength=n).astype(np.int64) * colnnz).sum())  # sum_k nnz(A(:,k)) nnz(A(k,:))
    rng = np.random.default_rng(11)
    sample = np.sort(rng.choice(n, size=args.check_cols, replace=False))
    got = {}

    def keep_sample(C, c0, c1):
        cp, jc, ir, num = be.arrays(C)
        sel = torch.nonzero(torch.isin(jc, torch.as_tensor(sample, device=jc.device))).flatten()
        for s in sel.tolist():
            j = int(jc[s].item())
            a, b = int(cp[s].item()), int(cp[s + 1].item())
            got[j] = (ir[a:b].cpu().numpy(), num[a:b].cpu().numpy())
        be.free(C)

    def step(consume):
        return pf.MemEfficientSpGEMM(cb.PlusTimesSRing, dA, dB, phases=0, hardThreshold=HARD, selectNum=SELECT,
                                     recoverNum=RECOVER, recoverPct=PCT, on_phase=consume)

    kept = {"nnz": 0}

    def count(C, c0, c1):
        kept["nnz"] += be.dims(C)[2]
        be.free(C)

    for _ in range(args.warmup):
        step(count)
    ctx.synchronize()
    torch.cuda.synchronize()
    ctx.reset_kernel_stats()
    ctx.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        kept["nnz"] = 0
        phases = step(count)
    ctx.synchronize()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    ctx.enable_timing(False)
    from bench import kernel_roofline

    roofline = kernel_roofline(ctx.kernel_stats())
    log(f"{args.steps} step(s): {dt * 1e3:.1f} ms/step, {phases} phases, nnz after prune {kept['nnz']}")
    step(keep_sample)  # the sampled pruned columns

    # the check: device expansion of the sample vs the oracle, and the oracle prune of it
    sys.path.insert(0, os.path.join(HERE, "tests"))
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import apps_oracle as AO
    import helpers as H

    d = H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num)
    cols = np.concatenate([np.arange(d.cp[j], d.cp[j + 1]) for j in sample])
    lens = np.array([d.cp[j + 1] - d.cp[j] for j in sample])
    Bs = H.Dcsc(n, args.check_cols, np.arange(args.check_cols), np.concatenate([[0], np.cumsum(lens)]),
                d.ir[cols], d.num[cols])
    dAs = dA.seq if not args.host_gen else cb.SpDCCols.from_host(ctx, cb.HostDcsc(d.m, d.n, d.jc, d.cp, d.ir, d.num))
    dev = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dAs,
                               cb.SpDCCols.from_host(ctx, cb.HostDcsc(Bs.m, Bs.n, Bs.jc, Bs.cp, Bs.ir, Bs.num))).to_host()
    devC = H.Dcsc(dev.m, dev.n, dev.jc, dev.cp, dev.ir, dev.num)
    ora = H.Oracle().spgemm(d, Bs, "plus_times", "hybrid", threads=int(os.environ.get("OMP_NUM_THREADS", "8")))
    exp_ok = bool(np.array_equal(devC.jc, ora.jc) and np.array_equal(devC.cp, ora.cp) and np.array_equal(devC.ir, ora.ir)
                  and np.allclose(devC.num, ora.num, rtol=1e-12, atol=0))
    pruned = AO.mcl_prune_recovery_select(devC, HARD, SELECT, RECOVER, PCT)
    bad = badv = 0
    first = None
    for i, j in enumerate(sample):
        s = np.searchsorted(pruned.jc, i)
        er = pruned.ir[pruned.cp[s]:pruned.cp[s + 1]] if s < pruned.jc.size and pruned.jc[s] == i else np.zeros(0)
        ev = pruned.num[pruned.cp[s]:pruned.cp[s + 1]] if s < pruned.jc.size and pruned.jc[s] == i else np.zeros(0)
        gr, gv = got.get(int(j), (np.zeros(0), np.zeros(0)))
        if not np.array_equal(gr, er):
            bad += 1
            if first is None:
                u = devC.cp[np.searchsorted(devC.jc, i) + 1] - devC.cp[np.searchsorted(devC.jc, i)]
                first = {"col": int(j), "got": int(gr.size), "expected": int(er.size), "unpruned": int(u),
                         "got_not_expected": int(np.setdiff1d(gr, er).size)}
        elif not np.allclose(gv, ev, rtol=1e-12, atol=0):
            badv += 1
    base = None if args.no_cpu_baseline else reference_baseline(A, flops, args.cpu_stride)
    out = {"metric": "HipMCL expansion A^2 + MCLPruneRecoverySelect (C5): semiring GFLOP/s of the expansion",
           "value": round(2.0 * flops / dt / 1e9, 3), "unit": "GFLOP/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "f64",
           "data": f"synthetic: planted-partition ({'host numpy' if args.host_gen else 'generated on the GPU: ' + args.gen}), "
                   f"column-stochastic, n = 2^{args.log2n}, {args.deg} draws/col",
           "config": {"workload": f"mcl_pp{args.log2n}_deg{args.deg}_A2_prune", "n": n, "nnzA": int(A.nnz),
                      "flops": flops, "phases": phases, "nnz_after_prune": int(kept["nnz"]),
                      "prune": {"hard": HARD, "select": SELECT, "recover": RECOVER, "pct": PCT},
                      "parallelism": "1 GPU (config C5 names 2x2x2)"},
           "roofline": roofline, "cpu_baseline": base,
           "check": {"sample_columns": int(args.check_cols), "expansion_matches_oracle": exp_ok,
                     "pruned_row_mismatches": bad,
                     "pruned_value_mismatches": badv, "first_mismatch": first, "ok": exp_ok and bad == 0 and badv == 0}}
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
