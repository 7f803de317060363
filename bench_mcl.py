#!/usr/bin/env python3
"""bench_mcl.py -- BASELINE.json config C5 on one MI355X: HipMCL's expansion A² followed by
MCLPruneRecoverySelect (Applications/MCL.cpp:574-577 -> ParFriends.h:449-730 with the prune of
:185-353), on the protein-similarity-like planted-partition input (combblas_amd.mclgen,
column-stochastic, ~100 nonzeros per column). The config names n = 2^24 on a 2×2×2 grid of 8 GPUs;
this line runs the same pipeline on one GPU at n = 2^20 by default (host generation of the input
takes ~50 s there and grows faster than linearly; the 8-GPU path is MemEfficientSpGEMM3D).

One step = parfriends.MemEfficientSpGEMM(PlusTimes, A, A, phases = planned from the exact symbolic
pass, hardThreshold = 1e-4, selectNum = 1100, recoverNum = 1400, recoverPct = 0.9 -- MCL.cpp's
defaults) on a 1×1 grid: every phase's block of A² is pruned on the device before it is kept.

Check on a sample of columns: the device expansion of those columns against the CPU oracle's
(structure exact, values within 1e-12), and the device's pruned columns against the oracle prune
(oracle/apps_oracle.py, pinned to the reference's MCLPruneRecoverySelect) of the device's own
unpruned columns (rows exact, values within 1e-12: the phased product and the sampled product may
split long columns into different chunk sums).
    python bench_mcl.py [--log2n 20] [--deg 100] [--steps 2] [--warmup 1]
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--log2n", type=int, default=20)
    p.add_argument("--deg", type=int, default=100)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--check-cols", type=int, default=100)
    args = p.parse_args()
    import torch

    import combblas_amd as cb
    from combblas_amd import parfriends as pf
    from combblas_amd.backend import HipBackend
    from combblas_amd.commgrid import CommGrid
    from combblas_amd.mclgen import planted_partition
    from combblas_amd.spparmat import SpParMat

    torch.cuda.set_device(0)
    n = 1 << args.log2n
    t0 = time.perf_counter()
    A = planted_partition(n, args.deg, 7)
    log(f"input: n {n}, nnz {A.nnz} ({time.perf_counter() - t0:.1f} s)")
    colnnz = np.zeros(n, np.int64)
    colnnz[A.jc] = np.diff(A.cp)
    flops = int((np.bincount(A.ir, minlength=n).astype(np.int64) * colnnz).sum())  # sum_k nnz(A(:,k)) nnz(A(k,:))
    ctx = cb.Context(0)
    be = HipBackend(ctx)
    grid = CommGrid()
    dA, dB = SpParMat.distribute(A, grid, be), SpParMat.distribute(A, grid, be)
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
    t0 = time.perf_counter()
    for _ in range(args.steps):
        kept["nnz"] = 0
        phases = step(count)
    ctx.synchronize()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
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
    hA = cb.HostDcsc(d.m, d.n, d.jc, d.cp, d.ir, d.num)
    dev = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, cb.SpDCCols.from_host(ctx, hA),
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
    # CPU baseline: the oracle expansion + prune of the first n/8 columns (OpenMP over the host cores)
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    nb = n // 8
    e = int(np.searchsorted(d.jc, nb))
    Bb = H.Dcsc(n, nb, d.jc[:e], d.cp[:e + 1] - d.cp[0], d.ir[d.cp[0]:d.cp[e]], d.num[d.cp[0]:d.cp[e]])
    bflops = int(colnnz[Bb.ir].sum())
    t1 = time.perf_counter()
    Cb = H.Oracle().spgemm(d, Bb, "plus_times", "hybrid", threads=cores)
    te = time.perf_counter() - t1
    AO.mcl_prune_recovery_select(Cb, HARD, SELECT, RECOVER, PCT)
    tb = time.perf_counter() - t1
    base = {"value": round(2.0 * bflops / tb / 1e9, 6), "unit": "GFLOP/s", "cores": cores, "kind": "port",
            "sample": f"columns [0, n/8) ({bflops} flops): CPU oracle expansion (restatement of the reference's "
                      f"LocalHybridSpGEMM, OpenMP over {cores} threads) + the numpy prune restatement, {tb:.2f} s (expansion alone {te:.2f} s = "
                      f"{2.0 * bflops / te / 1e9:.4f} GFLOP/s)"}
    out = {"metric": "HipMCL expansion A^2 + MCLPruneRecoverySelect (C5): semiring GFLOP/s of the expansion",
           "value": round(2.0 * flops / dt / 1e9, 3), "unit": "GFLOP/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "f64",
           "data": f"synthetic: planted-partition, column-stochastic, n = 2^{args.log2n}, ~{args.deg} nnz/col",
           "config": {"workload": f"mcl_pp{args.log2n}_deg{args.deg}_A2_prune", "n": n, "nnzA": int(A.nnz),
                      "flops": flops, "phases": phases, "nnz_after_prune": int(kept["nnz"]),
                      "prune": {"hard": HARD, "select": SELECT, "recover": RECOVER, "pct": PCT},
                      "parallelism": "1 GPU (config C5 names 2x2x2)"},
           "cpu_baseline": base,
           "check": {"sample_columns": int(args.check_cols), "expansion_matches_oracle": exp_ok,
                     "pruned_row_mismatches": bad,
                     "pruned_value_mismatches": badv, "first_mismatch": first, "ok": exp_ok and bad == 0 and badv == 0}}
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
