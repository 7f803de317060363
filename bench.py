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
reference distributes it (north_star): 2D SUMMA on a square world (4 GPUs = 2x2), 3D SUMMA otherwise
(2 GPUs = 1x1x2, 8 GPUs = 2x2x2: per-layer SUMMA + the fiber reduce-scatter), every phase of C
materialised in HBM -> "scaling": "strong". The host side is the C++ one north_star names
(--driver auto/cpp): rank 0 runs cxx/_build/bench_summa under mpirun -- the reference's SpParMat /
SpParMat3D over device blocks, RCCL broadcasts and fiber exchange -- while the torch ranks wait on
a CPU barrier; --driver python runs combblas_amd's Python drivers over torch.distributed instead
(auto falls back to them when the C++ run fails cleanly). Timing: barrier + synchronize around
exactly K steps, max over ranks.

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
# the task kernels of one product (bench kernel kinds -> rocprof names); the roofline line reports
# the one with the most time per step
KERNELS = {"num_large": "cbh::task_kernel<cbh::PlusTimesD<double>, 2048, 512, 512, 4, 1, false>",
           # round 5: the dense tasks' kernel (device/dense_kernel.h; CBH_DENSE_V2=0 builds the round-4
           # "cbh::task_kernel<cbh::PlusTimesD<double>, 4096, 512, 512, 8, 2, false>")
           "num_dense": "cbh::dense_kernel<cbh::PlusTimesD<double>, 1024, 512, 8, 163776, 0>",
           "sym_large": "cbh::task_kernel<cbh::PlusTimesD<long>, 8192, 512, 512, 16, 0, false>",
           # round 5: the symbolic pass's large bitmap tasks (device/dense_kernel.h, SYM)
           "sym_bmp": "cbh::dense_kernel<cbh::PlusTimesD<long>, 1024, 512, 8, 163776, 1>"}
# every task-kernel class of the f64 PlusTimes product (the application lines pick their dominant one)
ALL_KERNELS = dict(KERNELS, **{
    "num_mid": "cbh::task_kernel<cbh::PlusTimesD<double>, 2048, 256, 256, 4, 1, false>",
    # one task per wave (wave_kernel.h): per-wave key hash tables sized so that they never fill
    "num_small": "cbh::wave_kernel<cbh::PlusTimesD<double>, 512, 4, 4, 1>",
    "sym_mid": "cbh::task_kernel<cbh::PlusTimesD<long>, 4096, 256, 256, 4, 0, false>",
    "sym_small": "cbh::wave_kernel<cbh::PlusTimesD<long>, 2048, 4, 4, 0>"})


def kernel_roofline(ks, kernels=None):
    """roofline object of the task-kernel class with the most HIP-event time in the library's
    per-kind stats `ks` (ctx.kernel_stats()): algorithmic bytes of its launches / their duration"""
    kernels = kernels or ALL_KERNELS
    kinds = [k for k in kernels if ks.get(k, {}).get("ms", 0) > 0]
    if not kinds:
        return None

    def gbs(kind):
        return ks[kind]["alg_bytes"] / (ks[kind]["ms"] / 1e3) / 1e9

    dom = max(kinds, key=lambda kind: ks[kind]["ms"])
    k = ks[dom]
    a = gbs(dom)
    return {"bound": "hbm", "achieved": round(a, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(a / HBM_PEAK_GBS, 4), "traffic": None, "kernel": kernels[dom], "launches": k["launches"],
            "avg_launch_ms": round(k["ms"] / max(k["launches"], 1), 4),
            "alg_bytes_per_launch": round(k["alg_bytes"] / max(k["launches"], 1)),
            "others": {kind: round(gbs(kind) / HBM_PEAK_GBS, 4) for kind in kinds if kind != dom}}


_T0 = time.perf_counter()


def log(msg):
    """stage progress on stderr (the JSON line alone goes to stdout)"""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


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
    p.add_argument("--no-merge", action="store_true", help="skip the MultiwayMerge measurement (N=1)")
    p.add_argument("--merge-cols-frac", type=float, default=1.0 / 16, help="B column block of the merge sample")
    p.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on a node; gloo only for rehearsals")
    p.add_argument("--share-gpu", action="store_true", help="rehearsal: every rank on cuda:0 (needs gloo)")
    p.add_argument("--driver", default="auto", choices=["auto", "cpp", "python"],
                   help="N>1: cpp = the C++ host path (cxx/bench_summa under mpirun), python = combblas_amd's "
                        "drivers; auto = cpp when it is built, python if it fails to start")
    p.add_argument("--phases", type=int, default=0, help="N>1 cpp driver: column phases (0 = planned)")
    p.add_argument("--cpp-timeout", type=float, default=600.0, help="N>1 cpp driver: seconds before it is killed "
                                                                       "(auto: the python drivers run instead)")
    return p.parse_args()


def cpu_baseline(scale, ef, frac):
    """Reference Mult_AnXBn_Synch (MPI+OpenMP) on a bounded column sample of the same product,
    C = A * A(:, c % stride == 0) (stride = 1/frac: the sample spreads over every processor column
    of a multi-rank grid), on this host's cores: one untimed warm-up call, median of 5 timed calls,
    for 1 rank x all cores and 4 ranks (2x2 grid) x cores/4; the faster layout is reported.
    Falls back to the oracle port when oracle/_ref is absent."""
    n = 1 << scale
    stride = max(1, round(1 / frac))
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    ref = os.path.join(HERE, "oracle", "_ref", "ref_harness")
    sample = f"C = A*A(:, 0:{n}:{stride}) of R-MAT scale {scale} ef {ef} (1/{stride} of B's columns, strided)"
    if os.path.exists(ref):
        best, tried = None, []
        mpirun = "/opt/conda/bin/mpirun"
        layouts = [(1, cores)] + ([(4, max(1, cores // 4))] if cores >= 4 and os.path.exists(mpirun) else [])
        for ranks, thr in layouts:
            env = dict(os.environ, OMP_NUM_THREADS=str(thr),
                       LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:/opt/conda/lib")
            cmd = [ref, "slice", str(scale), str(ef), "0", str(n), "5", "pt_f64", str(stride)]
            if ranks > 1:
                cmd = [mpirun, "-np", str(ranks)] + cmd
            log(f"CPU baseline layout {ranks} rank(s) x {thr} threads")
            try:
                r = subprocess.run(cmd, env=env, cwd="/tmp", capture_output=True, text=True, timeout=600)
                line = [l for l in r.stdout.splitlines() if l.startswith("{")]
                if r.returncode == 0 and line:
                    d = json.loads(line[-1])
                    tried.append(f"{ranks}x{thr}: {d['gflops']:.4f} GFLOP/s (median {d['median_s']:.3f} s)")
                    if best is None or d["gflops"] > best["gflops"]:
                        best = d
                else:
                    tried.append(f"{ranks}x{thr}: failed rc={r.returncode}")
            except Exception as e:  # noqa: BLE001
                tried.append(f"{ranks}x{thr}: {e}")
        if best is not None:
            return {"value": round(best["gflops"], 6), "unit": "GFLOP/s", "cores": best["ranks"] * best["threads"],
                    "kind": "reference",
                    "sample": sample + f": {best['flops']} flops, median of {best['reps']} after 1 warm-up = "
                                       f"{best['median_s']:.3f} s on {best['ranks']} rank(s) x {best['threads']} "
                                       f"threads (Mult_AnXBn_Synch, oracle/_ref built from the reference sources); "
                                       f"layouts tried: " + "; ".join(tried)}
        print("reference CPU baseline failed: " + "; ".join(tried), file=sys.stderr)
    # port: the oracle restatement (tests-only code, used here only as the CPU baseline leg)
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import helpers as H
    import combblas_amd as cb

    A = cb.rmat(scale, ef, dtype=np.float64)
    d = H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num)
    keep = np.nonzero(d.jc % stride == 0)[0]
    B = H.Dcsc(d.m, d.n, d.jc[keep], np.concatenate([[0], np.cumsum(np.diff(d.cp)[keep])]),
               np.concatenate([d.ir[d.cp[i]:d.cp[i + 1]] for i in keep]),
               np.concatenate([d.num[d.cp[i]:d.cp[i + 1]] for i in keep]))
    O = H.Oracle()
    O.spgemm(d, B, "plus_times", "hybrid", threads=cores)  # warm-up
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        C = O.spgemm(d, B, "plus_times", "hybrid", threads=cores)
        ts.append(time.perf_counter() - t0)
    dt = sorted(ts)[2]
    flops = O.symbolic(d, B, threads=cores)[0]
    return {"value": round(2 * flops / dt / 1e9, 6), "unit": "GFLOP/s", "cores": cores, "kind": "port",
            "sample": sample + f": {flops} flops, median of 5 after 1 warm-up = {dt:.3f} s (oracle restatement), "
                               f"nnzC {C.nnz}"}


def host_block(A, c0, c1, r0, r1):
    """A(r0:r1, c0:c1) of a HostDcsc with the same dimensions (entries outside are dropped)"""
    import combblas_amd as cb

    cols = np.repeat(A.jc, np.diff(A.cp))
    keep = (cols >= c0) & (cols < c1) & (A.ir >= r0) & (A.ir < r1)
    c = cols[keep]
    jc, counts = np.unique(c, return_counts=True)
    return cb.HostDcsc(A.m, A.n, jc, np.concatenate([[0], np.cumsum(counts)]), A.ir[keep], A.num[keep])


def merge_measurement(A, frac, steps):
    """MultiwayMerge (MultiwayMerge.h:411-526) of two SUMMA-stage partials on one GPU, as a 2-stage
    SUMMA would produce them: the inner dimension split in halves, P_s = A(:, K_s) * A(K_s, J) for a
    block J of B's columns, then C(:, J) = P_1 + P_2 by cbh_merge. Timed with HIP events on the
    library stream (merge_sym + merge_num kernels), checked against the unsplit product."""
    import combblas_amd as cb

    ctx = cb.Context(0)  # torch-allocated: the check compares device tensors
    n = A.n
    J = max(1, int(n * frac))
    h = n // 2
    B = host_block(A, 0, J, 0, n)
    dA = [cb.SpDCCols.from_host(ctx, host_block(A, 0, h, 0, n)), cb.SpDCCols.from_host(ctx, host_block(A, h, n, 0, n))]
    dB = [cb.SpDCCols.from_host(ctx, host_block(B, 0, J, 0, h)), cb.SpDCCols.from_host(ctx, host_block(B, 0, J, h, n))]
    P = [cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dA[i], dB[i]) for i in range(2)]
    for x in dA + dB:
        x.free()
    ctx.synchronize()
    ctx.reset_kernel_stats()
    ctx.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        M = cb.MultiwayMerge(cb.PlusTimesSRing, P, A.m, A.n)
        M.free()
    ctx.synchronize()
    wall = (time.perf_counter() - t0) / steps
    ctx.enable_timing(False)
    ks = ctx.kernel_stats()
    M = cb.MultiwayMerge(cb.PlusTimesSRing, P, A.m, A.n)
    full = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, cb.SpDCCols.from_host(ctx, A), cb.SpDCCols.from_host(ctx, B))
    ok = M.nnz == full.nnz and bool((M.tensors()[2] == full.tensors()[2]).all().item()) and \
        bool((M.tensors()[3] == full.tensors()[3]).all().item())
    kms = (ks["merge_sym"]["ms"] + ks["merge_num"]["ms"]) / steps
    num_ms = ks["merge_num"]["ms"] / max(ks["merge_num"]["launches"], 1) * (ks["merge_num"]["launches"] / steps)
    alg = ks["merge_num"]["alg_bytes"] / steps  # (s_i+s_v) * (entries read + outputs written)
    out = {"sample": f"C(:, 0:{J}) = P1 + P2, inner dimension split at {h} (2-stage SUMMA partials)",
           "nnz_partials": [P[0].nnz, P[1].nnz], "nnz_merged": M.nnz, "matches_unsplit_product": ok,
           "merge_ms": round(kms, 3), "merge_num_ms": round(num_ms, 3), "wall_ms": round(wall * 1e3, 3),
           "roofline": {"bound": "hbm", "achieved": round(alg / (num_ms / 1e3) / 1e9, 2) if num_ms > 0 else 0.0,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(alg / (num_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4) if num_ms > 0 else 0.0,
                        "alg_bytes_per_merge": round(alg)}}
    for x in P + [M, full]:
        x.free()
    ctx.close()
    return out


def grid_shape(world):
    """2D SUMMA on a square world (1, 4, 9, ...); otherwise 3D with the fewest layers that leave a
    square layer grid (2 -> 1x1x2, 8 -> 2x2x2), as BASELINE.json's north_star lays out."""
    import math

    for layers in range(1, world + 1):
        if world % layers == 0 and math.isqrt(world // layers) ** 2 == world // layers:
            return layers
    return world


def product_value_sum(A):
    """closed form of sum(A*A) under PlusTimes: sum_k colsum_k(A) * rowsum_k(A) (exact: integer
    multiplicities)"""
    colsum = np.zeros(A.n, np.float64)
    colsum[A.jc] = np.add.reduceat(A.num.astype(np.float64), A.cp[:-1]) if A.nnz else 0
    rowsum = np.bincount(A.ir, weights=A.num.astype(np.float64), minlength=A.m)
    return int(np.dot(colsum.astype(np.int64), rowsum.astype(np.int64)))


def reference_digest(scale, ef):
    """order-sensitive digest of the whole f64 product computed by the reference's own
    LocalHybridSpGEMM (tests/golden/make_golden_s22.py), when it is on file for this size"""
    p = os.path.join(HERE, "tests", "golden", f"scale{scale}.json")
    try:
        g = json.load(open(p))
        return g["pt_f64"]["total"]["digest"] if g.get("edgefactor") == ef else None
    except Exception:  # noqa: BLE001
        return None


def host_flops(A):
    """flops(A*A) = sum_k nnz(A(:,k)) * nnz(A(k,:)) (EstimateFLOP, ParFriends.h:355-441)"""
    colnnz = np.zeros(A.n, np.int64)
    colnnz[A.jc] = np.diff(A.cp)
    rownnz = np.bincount(A.ir, minlength=A.m).astype(np.int64)
    return int(np.dot(colnnz, rownnz))


# (CBH_BENCH_SUMMA / CBH_MPIRUN: test hooks, tests/test_bench_launcher.py runs the launcher on CPU
# with a stand-in binary)
CPP_BENCH = os.environ.get("CBH_BENCH_SUMMA", os.path.join(HERE, "cxx", "_build", "bench_summa"))
MPIRUN = os.environ.get("CBH_MPIRUN", "/opt/conda/bin/mpirun")
KNOWN_NNZC = {22: 24766243778, 20: 3284757756, 18: 425342972, 16: 53638834, 14: 6471508}


def cpp_driver(args, world, rank):
    """N>1 through the C++ host path north_star names: every torch.distributed rank joins a CPU
    (gloo) group, rank 0 starts `mpirun -np N cxx/_build/bench_summa` (the reference's SpParMat /
    SpParMat3D over device blocks, RCCL collectives; one MPI rank per GPU) with the launcher's
    variables removed, and the other ranks wait on the group; none of these processes touches a GPU.
    Returns the JSON line (rank 0) or None; raises RuntimeError when the C++ run failed cleanly
    (auto: the python drivers run instead)."""
    import datetime

    import torch.distributed as dist
    import combblas_amd as cb

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    dist.init_process_group("gloo", timeout=datetime.timedelta(hours=4))
    status = [None]
    if rank == 0:
        try:
            status[0] = _cpp_rank0(args, world, cb)
        except Exception as e:  # noqa: BLE001
            status[0] = {"error": str(e)}
    dist.broadcast_object_list(status, src=0)
    dist.destroy_process_group()
    st = status[0]
    if "error" in st:
        if st.get("fatal") or args.driver == "cpp":
            print(f"C++ driver failed: {st['error']}", file=sys.stderr, flush=True)
            sys.exit(1)
        raise RuntimeError(st["error"])
    return st if rank == 0 else None


def _cpp_rank0(args, world, cb):
    log(f"generating R-MAT scale {args.scale} (flops and the closed-form checksum)")
    A = cb.rmat(args.scale, args.edgefactor, dtype=np.float64)
    flops, closed_sum, nnzA = host_flops(A), product_value_sum(A), A.nnz
    del A
    drop = {"RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE", "ROLE_RANK",
            "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
            "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_USE_AGENT_STORE",
            "TORCH_NCCL_ASYNC_ERROR_HANDLING", "OMP_NUM_THREADS"}
    env = {k: v for k, v in os.environ.items() if k not in drop and not k.startswith("TORCHELASTIC_")}
    env["LD_LIBRARY_PATH"] = "/usr/lib/x86_64-linux-gnu:/opt/conda/lib:" + env.get("LD_LIBRARY_PATH", "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["OMP_NUM_THREADS"] = "4"
    if args.share_gpu:  # rehearsal: the ranks share cuda:0, so the exchanges are staged through host MPI
        env["COMBBLAS_HIP_COMM"] = "mpi"
    cmd = [MPIRUN, "-np", str(world), CPP_BENCH, str(args.scale), str(args.steps), str(args.warmup), str(args.phases)]
    log("C++ driver: " + " ".join(cmd))
    t0 = time.perf_counter()
    # own session: on a time-out the whole mpirun tree (hydra proxies and ranks) is killed
    pr = subprocess.Popen(cmd, env=env, cwd=HERE, stdout=subprocess.PIPE, text=True, start_new_session=True)
    try:
        stdout, _ = pr.communicate(timeout=args.cpp_timeout)  # stderr streams through
        rc = pr.returncode
    except subprocess.TimeoutExpired:
        os.killpg(pr.pid, 9)
        stdout, _ = pr.communicate()
        return {"error": f"bench_summa exceeded {args.cpp_timeout} s (killed)", "fatal": False}
    wall = time.perf_counter() - t0
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    if rc != 0 or not lines:
        crashed = rc < 0 or rc in (124, 134, 137, 139)
        return {"error": f"bench_summa rc={rc}: {stdout[-2000:]}", "fatal": crashed}
    d = json.loads(lines[-1])
    step_s = d["ms_per_step"] / 1e3
    known = KNOWN_NNZC.get(args.scale)
    gold = reference_digest(args.scale, args.edgefactor)
    dg = d.get("digest")
    check = {"nnzC": d["nnzC"], "expected_nnzC": known, "value_sum": d["value_sum"],
             "expected_value_sum": float(closed_sum), "digest": dg, "reference_digest": gold}
    check["ok"] = bool((known is None or d["nnzC"] == known) and d["value_sum"] == float(closed_sum)
                       and (gold is None or dg == gold))
    ks = {k: {"ms": v[0], "launches": v[1], "alg_bytes": v[2]} for k, v in d.get("kernel_stats_rank0", {}).items()}
    roofline = kernel_roofline(ks, KERNELS) if ks else None
    if roofline:
        roofline["note"] = "rank 0's kernels (HIP events inside the C++ driver)"
    return {
        "metric": METRIC, "value": round(2.0 * flops / step_s / 1e9, 3), "unit": "GFLOP/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(d["ms_per_step"], 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: packed Graph500 R-MAT (seed 0xDECAFBAD), bit-identical to the reference generator",
        "config": {"workload": f"rmat{args.scale}_ef{args.edgefactor}_AxA_PlusTimes_f64", "scale": args.scale,
                   "edgefactor": args.edgefactor, "nnzA": nnzA, "flops": int(flops), "nnzC": int(d["nnzC"]),
                   "phases": d["phases"], "parallelism": f"{d['grid']} ({d['transport']})",
                   "host_path": "C++: " + d["driver"] + ", mpirun -np " + str(world),
                   "kernel_ms": {k: round(v["ms"] / max(args.steps, 1), 3) for k, v in ks.items()},
                   "setup_s": d["setup_s"], "driver_wall_s": round(wall, 1)},
        "roofline": roofline, "cpu_baseline": None, "check": check, "merge": None,
    }


def main():
    args = parse()
    cpp_fallback = None
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and (args.driver == "cpp" or (args.driver == "auto" and os.path.exists(CPP_BENCH)
                                               and os.path.exists(MPIRUN))):
        try:
            out = cpp_driver(args, world, rank)
            if rank == 0:
                print(json.dumps(out), flush=True)
            return
        except RuntimeError as e:
            log(f"C++ driver did not run ({e}); python drivers instead")
            cpp_fallback = str(e)[:500]  # recorded in the JSON line: the line is NOT the C++ host path
    import torch
    import torch.distributed as dist
    import combblas_amd as cb

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
    log(f"generating R-MAT scale {args.scale}")
    A = cb.rmat(args.scale, args.edgefactor, dtype=np.float64)
    nnzA = A.nnz
    closed_sum = product_value_sum(A)
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
            return sv["nnz"], sv["value_sum"], sv["digest"]
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
            return acc["nnz"], acc["sum"], None

    log(f"{args.warmup} warm-up step(s)")
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
    log(f"{args.steps} timed step(s): {(t1 - t0) / max(args.steps, 1) * 1e3:.1f} ms/step")

    my_s = (t1 - t0) / max(args.steps, 1)
    step_s = allreduce(my_s, dist.ReduceOp.MAX if world > 1 else None)
    flops = float(st["flops"])  # the whole product's multiplies (every rank knows the total)
    nnzC = allreduce(float(st["nnz"]), dist.ReduceOp.SUM if world > 1 else None)
    value = 2.0 * flops / step_s / 1e9

    roofline = kernel_roofline(ks, KERNELS)
    dominant = [kind for kind, name in KERNELS.items() if name == roofline["kernel"]][0]
    pmc = os.path.join(HERE, "profiles", f"pmc_{dominant}.json")
    if os.path.exists(pmc):  # PMC passes of the same kernel (tools/pmc_traffic.py); stale files are ignored
        try:
            p = json.load(open(pmc))
            if p.get("kernel") == KERNELS[dominant]:
                roofline["traffic"] = p.get("hbm_bytes_per_launch")
                roofline["traffic_note"] = (f"HBM bytes per launch from rocprofv3 PMC (2xFETCH_SIZE+WRITE_SIZE, gfx950 "
                                            f"correction; raw {p.get('hbm_bytes_per_launch_raw')}), {p.get('source')}")
        except Exception:  # noqa: BLE001
            pass

    check = None
    if not args.no_verify:
        log("verification product (checksums)")
        nz, vs, dg = verify()
        nnz_all = allreduce(float(nz), dist.ReduceOp.SUM if world > 1 else None)
        vsum = allreduce(vs, dist.ReduceOp.SUM if world > 1 else None)
        known = KNOWN_NNZC.get(args.scale)
        gold = reference_digest(args.scale, args.edgefactor)
        check = {"nnzC": int(nnz_all), "expected_nnzC": known, "value_sum": vsum,
                 "expected_value_sum": float(closed_sum), "digest": str(dg) if dg is not None else None,
                 "reference_digest": gold}
        check["ok"] = bool((known is None or int(nnz_all) == known) and vsum == float(closed_sum)
                           and (dg is None or gold is None or str(dg) == gold))

    merge = None
    if world == 1 and not args.no_merge:
        del dA, dB
        ctx.close()  # releases the phase workspace before the merge sample allocates its own
        log("MultiwayMerge sample")
        merge = merge_measurement(cb.rmat(args.scale, args.edgefactor, dtype=np.float64), args.merge_cols_frac, 3)
    if rank == 0:
        base = None
        if world == 1 and not args.no_cpu_baseline:
            log("CPU baseline (reference harness on a column sample)")
            base = cpu_baseline(args.scale, args.edgefactor, args.cpu_cols_frac)
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "GFLOP/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: packed Graph500 R-MAT (seed 0xDECAFBAD), bit-identical to the reference generator",
            "config": {"workload": f"rmat{args.scale}_ef{args.edgefactor}_AxA_PlusTimes_f64", "scale": args.scale,
                       "edgefactor": args.edgefactor, "nnzA": nnzA, "flops": int(flops), "nnzC": int(nnzC),
                       "phases": st["phases"], "parallelism": parallelism, "cpp_fallback": cpp_fallback,
                       "kernel_ms": {n: round(v["ms"] / max(args.steps, 1), 3) for n, v in ks.items()}},
            "roofline": roofline, "cpu_baseline": base, "check": check, "merge": merge,
        }
        print(json.dumps(out), flush=True)
    barrier()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
