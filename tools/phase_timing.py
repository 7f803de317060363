#!/usr/bin/env python3
"""Times the phased R-MAT A^2 product NCALLS times (GPU box tool; diagnostic, not the bench).

    python tools/phase_timing.py SCALE NCALLS

Prints one "call i: <ms> ms nnz=<n>" line per call and, last, the per-kernel stats of the final
call as a dict literal (A/B scripts parse it). With CBH_LIB=stamps CBH_DIAG=1 the library
prints per-sub-bin launch times and phase cycle shares to stderr.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    # torch's bundled HIP runtime must initialise before the library's (combblas_amd.Context)
    import torch

    torch.cuda.set_device(0)
    import combblas_amd as cb

    A = cb.rmat(scale, 16, dtype=np.float64)
    ctx = cb.Context(0, torch_allocator=False)
    dA = cb.SpDCCols.from_host(ctx, A)
    dB = cb.SpDCCols.from_host(ctx, A)
    ks = {}
    nnz0 = None
    for i in range(ncalls):
        ctx.synchronize()
        ctx.enable_timing(i >= int(os.environ.get("PT_TIMING_FROM", "0")))
        ctx.reset_kernel_stats()
        t0 = time.perf_counter()
        st = cb.PhasedSpGEMM(cb.PlusTimesSRing, dA, dB)
        ctx.synchronize()
        dt = time.perf_counter() - t0
        ks = ctx.kernel_stats()
        if os.environ.get("PT_VERBOSE"):
            print({k: round(v["ms"], 1) for k, v in ks.items()}, flush=True)
        ctx.enable_timing(False)
        print(f"call {i}: {dt * 1e3:.1f} ms nnz={st['nnz']} flops={st['flops']} "
              f"GFLOP/s={2 * st['flops'] / dt / 1e9:.2f}", flush=True)
        if i == 0:
            nnz0 = st["nnz"]
        elif st["nnz"] != nnz0:  # diagnose: were the inputs overwritten by the previous call?
            for nm, d in (("A", dA), ("B", dB)):
                h = d.to_host()
                print(f"  inputs intact {nm}: {np.array_equal(h.ir, A.ir) and np.array_equal(h.cp, A.cp)}"
                      f" {np.array_equal(h.jc, A.jc) and np.array_equal(h.num, A.num)}", flush=True)
            raise SystemExit(f"call {i}: nnz {st['nnz']} != call 0's {nnz0}")
    print(repr(ks), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
