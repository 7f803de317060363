#!/usr/bin/env python3
"""Dev tool: timing of TC's masked (L*L) .* L on the device (dot form) over R-MAT scales.
    python tools/tc_timing.py 16 18 20 22 24
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import combblas_amd as cb
    from combblas_amd.apps import MaskedSpGEMM, TCLower
    from combblas_amd.semirings import PlusTimesSRing

    ctx = cb.Context(0)
    for s in [int(x) for x in sys.argv[1:]]:
        t0 = time.perf_counter()
        L = TCLower(ctx, s)
        L2 = TCLower(ctx, s)
        ctx.synchronize()
        t1 = time.perf_counter()
        for rep in range(2):
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            C = MaskedSpGEMM(PlusTimesSRing, L, L2, L, method="dot")
            ctx.synchronize()
            t3 = time.perf_counter()
            tri = int(C.tensors()[3].sum().item())
            print(f"scale {s}: nnzL {L.nnz} build {t1 - t0:.2f} s; masked dot {1e3 * (t3 - t2):.1f} ms (rep {rep}); "
                  f"nnzC {C.nnz} triangles {tri}", flush=True)
            C.free()
        L.free()
        L2.free()
        ctx.trim()
    ctx.close()


if __name__ == "__main__":
    main()
