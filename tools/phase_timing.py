"""Dev tool: host wall time of consecutive phased products, and a check that the inputs are
left untouched by every call (GPU box)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import combblas_amd as cb

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 4
A = cb.rmat(scale, dtype=np.float64)
ctx = cb.Context(0, torch_allocator=False)
dA, dB = cb.SpDCCols.from_host(ctx, A), cb.SpDCCols.from_host(ctx, A)


def same(h):
    return (np.array_equal(h.ir, A.ir) and np.array_equal(h.cp, A.cp) and np.array_equal(h.jc, A.jc)
            and np.array_equal(h.num, A.num))


for it in range(ncalls):
    if it == 2:
        ctx.enable_timing(True)
    t = time.perf_counter()
    try:
        st = cb.PhasedSpGEMM(cb.PlusTimesSRing, dA, dB)
        ctx.synchronize()
        print(f"call {it}: {time.perf_counter() - t:.3f} s phases={st['phases']} nnz={st['nnz']}", flush=True)
    except Exception as e:
        print(f"call {it} failed: {e}", flush=True)
    print(f"  inputs intact: A {same(dA.to_host())} B {same(dB.to_host())}", flush=True)
print(ctx.kernel_stats())
