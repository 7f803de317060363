"""GPU probe of cbh_mat_col_concat_consume's peak near HBM capacity (C5's 148 GB of pruned pieces):
k uninitialised pieces of the given total size beside a ballast block, then the consuming
concatenation, printing the allocator and device memory at each step.
    python tools/concat_mem_probe.py [total_GB=148] [pieces=5] [ballast_GB=18]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402  (torch's HIP runtime initialises first, as in the library's Context)

torch.cuda.init()
from combblas_amd._lib import check, lib  # noqa: E402

CBH_F64 = 0  # include/combblas_hip.h cbh_dtype

L = lib()
total_gb = float(sys.argv[1]) if len(sys.argv) > 1 else 148.0
k = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ballast_gb = float(sys.argv[3]) if len(sys.argv) > 3 else 18.0
ctx = ctypes.c_void_p()
check(L.cbh_ctx_create(0, ctypes.byref(ctx)))


def mem(tag):
    v = [ctypes.c_int64() for _ in range(4)]
    check(L.cbh_ctx_memory(ctx, *[ctypes.byref(x) for x in v]), ctx)
    print(f"{tag:28s} live {v[0].value / 1e9:7.2f} GB  cached {v[1].value / 1e9:7.2f} GB  "
          f"device free {v[2].value / 1e9:7.2f} of {v[3].value / 1e9:.2f} GB", flush=True)


def mat(nnz, nzc=1):
    h = ctypes.c_void_p()
    check(L.cbh_mat_create(ctx, 1 << 20, nzc, nnz, nzc, CBH_F64, 8, ctypes.byref(h)), ctx)
    return h.value


mem("start")
ballast = mat(int(ballast_gb * 1e9 / 12))
per = int(total_gb * 1e9 / 12 / k)
parts = (ctypes.c_void_p * k)(*[mat(per) for _ in range(k)])
check(L.cbh_ctx_synchronize(ctx), ctx)
mem(f"{k} pieces + ballast")
out = ctypes.c_void_p()
rc = L.cbh_mat_col_concat_consume(ctx, k, parts, ctypes.byref(out))
print("consume rc", rc, L.cbh_last_error(ctx).decode(), flush=True)
mem("after concat")
