"""Builds the in-tree HIP library combblas_amd/libcombblas_hip.so for gfx950.

Plain `hipcc` (no cmake, no JIT cache): the resulting .so lives next to this file so that it
travels with the repository snapshot to the GPU box and is the library the tests load.
"""
from __future__ import annotations

import os
import re
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libcombblas_hip.so")
SOURCES = ["spgemm.hip", "rmat.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("CBH_OFFLOAD_ARCH", "gfx950")


def _deps() -> list:
    """the sources and every header they reach through #include "..." (quoted includes only)"""
    seen, todo = set(), [os.path.join(CSRC, f) for f in SOURCES]
    while todo:
        f = os.path.normpath(todo.pop())
        if f in seen or not os.path.exists(f):
            continue
        seen.add(f)
        with open(f, errors="replace") as fh:
            for line in fh:
                m = _INC.match(line)
                if m:
                    todo.append(os.path.join(os.path.dirname(f), m.group(1)))
    return sorted(seen)


_INC = re.compile(r'\s*#\s*include\s+"([^"]+)"')


def _stale(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(d) > t for d in _deps())


def build(force: bool = False, verbose: bool = False, stamps: bool = False, variant: str = "",
          defines: tuple = ()) -> str:
    """stamps=True builds the diagnostic variant libcombblas_hip_stamps.so (-DCBH_STAMPS: per-phase
    s_memtime cycle counts, printed with CBH_DIAG=1; load it with CBH_LIB=stamps). variant/defines
    build other diagnostic variants (e.g. variant="abl1", defines=("CBH_ABL=1",): kernel-phase
    ablations) as libcombblas_hip_<variant>.so, loaded with CBH_LIB=<variant>. Never the product."""
    if stamps:
        variant, defines = "stamps", tuple(defines) + ("CBH_STAMPS",)
    lib = LIB.replace(".so", f"_{variant}.so") if variant else LIB
    if not force and not _stale(lib):
        return lib
    # -ffp-contract=off: no a*b+c fused into one rounding -- the reference's host build (g++, x86-64
    # without FMA) rounds every product and every sum, and the reference-order pass reproduces it bit for bit
    cmd = [HIPCC, "-O3", "-ffp-contract=off", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-std=c++17", "-Wall",
           "-Wno-unused-function", "-Wl,-soname," + os.path.basename(lib), "-o", lib + ".tmp"] + \
        [f"-D{d}" for d in defines] + [os.path.join(CSRC, s) for s in SOURCES] + ["-lpthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    import sys

    args = sys.argv[1:]
    if "--variant" in args:  # --variant NAME DEF [DEF ...]
        k = args.index("--variant")
        print(build(force=True, verbose=True, variant=args[k + 1], defines=tuple(args[k + 2:])))
    else:
        print(build(force=True, verbose=True, stamps="--stamps" in args))
