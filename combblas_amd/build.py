"""Builds the in-tree HIP library combblas_amd/libcombblas_hip.so for gfx950.

Plain `hipcc` (no cmake, no JIT cache): the resulting .so lives next to this file so that it
travels with the repository snapshot to the GPU box and is the library the tests load.
"""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libcombblas_hip.so")
SOURCES = ["spgemm.hip", "rmat.cpp"]
HEADERS = ["semiring.h", "tile_kernel.h", "host_util.h", os.path.join("..", "..", "include", "combblas_hip.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("CBH_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    cmd = [HIPCC, "-O3", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-std=c++17", "-Wall",
           "-Wno-unused-function", "-Wl,-soname,libcombblas_hip.so", "-o", LIB + ".tmp"] + [os.path.join(CSRC, s) for s in SOURCES] + ["-lpthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
