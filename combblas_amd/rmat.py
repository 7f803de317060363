"""Synthetic inputs: the deterministic packed Graph500 R-MAT generator used by every R-MAT
configuration (RefGen21.h, DistEdgeList::GenGraph500Data(packed=true), SpParMat(DEL,
removeloops)), via the C-ABI (combblas_amd/csrc/rmat.cpp). Bit-identical to the reference's
generator (pinned by tests/test_generator.py against tests/golden/golden.json).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib
from .spdccols import HostDcsc

DEFAULT_SEED = 0xDECAFBAD  # RefGen21::init_random (RefGen21.h:306-318) without SEED in the env


def rmat_edges(scale: int, edgefactor: int = 16, seed: int = DEFAULT_SEED, start=0, end=None):
    M = (1 << scale) * edgefactor
    end = M if end is None else end
    src = np.empty(end - start, np.int64)
    dst = np.empty(end - start, np.int64)
    check(lib().cbh_rmat_edges(scale, seed, start, end, src.ctypes.data, dst.ctypes.data))
    return src, dst


def rmat(scale: int, edgefactor: int = 16, seed: int = DEFAULT_SEED, removeloops: bool = False,
         dtype=np.int64) -> HostDcsc:
    """A(v0, v1) = multiplicity of edge (v0, v1); n = 2^scale. Values cast to `dtype`."""
    n = 1 << scale
    src, dst = rmat_edges(scale, edgefactor, seed)
    colptr = np.empty(n + 1, np.int64)
    rowidx = np.empty(src.size, np.int32)
    count = np.empty(src.size, np.int64)
    nnz = ctypes.c_int64()
    check(lib().cbh_edges_to_csc(n, n, src.size, src.ctypes.data, dst.ctypes.data, int(removeloops),
                                 colptr.ctypes.data, rowidx.ctypes.data, count.ctypes.data, ctypes.byref(nnz)))
    del src, dst
    k = nnz.value
    return HostDcsc.from_csc(n, n, colptr, rowidx[:k], count[:k].astype(dtype))
