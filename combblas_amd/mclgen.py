"""Protein-similarity-like synthetic input of BASELINE.json config C5 (HipMCL expansion + prune).

The reference ships no generator for it; this one follows the stated recipe:
a planted-partition graph with power-law cluster sizes, about `avg_deg` neighbours per vertex of
which a fraction `p_in` fall inside the vertex's cluster, symmetric, uniform (0, 1] weights drawn
from a fixed seed, self loops of weight 1 (HipMCL adds them before the first iteration), then
made column-stochastic as MakeColStochastic does (Applications/MCL.cpp:390-396: every column
divided by its sum). Host numpy; returns a HostDcsc with f64 values.
"""
from __future__ import annotations

import numpy as np

from .spdccols import HostDcsc


def planted_partition(n: int, avg_deg: int = 16, seed: int = 7, p_in: float = 0.9, alpha: float = 1.6) -> HostDcsc:
    rng = np.random.default_rng(seed)
    sizes = []
    while sum(sizes) < n:
        sizes.append(int(min(n, 2 + np.floor(rng.pareto(alpha) * 6))))
    sizes[-1] -= sum(sizes) - n
    sizes = np.array([s for s in sizes if s > 0], np.int64)
    start = np.concatenate([[0], np.cumsum(sizes)])
    perm = rng.permutation(n)  # cluster members are scattered over the vertex ids
    cl = np.repeat(np.arange(sizes.size), sizes)
    v = np.repeat(np.arange(n, dtype=np.int64), avg_deg // 2)
    inside = rng.random(v.size) < p_in
    c = cl[v]
    u_in = start[c] + np.floor(rng.random(v.size) * sizes[c]).astype(np.int64)
    u_out = rng.integers(0, n, v.size)
    u = np.where(inside, u_in, u_out)
    a, b = perm[v], perm[u]
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    key = np.unique(lo * n + hi)
    key = key[(key // n) != (key % n)]
    w = 1.0 - rng.random(key.size)  # (0, 1]
    r = np.concatenate([key // n, key % n, np.arange(n)])
    col = np.concatenate([key % n, key // n, np.arange(n)])
    val = np.concatenate([w, w, np.ones(n)])
    order = np.lexsort((r, col))
    r, col, val = r[order], col[order], val[order]
    colsum = np.bincount(col, weights=val, minlength=n)
    val = val / colsum[col]
    colptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(col, minlength=n), out=colptr[1:])
    return HostDcsc.from_csc(n, n, colptr, r.astype(np.int32), val)
