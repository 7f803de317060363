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


def cluster_sizes(n: int, rng, alpha: float = 1.6) -> np.ndarray:
    """power-law cluster sizes 2 + floor(6 * Pareto(alpha)) summing to n (vectorised batches of the
    draw planted_partition makes one at a time)"""
    out, total = [], 0
    while total < n:
        s = np.minimum(n, 2 + np.floor(rng.pareto(alpha, max(1024, (n - total) // 8)) * 6)).astype(np.int64)
        c = np.cumsum(s)
        k = int(np.searchsorted(c, n - total))  # first batch index whose running sum reaches the rest
        if k < s.size:
            s = s[:k + 1]
        out.append(s)
        total += int(s.sum())
    sizes = np.concatenate(out)
    sizes[-1] -= int(sizes.sum()) - n
    return sizes[sizes > 0]


def planted_partition_coo(n: int, avg_deg: int = 100, seed: int = 7, p_in: float = 0.9, alpha: float = 1.6,
                          device="cuda", chunk: int = 1 << 27):
    """COO (rows int64, cols int64, vals f64 torch tensors on `device`) of planted_partition's
    recipe drawn with the torch RNG seeded with `seed` (cluster sizes and the vertex permutation
    from numpy): avg_deg/2 draws per vertex, a fraction p_in inside its cluster, symmetric, uniform
    (0, 1] weights, unit self loops, every column divided by its sum (MakeColStochastic,
    MCL.cpp:390-396). Entries are distinct. Not bit-identical to planted_partition (other RNG
    streams)."""
    import torch

    dev = torch.device(device)
    rng = np.random.default_rng(seed)
    sizes = cluster_sizes(n, rng, alpha)
    start = torch.as_tensor(np.concatenate([[0], np.cumsum(sizes)[:-1]]), device=dev)
    szs = torch.as_tensor(sizes, device=dev)
    perm = torch.as_tensor(rng.permutation(n), device=dev)
    cl = torch.repeat_interleave(torch.arange(sizes.size, device=dev), szs)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    half = max(1, avg_deg // 2)
    draws = n * half
    keys = []
    for d0 in range(0, draws, chunk):
        d1 = min(draws, d0 + chunk)
        v = torch.arange(d0, d1, device=dev, dtype=torch.int64) // half
        c = cl[v]
        inside = torch.rand(d1 - d0, device=dev, generator=g) < p_in
        u_in = start[c] + (torch.rand(d1 - d0, device=dev, generator=g, dtype=torch.float64) * szs[c]).long()
        u_out = torch.randint(0, n, (d1 - d0,), device=dev, generator=g)
        u = torch.where(inside, u_in, u_out)
        a, b = perm[v], perm[u]
        del v, c, inside, u_in, u_out, u
        k = torch.minimum(a, b) * n + torch.maximum(a, b)
        keys.append(torch.unique(k[a != b]))
        del a, b, k
    key = torch.unique(torch.cat(keys))
    del keys
    w = 1.0 - torch.rand(key.numel(), device=dev, generator=g, dtype=torch.float64)  # (0, 1]
    lo, hi = key // n, key % n
    del key
    diag = torch.arange(n, device=dev, dtype=torch.int64)
    rows = torch.cat([lo, hi, diag])
    cols = torch.cat([hi, lo, diag])
    del lo, hi
    vals = torch.cat([w, w, torch.ones(n, device=dev, dtype=torch.float64)])
    del w
    colsum = torch.zeros(n, device=dev, dtype=torch.float64).index_add_(0, cols, vals)
    vals /= colsum[cols]
    return rows, cols, vals


def planted_partition_device(ctx, n: int, avg_deg: int = 100, seed: int = 7, p_in: float = 0.9,
                             alpha: float = 1.6):
    """planted_partition_coo on ctx's GPU, built into a device SpDCCols (f64) by the library's
    tuple sort (cbh_tuples_to_dcsc): n = 2^24 (config C5's size) in seconds"""
    import torch

    from .spdccols import SpDCCols

    rows, cols, vals = planted_partition_coo(n, avg_deg, seed, p_in, alpha, device=f"cuda:{ctx.device}")
    M = SpDCCols.from_tuples(ctx, n, n, rows.to(torch.int32), cols, vals)
    del rows, cols, vals
    torch.cuda.synchronize(ctx.device)
    return M


def planted_partition_lib(ctx, n: int, avg_deg: int = 100, seed: int = 7, p_in: float = 0.9, alpha: float = 1.6):
    """the same recipe generated by the library (cbh_gen_planted_partition, csrc/mclgen.h): counter-based
    draws, so the matrix depends on the arguments only -- the input the C++ C5 harness
    (tests/dropin/mclbench_harness.cpp) builds too. Returns a device SpDCCols (f64)."""
    import ctypes

    from ._lib import check, lib
    from .spdccols import SpDCCols

    h = ctypes.c_void_p()
    check(lib().cbh_gen_planted_partition(ctx.h, int(n), int(avg_deg), int(seed), float(p_in), float(alpha),
                                          ctypes.byref(h)), ctx.h)
    return SpDCCols(ctx, h)
