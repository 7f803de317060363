"""Inputs of BASELINE.json config C3 (Galerkin triple product RᵀAR, ReleaseTests/GalerkinNew.cpp).

The reference reads its operators from files; the config names the 27-point Poisson operator on
a 256³ grid and trilinear full-weighting prolongation, so these host generators build them:
  poisson27(nx)     n = nx³ rows, 26 on the diagonal, -1 for each of the (up to) 26 neighbours
  prolongation(nx)  T: fine nx³ x coarse (nx/2)³; fine index f = 2c -> weight 1 from coarse c,
                    f = 2c+1 -> 1/2 from c and c+1 (where c+1 exists); 3-D weights are products
                    (1, 1/2, 1/4, 1/8). All values are dyadic, so every f64 sum of the triple
                    product is exact and the result is bit-identical under any summation order.
GalerkinNew.cpp:100-106 then forms S = Tᵀ, AT = PSpGEMM(A, T), SAT = PSpGEMM(S, AT).
"""
from __future__ import annotations

import numpy as np

from .spdccols import HostDcsc


def _from_coo(m, n, rows, cols, vals) -> HostDcsc:
    o = np.lexsort((rows, cols))
    rows, cols, vals = rows[o], cols[o], vals[o]
    colptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(cols, minlength=n), out=colptr[1:])
    return HostDcsc.from_csc(m, n, colptr, rows.astype(np.int32), vals.astype(np.float64))


def poisson27(nx: int) -> HostDcsc:
    g = np.arange(nx)
    x, y, z = np.meshgrid(g, g, g, indexing="ij")
    x, y, z = x.ravel(), y.ravel(), z.ravel()
    idx = (x * nx + y) * nx + z
    rows, cols, vals = [], [], []
    for dx in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dz in (-1, 0, 1):
                ok = (x + dx >= 0) & (x + dx < nx) & (y + dy >= 0) & (y + dy < nx) & (z + dz >= 0) & (z + dz < nx)
                nb = ((x + dx) * nx + (y + dy)) * nx + (z + dz)
                rows.append(idx[ok])
                cols.append(nb[ok])
                vals.append(np.full(ok.sum(), 26.0 if (dx, dy, dz) == (0, 0, 0) else -1.0))
    n = nx ** 3
    return _from_coo(n, n, np.concatenate(rows), np.concatenate(cols), np.concatenate(vals))


def _prolong_1d(nx):
    nc = nx // 2
    f, c, w = [], [], []
    for i in range(nx):
        if i % 2 == 0:
            f.append(i), c.append(i // 2), w.append(1.0)
        else:
            f.append(i), c.append(i // 2), w.append(0.5)
            if i // 2 + 1 < nc:
                f.append(i), c.append(i // 2 + 1), w.append(0.5)
    return np.array(f), np.array(c), np.array(w), nc


def prolongation(nx: int) -> HostDcsc:
    f1, c1, w1, nc = _prolong_1d(nx)
    k = np.arange(f1.size)
    a, b, d = np.meshgrid(k, k, k, indexing="ij")
    a, b, d = a.ravel(), b.ravel(), d.ravel()
    rows = (f1[a] * nx + f1[b]) * nx + f1[d]
    cols = (c1[a] * nc + c1[b]) * nc + c1[d]
    vals = w1[a] * w1[b] * w1[d]
    return _from_coo(nx ** 3, nc ** 3, rows, cols, vals)


def _offsets_1d(nx):
    """per 1-D grid point: its 3 stencil neighbours (-1, 0, +1) and whether each exists"""
    g = np.arange(nx, dtype=np.int64)
    nb = g[:, None] + np.array([-1, 0, 1])[None, :]
    return nb, (nb >= 0) & (nb < nx)


def poisson27_csc(nx: int) -> HostDcsc:
    """poisson27(nx) built straight in column order (no sort): column c's rows are its stencil
    neighbours, and (dx, dy, dz) in lexicographic order gives ascending row ids -- for the 256^3
    operator of config C3 (449 M entries) in seconds"""
    nb, ok = _offsets_1d(nx)
    n = nx ** 3
    # neighbour ids / validity per (column, 27 offsets): separable in x, y, z
    x = nb[:, None, None, :, None, None] * nx * nx + nb[None, :, None, None, :, None] * nx + nb[None, None, :, None, None, :]
    v = ok[:, None, None, :, None, None] & ok[None, :, None, None, :, None] & ok[None, None, :, None, None, :]
    x = x.reshape(n, 27)
    v = v.reshape(n, 27)
    rows = x[v].astype(np.int32)
    counts = v.sum(axis=1)
    colptr = np.zeros(n + 1, np.int64)
    np.cumsum(counts, out=colptr[1:])
    vals = np.where(np.broadcast_to(np.arange(27) == 13, v.shape)[v], 26.0, -1.0)
    return HostDcsc.from_csc(n, n, colptr, rows, vals)


def prolongation_csc(nx: int) -> HostDcsc:
    """prolongation(nx) built straight in column order: coarse column j of the 1-D operator has
    fine rows 2j-1 (weight 1/2, when j >= 1), 2j (1) and 2j+1 (1/2); 3-D columns are products"""
    nc = nx // 2
    j = np.arange(nc, dtype=np.int64)
    f = np.stack([2 * j - 1, 2 * j, 2 * j + 1], axis=1)
    w = np.broadcast_to(np.array([0.5, 1.0, 0.5]), f.shape)
    ok = f >= 0
    rows = f[:, None, None, :, None, None] * nx * nx + f[None, :, None, None, :, None] * nx + f[None, None, :, None, None, :]
    val = w[:, None, None, :, None, None] * w[None, :, None, None, :, None] * w[None, None, :, None, None, :]
    v = ok[:, None, None, :, None, None] & ok[None, :, None, None, :, None] & ok[None, None, :, None, None, :]
    m = nc ** 3
    rows, val, v = rows.reshape(m, 27), val.reshape(m, 27), v.reshape(m, 27)
    colptr = np.zeros(m + 1, np.int64)
    np.cumsum(v.sum(axis=1), out=colptr[1:])
    return HostDcsc.from_csc(nx ** 3, m, colptr, rows[v].astype(np.int32), val[v].astype(np.float64))


def transpose(h: HostDcsc) -> HostDcsc:
    """host transpose (SpParMat::Transpose for the test inputs)"""
    cols = np.repeat(h.jc, np.diff(h.cp))
    return _from_coo(h.n, h.m, cols, h.ir.astype(np.int64), h.num)
