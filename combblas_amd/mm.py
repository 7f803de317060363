"""Matrix Market I/O of local blocks.

  mmread / ReadMM    SpParMat::ParallelReadMM (SpParMat.cpp:3978-4126): coordinate banner
                     (real | integer | pattern, general | symmetric), one-based indices by default,
                     pattern entries valued 1, symmetric files expanded with (j, i) for i != j,
                     duplicates combined with the default SumOp. A file without a banner is read as
                     "coordinate real general" (the reference's ReleaseTests/small_nonsym.mtx).
  WriteMM            SpParMat::ParallelWriteMM (SpParMat.cpp:4128-4230): banner, dimensions, then
                     one "row col value" line per entry in column-major order.

Text parsing runs on the host (files are read once); the tuples go to HBM and ReadMM builds the
DCSC block on the device (cbh_tuples_to_dcsc: radix sort + duplicate sum + column heads), so the
SpTuples -> SpDCCols conversion never runs on the CPU.
"""
from __future__ import annotations

import io

import numpy as np

from .spdccols import Context, SpDCCols


def _banner(first: str):
    t = first.lower().split()
    if not t or not t[0].startswith("%%matrixmarket"):
        return None
    if len(t) < 5 or t[1] != "matrix" or t[2] != "coordinate":
        raise ValueError(f"unsupported Matrix Market banner: {first.strip()}")
    if t[3] not in ("real", "integer", "pattern") or t[4] not in ("general", "symmetric"):
        raise ValueError(f"unsupported Matrix Market field/symmetry: {first.strip()}")
    return t[3], t[4]


def mmread(path, onebased=True, expand_symmetric=True):
    """-> (m, n, rows int64, cols int64, vals ndarray, field, symmetry); entries in file order
    (plus the mirrored entries of a symmetric file), duplicates not yet combined."""
    with open(path) as f:
        text = f.read()
    lines = text.splitlines()
    ban = _banner(lines[0]) if lines else None
    field, sym = ban if ban else ("real", "general")
    body = [ln for ln in lines if ln.strip() and not ln.lstrip().startswith("%")]
    m, n, nnz = (int(x) for x in body[0].split()[:3])
    ncol = 2 if field == "pattern" else 3
    data = np.loadtxt(io.StringIO("\n".join(body[1:1 + nnz])), ndmin=2) if nnz else np.zeros((0, ncol))
    if data.shape[0] != nnz:
        raise ValueError(f"{path}: {data.shape[0]} entries, banner says {nnz}")
    rows = data[:, 0].astype(np.int64) - (1 if onebased else 0)
    cols = data[:, 1].astype(np.int64) - (1 if onebased else 0)
    if field == "pattern" or data.shape[1] < 3:
        vals = np.ones(nnz, np.float64)
    elif field == "integer":
        vals = data[:, 2].astype(np.int64)
    else:
        vals = data[:, 2].astype(np.float64)
    if sym == "symmetric" and expand_symmetric:
        off = rows != cols
        rows, cols, vals = (np.concatenate([rows, cols[off]]), np.concatenate([cols, rows[off]]),
                            np.concatenate([vals, vals[off]]))
    if nnz and (rows.min() < 0 or cols.min() < 0 or rows.max() >= m or cols.max() >= n):
        raise ValueError(f"{path}: index out of range for a {m} x {n} matrix")
    return m, n, rows, cols, vals, field, sym


def ReadMM(ctx: Context, path, onebased=True, removeloops=False, dtype=None, expand_symmetric=True) -> SpDCCols:
    """A Matrix Market file as a device DCSC block (tuples -> DCSC on the gfx950 kernels)."""
    import torch

    m, n, rows, cols, vals, _, _ = mmread(path, onebased, expand_symmetric)
    if dtype is not None:
        vals = vals.astype(dtype)
    dev = ctx.tdevice or torch.device("cuda", ctx.device)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    return SpDCCols.from_tuples(ctx, m, n, t(rows.astype(np.int32)), t(cols), t(vals), removeloops=removeloops)


def WriteMM(path, M: SpDCCols, onebased=True):
    """ParallelWriteMM for one block: entries column-major, rows ascending within a column."""
    r, c, v = (x.cpu().numpy() for x in M.to_tuples())
    integer = np.issubdtype(v.dtype, np.integer)
    with open(path, "w") as f:
        f.write(f"%%MatrixMarket matrix coordinate {'integer' if integer else 'real'} general\n")
        f.write(f"{M.m}\t{M.n}\t{M.nnz}\n")
        o = 1 if onebased else 0
        fmt = "%d\t%d\t%d" if integer else "%d\t%d\t%.17g"
        if M.nnz:
            cols3 = [r.astype(np.int64) + o, c + o, v.astype(np.int64) if integer else v.astype(np.float64)]
            np.savetxt(f, np.column_stack(cols3), fmt=fmt)
