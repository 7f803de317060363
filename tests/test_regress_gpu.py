"""GPU regression tests for the device faults of round 2 and the retry path of the hash kernel
("What's weak" 2):

1. A large numeric HASH sub-tile that overflows must be retried with half its row range from the
   cursors BEFORE it (round 2 faulted on a retry that read cursors the segment scan had already
   moved). (a) The probe limit: K = 2000 consecutive rows plus one row at the end of a 10^7-row
   span -> one task of K + 1 outputs (the large hash bin: > 1024 outputs), and the order-preserving
   slot map (row - lo) * T / span puts the K rows on one home slot: the probe chain passes
   kPmax = 64 and the sub-tile is halved until its rows spread. (b) task_kernel's commit queue
   (WIN = U * BS entries < the T + 64 slots, cbh_hash_config): a sub-tile that inserts without a
   probe overflow but occupies more slots than the queue holds (K = WIN + 4 rows 128*m plus one row
   at 3*X - 1, X = 128*K: R = 3 sub-tiles of X rows, the first with K occupied slots, at most 2 rows
   per home slot). The retry counter (cbh_ctx_take_retries) must see both. Variants: the
   column's products from ONE B entry (cursors in LDS) and from 600 / 1200 B entries (chunked,
   cursors double-buffered in HBM); f64 and int64 values. (b) is skipped for a kernel whose queue
   holds every slot (dense_kernel.h KHASH, built with CBH_HASH_V2=1).
2. The TC dot-form piece kernels are wave-strided with a capped grid (an AQL dispatch counts
   work-items in 32 bits; scale 22 overflowed the direct grid, fixed in 2b52875). The test-only
   CBH_TEST_GRID_CAP lowers the cap to 1 block (4 waves) so that scale 12/14 runs many strides
   per wave; the result must equal the reference's C (tests/golden/tc.json digests).
"""
import json
import os

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu

K_CLUSTER = 2000  # > the mid bin's 1024 outputs: the task runs the large hash kernel


def _probe_overflow_operands(nentries, dtype, seed):
    import ctypes

    from combblas_amd._lib import lib

    T, bs, u = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    lib().cbh_hash_config(ctypes.byref(T), ctypes.byref(bs), ctypes.byref(u))
    assert T.value >= 1024, T.value
    rng = np.random.default_rng(seed)
    m = 10_000_000
    rows = np.concatenate([np.arange(K_CLUSTER, dtype=np.int64), [m - 1]])
    owner = np.concatenate([np.arange(K_CLUSTER) % nentries, [nentries - 1]])  # A column of each row
    order = np.lexsort((rows, owner))
    rows, owner = rows[order], owner[order]
    vals = rng.integers(1, 9, rows.size).astype(dtype) * (1 if dtype == np.int64 else 0.5)
    cp = np.searchsorted(owner, np.arange(nentries + 1)).astype(np.int64)
    A = H.Dcsc(m, nentries, np.arange(nentries, dtype=np.int64), cp, rows.astype(np.int32), vals.astype(dtype))
    bv = rng.integers(1, 5, nentries).astype(dtype) * (1 if dtype == np.int64 else 0.25)
    B = H.Dcsc(nentries, 1, np.zeros(1, np.int64), np.array([0, nentries], np.int64),
               np.arange(nentries, dtype=np.int32), bv.astype(dtype))
    return A, B


@pytest.mark.parametrize("nentries", [1, 1200])
@pytest.mark.parametrize("dtype", [np.float64, np.int64])
def test_hash_probe_overflow_retry(ctx, oracle, nentries, dtype):
    import combblas_amd as cb

    A, B = _probe_overflow_operands(nentries, dtype, 7 + nentries)
    dA = cb.SpDCCols.from_host(ctx, cb.HostDcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))
    dB = cb.SpDCCols.from_host(ctx, cb.HostDcsc(B.m, B.n, B.jc, B.cp, B.ir, B.num))
    ctx.take_retries()  # reset the device retry counter
    C = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dA, dB)
    retries = ctx.take_retries()
    h = C.to_host()
    got = H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num)
    exp = oracle.spgemm(A, B, "plus_times", "hybrid")
    assert exp.nnz == K_CLUSTER + 1
    H.assert_dcsc_equal(got, exp, msg=f"probe overflow, {nentries} B entries, {np.dtype(dtype).name}")
    # the retry path fired: the clustered sub-tile was redone with half its rows until they spread
    assert retries >= 1, "the probe overflow did not trigger a sub-tile retry"
    for S in (C, dA, dB):
        S.free()


def _queue_rows():
    """K = the commit queue + 4 (see the module docstring), from the library's configuration"""
    import ctypes

    from combblas_amd._lib import lib

    T, bs, u = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    lib().cbh_hash_config(ctypes.byref(T), ctypes.byref(bs), ctypes.byref(u))
    if bs.value == 1024:  # the KHASH kernel (CBH_HASH_V2=1): its commit queue holds every slot
        pytest.skip("the shipped hash kernel's commit queue holds every slot")
    K = bs.value * u.value + 4
    assert K <= T.value + 64 and -(-(K + 1) // (T.value // 2)) == 3, (T.value, bs.value, u.value)
    return K


def _queue_overflow_operands(nentries, dtype, seed):
    rng = np.random.default_rng(seed)
    K = _queue_rows()
    X = 128 * K  # rows of the first hash sub-tile
    m = 3 * X
    rows = np.concatenate([np.arange(K, dtype=np.int64) * 128, [m - 1]])
    owner = np.concatenate([np.arange(K) % nentries, [nentries - 1]])  # A column of each row
    order = np.lexsort((rows, owner))
    rows, owner = rows[order], owner[order]
    vals = rng.integers(1, 9, rows.size).astype(dtype) * (1 if dtype == np.int64 else 0.5)
    cp = np.searchsorted(owner, np.arange(nentries + 1)).astype(np.int64)
    A = H.Dcsc(m, nentries, np.arange(nentries, dtype=np.int64), cp, rows.astype(np.int32), vals.astype(dtype))
    bv = rng.integers(1, 5, nentries).astype(dtype) * (1 if dtype == np.int64 else 0.25)
    B = H.Dcsc(nentries, 1, np.zeros(1, np.int64), np.array([0, nentries], np.int64),
               np.arange(nentries, dtype=np.int32), bv.astype(dtype))
    return A, B


@pytest.mark.parametrize("nentries", [1, 600])
@pytest.mark.parametrize("dtype", [np.float64, np.int64])
def test_hash_commit_queue_only_overflow(ctx, oracle, nentries, dtype):
    import combblas_amd as cb

    A, B = _queue_overflow_operands(nentries, dtype, 7 + nentries)
    dA = cb.SpDCCols.from_host(ctx, cb.HostDcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))
    dB = cb.SpDCCols.from_host(ctx, cb.HostDcsc(B.m, B.n, B.jc, B.cp, B.ir, B.num))
    ctx.take_retries()  # reset the device retry counter
    C = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dA, dB)
    retries = ctx.take_retries()
    h = C.to_host()
    got = H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num)
    exp = oracle.spgemm(A, B, "plus_times", "hybrid")
    assert exp.nnz == _queue_rows() + 1
    H.assert_dcsc_equal(got, exp, msg=f"queue-only overflow, {nentries} B entries, {np.dtype(dtype).name}")
    # the retry path fired: the first sub-tile (K occupied slots > the K - 4 queue entries) was
    # redone with half its rows
    assert retries >= 1, "the commit-queue overflow did not trigger a sub-tile retry"
    for S in (C, dA, dB):
        S.free()


@pytest.mark.parametrize("scale", [12, 14])
@pytest.mark.parametrize("hub", [None, "1"])
def test_tc_dot_grid_cap_strides(ctx, scale, hub, monkeypatch):
    from combblas_amd.apps import MaskedSpGEMM, TCLower
    from combblas_amd.semirings import PlusTimesSRing

    with open(os.path.join(H.GOLDEN, "tc.json")) as f:
        ref = json.load(f)["scales"][str(scale)]
    monkeypatch.setenv("CBH_TEST_GRID_CAP", "1")  # 4 waves stride over every piece
    if hub is not None:  # every binary-search entry in a hub group: one workgroup strides over them
        monkeypatch.setenv("CBH_DOT_HUB_MIN", hub)
    L, L2 = TCLower(ctx, scale), TCLower(ctx, scale)
    C = MaskedSpGEMM(PlusTimesSRing, L, L2, L, method="dot")
    h = C.to_host()
    c = H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num)
    vs, dg = H.digest(c)
    assert (c.nnz, c.nzc) == (ref["nnzC"], ref["nzcC"])
    assert int(c.num.sum()) == ref["triangles"] and vs == ref["sumC"] and dg == int(ref["digestC"])
    for S in (C, L, L2):
        S.free()


def _wave_overflow_operands(dtype, seed):
    """Small tasks (<= 256 outputs: the one-task-per-wave kernel) whose rows cluster: 202 rows, 200
    of them consecutive, over a 10^6-row span (an order-preserving slot map would put the 200 rows
    on one home slot; the wave kernel's key hash and counting commit must order them)."""
    rng = np.random.default_rng(seed)
    m, n = 1_000_000, 60
    cols, rows = [], []
    for c in range(n):
        if c % 3 == 0:
            r = np.concatenate([[0], 500_000 + 300 * c + np.arange(200), [m - 1]])
        else:
            r = np.sort(rng.choice(m, 40, replace=False))
        rows.append(r)
        cols.append(np.full(r.size, c))
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    cp = np.searchsorted(cols, np.arange(n + 1)).astype(np.int64)
    av = rng.integers(1, 9, rows.size).astype(dtype) * (1 if dtype == np.int64 else 0.5)
    A = H.Dcsc(m, n, np.arange(n, dtype=np.int64), cp, rows.astype(np.int32), av)
    nb = n // 2
    bv = rng.integers(1, 5, n).astype(dtype) * (1 if dtype == np.int64 else 0.25)
    B = H.Dcsc(n, nb, np.arange(nb, dtype=np.int64), np.arange(0, n + 1, 2, dtype=np.int64),
               np.arange(n, dtype=np.int32), bv)
    return A, B


@pytest.mark.parametrize("dtype", [np.float64, np.int64])
def test_wave_clustered_rows(ctx, oracle, dtype):
    import combblas_amd as cb

    A, B = _wave_overflow_operands(dtype, 5)
    dA = cb.SpDCCols.from_host(ctx, cb.HostDcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))
    dB = cb.SpDCCols.from_host(ctx, cb.HostDcsc(B.m, B.n, B.jc, B.cp, B.ir, B.num))
    C = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dA, dB)
    h = C.to_host()
    got = H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num)
    exp = oracle.spgemm(A, B, "plus_times", "hybrid")
    assert np.diff(exp.cp).max() <= 256  # every column is a small (wave) task
    H.assert_dcsc_equal(got, exp, msg=f"wave clustered rows, {np.dtype(dtype).name}")
    for S in (C, dA, dB):
        S.free()


@pytest.mark.parametrize("dtype", [np.float64, np.int64])
def test_high_cr_short_columns_leave_the_wave_kernel(ctx, oracle, dtype):
    """Columns with few outputs but many products (compression ratio 100: 64 output rows, 10,240
    products) are routed by their ratio to the mid workgroup kernel (dense_split_kernel,
    kWaveProducts); every other column of the product stays on the wave kernel. Checked against
    the oracle."""
    import combblas_amd as cb

    rng = np.random.default_rng(3)
    m, n = 4096, 400
    rows, cols = [], []
    for c in range(n):
        r = np.sort(rng.choice(64, 64, replace=False)) * 61 if c < 160 else np.sort(rng.choice(m, 12, replace=False))
        rows.append(r)
        cols.append(np.full(r.size, c))
    rows, cols = np.concatenate(rows), np.concatenate(cols)
    cp = np.searchsorted(cols, np.arange(n + 1)).astype(np.int64)
    av = rng.integers(1, 9, rows.size).astype(dtype) * (1 if dtype == np.int64 else 0.5)
    A = H.Dcsc(m, n, np.arange(n, dtype=np.int64), cp, rows.astype(np.int32), av)
    # B column 0: all 160 "cluster" columns of A (160 x 64 products onto 64 rows); the rest sparse
    bcols = [np.arange(160)] + [np.sort(rng.choice(np.arange(160, n), 5, replace=False)) for _ in range(63)]
    bcp = np.concatenate([[0], np.cumsum([b.size for b in bcols])]).astype(np.int64)
    bv = rng.integers(1, 5, int(bcp[-1])).astype(dtype) * (1 if dtype == np.int64 else 0.25)
    B = H.Dcsc(n, 64, np.arange(64, dtype=np.int64), bcp, np.concatenate(bcols).astype(np.int32), bv)
    dA = cb.SpDCCols.from_host(ctx, cb.HostDcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num))
    dB = cb.SpDCCols.from_host(ctx, cb.HostDcsc(B.m, B.n, B.jc, B.cp, B.ir, B.num))
    C = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dA, dB)
    h = C.to_host()
    got = H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num)
    exp = oracle.spgemm(A, B, "plus_times", "hybrid")
    assert exp.cp[1] - exp.cp[0] == 64  # 10,240 products onto 64 rows
    H.assert_dcsc_equal(got, exp, msg=f"high-cr short column, {np.dtype(dtype).name}")
    for S in (C, dA, dB):
        S.free()
