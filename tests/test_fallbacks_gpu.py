"""GPU tests of the driver-level fallbacks and hooks around the kernels:

* the stored dense-candidate bitmaps are sized before nnz(C) is known; when C does not fit beside
  them they are dropped and every task runs on the hash kernels (spgemm.hip new_result). The
  test-only CBH_TEST_RESULT_OOM makes the first allocation of C report an OOM while bitmaps are
  held; the product must still equal the oracle's, without any dense launch;
* count-only symbolic callers (estimateFLOPandNNZ = cbh_spgemm_symbolic, EstPerProcessNnzSUMMA)
  allocate no bitmaps: their counts equal the plan's;
* the per-phase consumer of cbh_spgemm_phased (MemEfficientSpGEMM's prune hook) sees every phase of
  a many-phase product, the concatenation of its cloned views equals the single-call product, and
  an exception raised inside it comes back out of PhasedSpGEMM.
"""
import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rmat14(oracle):
    import combblas_amd as cb

    A = cb.rmat(14)
    d = H.Dcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num)
    return d, oracle.spgemm(d, d, "plus_times", threads=8)


def _dense_launches(ctx, A, monkeypatch=None):
    import combblas_amd as cb

    h = cb.HostDcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num)
    dA, dB = cb.SpDCCols.from_host(ctx, h), cb.SpDCCols.from_host(ctx, h)
    ctx.synchronize()
    ctx.reset_kernel_stats()
    ctx.enable_timing(True)
    C = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dA, dB)
    ctx.synchronize()
    ctx.enable_timing(False)
    ks = ctx.kernel_stats()
    c = C.to_host()
    for S in (C, dA, dB):
        S.free()
    return ks["num_dense"]["launches"], H.Dcsc(c.m, c.n, c.jc, c.cp, c.ir, c.num)


def test_result_oom_drops_stored_bitmaps(ctx, rmat14, monkeypatch):
    A, exp = rmat14
    nd, got = _dense_launches(ctx, A)
    assert nd > 0, "scale-14 A^2 has no dense-window tasks: the fallback would not be exercised"
    H.assert_dcsc_equal(got, exp, msg="scale-14 A^2")
    monkeypatch.setenv("CBH_TEST_RESULT_OOM", "1")
    nd2, got2 = _dense_launches(ctx, A)
    assert nd2 == 0, "C's allocation failed beside the bitmaps, yet the dense kernel still ran"
    H.assert_dcsc_equal(got2, exp, msg="scale-14 A^2 after dropping the stored bitmaps")


def test_count_only_symbolic_matches_plan(ctx, rmat14):
    import combblas_amd as cb

    A, exp = rmat14
    h = cb.HostDcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num)
    dA, dB = cb.SpDCCols.from_host(ctx, h), cb.SpDCCols.from_host(ctx, h)
    f, z, cf, cz = cb.estimateFLOPandNNZ(dA, dB, per_column=True)
    plan = cb.SpGEMMPlan(dA, dB)
    assert plan.info() == (f, z) and z == exp.nnz
    assert bool((plan.col_nnz() == cz).all().item())
    cz = cz.cpu().numpy()  # per nonzero column of B; C drops the empty product columns
    assert np.array_equal(cz[cz > 0], np.diff(exp.cp))
    plan.close()
    dA.free()
    dB.free()


def test_phase_consumer_sees_every_phase(ctx, rmat14):
    import torch
    import combblas_amd as cb

    A, exp = rmat14
    h = cb.HostDcsc(A.m, A.n, A.jc, A.cp, A.ir, A.num)
    dA, dB = cb.SpDCCols.from_host(ctx, h), cb.SpDCCols.from_host(ctx, h)
    parts = []

    def keep(phase, s0, s1, C):
        parts.append((phase, s0, s1, C.clone()))

    budget = 12 * exp.nnz // 7  # ~7 phases of 12-byte entries
    try:
        _consumer_checks(ctx, cb, A, exp, dA, dB, parts, keep, budget)
    finally:
        ctx.set_phase_budget(0)  # the session context's default (half of free HBM)
    torch.cuda.synchronize()
    dA.free()
    dB.free()


def _consumer_checks(ctx, cb, A, exp, dA, dB, parts, keep, budget):
    st = cb.PhasedSpGEMM(cb.PlusTimesSRing, dA, dB, checksum=True, budget_bytes=budget, on_phase=keep)
    assert st["phases"] == len(parts) >= 5, (st["phases"], len(parts))
    assert [p[0] for p in parts] == list(range(len(parts)))
    assert parts[0][1] == 0 and parts[-1][2] == dB.nzc
    assert all(parts[i][2] == parts[i + 1][1] for i in range(len(parts) - 1))
    # concatenated views = the single-call product (empty columns of a view are dropped here)
    rows, vals, cols = [], [], []
    for _, _, _, C in parts:
        cp, jc, ir, num = (t.cpu().numpy() for t in C.tensors())
        counts = np.diff(cp)
        cols.append(np.repeat(jc, counts))
        rows.append(ir[:cp[-1]])
        vals.append(num[:cp[-1]])
        C.free()
    got = H.Dcsc.from_coo(A.m, A.n, np.concatenate(rows), np.concatenate(cols), np.concatenate(vals))
    H.assert_dcsc_equal(got, exp, msg="concatenated phase views")
    assert (st["value_sum"], st["digest"]) == H.digest(exp)

    class Boom(RuntimeError):
        pass

    def explode(phase, s0, s1, C):
        if phase == 2:
            raise Boom("consumer failure in phase 2")

    with pytest.raises(Boom):
        cb.PhasedSpGEMM(cb.PlusTimesSRing, dA, dB, budget_bytes=budget, on_phase=explode)
    # the context is usable afterwards
    st2 = cb.PhasedSpGEMM(cb.PlusTimesSRing, dA, dB, checksum=True, budget_bytes=budget)
    assert (st2["value_sum"], st2["digest"]) == H.digest(exp)


def test_consuming_col_concat_matches_copy(ctx):
    """cbh_mat_col_concat_consume (the C++ phased drivers' ColConcatenate: parts released array kind
    by array kind, so a C5 step's 148 GB of pruned pieces concatenate within HBM) builds the same
    block as the copying cbh_mat_col_concat, and frees and clears every part."""
    import ctypes

    import combblas_amd as cb
    from combblas_amd._lib import check, lib

    A = cb.rmat(12)
    dA = cb.SpDCCols.from_host(ctx, A)
    cuts = [0, 700, 701, 2500, A.n]

    def pieces():
        out = []
        for c0, c1 in zip(cuts[:-1], cuts[1:]):
            h = ctypes.c_void_p()
            check(lib().cbh_mat_col_slice(ctx.h, dA.h, c0, c1, ctypes.byref(h)), ctx.h)
            out.append(h.value)
        return (ctypes.c_void_p * len(out))(*out)

    k = len(cuts) - 1
    p1, p2 = pieces(), pieces()
    o1, o2 = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib().cbh_mat_col_concat(ctx.h, k, p1, ctypes.byref(o1)), ctx.h)
    check(lib().cbh_mat_col_concat_consume(ctx.h, k, p2, ctypes.byref(o2)), ctx.h)
    assert all(p2[i] is None for i in range(k)), "consumed parts must be cleared"
    for i in range(k):
        check(lib().cbh_mat_free(ctx.h, ctypes.c_void_p(p1[i])), ctx.h)
    C1, C2 = cb.SpDCCols(ctx, o1), cb.SpDCCols(ctx, o2)
    h1, h2 = C1.to_host(), C2.to_host()
    for a, b, ref in ((h1.jc, h2.jc, A.jc), (h1.cp, h2.cp, A.cp), (h1.ir, h2.ir, A.ir), (h1.num, h2.num, A.num)):
        assert np.array_equal(a, b) and np.array_equal(b, ref)
    for S in (C1, C2, dA):
        S.free()


@pytest.mark.parametrize("cap_frac", [1.0, 0.3])
def test_arena_prune_concat_matches_copying_path(ctx, cap_frac):
    """The C++ phased MCL driver prunes each phase's piece into one output arena and hands the
    arena's arrays to the concatenated result (cbh_mcl_prune_recovery_select_arena +
    cbh_arena_concat); the result equals the copying path (separate pieces + consuming
    concatenation). cap_frac 0.3: the arena overflows after the first piece(s) and the concat falls
    back to copying, with the same result."""
    import ctypes

    import combblas_amd as cb
    from combblas_amd._lib import check, lib

    rng = np.random.default_rng(5)
    A = cb.rmat(12)
    h = cb.HostDcsc(A.m, A.n, A.jc, A.cp, A.ir, rng.integers(1, 1 << 20, A.nnz) / float(1 << 20))
    dA, dB = cb.SpDCCols.from_host(ctx, h), cb.SpDCCols.from_host(ctx, h)
    P = cb.LocalHybridSpGEMM(cb.PlusTimesSRing, dA, dB)
    cuts = [0, 1000, 2500, A.n]
    k = len(cuts) - 1
    hard, sel, rec, pct = 1e-3, 40, 60, 0.9

    def pieces():
        out = []
        for c0, c1 in zip(cuts[:-1], cuts[1:]):
            s = ctypes.c_void_p()
            check(lib().cbh_mat_col_slice(ctx.h, P.h, c0, c1, ctypes.byref(s)), ctx.h)
            out.append(s.value)
        return out

    def pruned(arena):
        res = []
        for s in pieces():
            o = ctypes.c_void_p()
            if arena is None:
                check(lib().cbh_mcl_prune_recovery_select(ctx.h, ctypes.c_void_p(s), hard, sel, rec, pct, None, None,
                                                          ctypes.byref(o)), ctx.h)
            else:
                check(lib().cbh_mcl_prune_recovery_select_arena(ctx.h, ctypes.c_void_p(s), hard, sel, rec, pct, None,
                                                                None, arena, ctypes.byref(o)), ctx.h)
            check(lib().cbh_mat_free(ctx.h, ctypes.c_void_p(s)), ctx.h)
            res.append(o.value)
        return (ctypes.c_void_p * k)(*res)

    p1 = pruned(None)
    o1 = ctypes.c_void_p()
    check(lib().cbh_mat_col_concat_consume(ctx.h, k, p1, ctypes.byref(o1)), ctx.h)
    ar = ctypes.c_void_p()
    nnz1 = cb.SpDCCols(ctx, o1, borrowed=True).nnz
    check(lib().cbh_arena_create(ctx.h, max(1, int(cap_frac * nnz1)), 8, ctypes.byref(ar)), ctx.h)
    p2 = pruned(ar)
    o2 = ctypes.c_void_p()
    check(lib().cbh_arena_concat(ctx.h, k, p2, ar, ctypes.byref(o2)), ctx.h)
    check(lib().cbh_arena_destroy(ctx.h, ar), ctx.h)
    assert all(p2[i] is None for i in range(k))
    C1, C2 = cb.SpDCCols(ctx, o1), cb.SpDCCols(ctx, o2)
    h1, h2 = C1.to_host(), C2.to_host()
    assert h1.nnz == h2.nnz > 0
    for a, b in ((h1.jc, h2.jc), (h1.cp, h2.cp), (h1.ir, h2.ir), (h1.num, h2.num)):
        assert np.array_equal(a, b)
    for S in (C1, C2, P, dA, dB):
        S.free()
