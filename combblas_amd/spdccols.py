"""Device-resident DCSC blocks and the per-device context.

`SpDCCols` mirrors combblas::SpDCCols<IT,NT> (include/CombBLAS/SpDCCols.h:51-340) for one
local block: the Dcsc arrays cp[nzc+1], jc[nzc], ir[nnz], numx[nnz] (dcsc.h:124-130), kept in
HBM. Row ids are local int32, pointers int64 (see DESIGN.md §2 for the layout).

`Context` owns a cbh_ctx (device + stream). By default every device allocation the library
makes goes through torch's caching allocator on the context's stream, so matrices produced by
the HIP kernels are plain torch tensors that torch.distributed (RCCL) can broadcast.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib

DTYPE_CODE = {np.dtype(np.float64): 0, np.dtype(np.int64): 1, np.dtype(np.uint8): 2, np.dtype(np.bool_): 2,
              np.dtype(np.float32): 3, np.dtype(np.int32): 4}
NP_OF_CODE = {0: np.float64, 1: np.int64, 2: np.uint8, 3: np.float32, 4: np.int32}


def _torch():
    import torch  # plumbing only (device memory, streams, torch.distributed)
    return torch


def torch_dtype(code):
    t = _torch()
    return {0: t.float64, 1: t.int64, 2: t.uint8, 3: t.float32, 4: t.int32}[code]


class HostDcsc:
    """Host copy of a DCSC block (numpy)."""

    def __init__(self, m, n, jc, cp, ir, num):
        self.m, self.n = int(m), int(n)
        self.jc = np.ascontiguousarray(jc, np.int64)
        self.cp = np.ascontiguousarray(cp if len(cp) else [0], np.int64)
        self.ir = np.ascontiguousarray(ir, np.int32)
        num = np.asarray(num)
        self.num = np.ascontiguousarray(num.astype(np.uint8) if num.dtype == np.bool_ else num)

    nnz = property(lambda s: int(s.ir.size))
    nzc = property(lambda s: int(s.jc.size))

    @staticmethod
    def from_csc(m, n, colptr, rowidx, vals):
        colptr = np.asarray(colptr, np.int64)
        lens = np.diff(colptr)
        jc = np.nonzero(lens)[0].astype(np.int64)
        cp = np.concatenate([colptr[jc], colptr[-1:]]) if jc.size else np.zeros(1, np.int64)
        return HostDcsc(m, n, jc, cp - (cp[0] if cp.size else 0), rowidx[colptr[0]:colptr[-1]], vals[colptr[0]:colptr[-1]])

    def astype(self, dt):
        return HostDcsc(self.m, self.n, self.jc, self.cp, self.ir, self.num.astype(dt))


class Context:
    """One HIP device + stream for the hot path (the reference's one-rank-one-thread model)."""

    def __init__(self, device: int = 0, torch_allocator: bool = True, stream=None):
        # torch ships its own HIP runtime (torch/lib/libamdhip64.so) beside the one this library links
        # (/opt/rocm): torch's must initialise first, or its later first use in the process finds no
        # device (seen on the GPU box: torch.cuda.Stream after a torch-free Context)
        try:
            torch = _torch()
            if torch.cuda.is_available():
                torch.cuda.init()
        except ImportError:
            pass
        L = lib()
        h = ctypes.c_void_p()
        check(L.cbh_ctx_create(device, ctypes.byref(h)))
        self.h = h
        self.device = device
        self._live = {}
        self._alloc_cb = self._free_cb = None
        self.tdevice = None
        if torch_allocator or stream is not None:
            torch = _torch()
            self.tdevice = torch.device("cuda", device)
            s = stream
            if s is None or s.cuda_stream == 0:
                # torch's default stream is the legacy NULL stream, which the C-ABI cannot name
                # (NULL = "own stream"): give library and torch one explicit stream instead, and
                # make it this thread's current stream so torch ops on library outputs (and the
                # collectives that sync with the current stream) are ordered with the kernels.
                s = torch.cuda.Stream(self.tdevice)
                torch.cuda.set_stream(s)
            self.tstream = s
            check(L.cbh_ctx_set_stream(self.h, ctypes.c_void_p(s.cuda_stream)), self.h)
        if torch_allocator:
            torch = _torch()

            def _alloc(user, nbytes, stream):
                # the block belongs to the library's stream (whatever stream is current in the
                # caller): torch's caching allocator then reuses it only in that stream's order,
                # which is the order every library kernel and free happens in
                with torch.cuda.stream(self.tstream):
                    t = torch.empty(int(nbytes), dtype=torch.uint8, device=self.tdevice)
                p = t.data_ptr()
                self._live[p] = t
                return p

            def _free(user, ptr, stream):
                self._live.pop(ptr, None)

            self._alloc_cb = _lib.ALLOC_FN(_alloc)
            self._free_cb = _lib.FREE_FN(_free)
            check(L.cbh_ctx_set_allocator(self.h, self._alloc_cb, self._free_cb, None), self.h)

    def tensor_at(self, ptr, nbytes):
        """torch uint8 view of library memory allocated through the torch allocator"""
        t = self._live.get(ptr)
        if t is None:
            raise KeyError("pointer not allocated through this context's torch allocator")
        return t[:nbytes]

    def synchronize(self):
        check(lib().cbh_ctx_synchronize(self.h), self.h)

    def trim(self):
        """return the built-in allocator's cached blocks and the phase workspace to HIP"""
        check(lib().cbh_ctx_trim(self.h), self.h)

    def release(self, nbytes):
        """return at least nbytes of the built-in allocator's cached blocks to HIP, largest first"""
        check(lib().cbh_ctx_release(self.h, int(nbytes)), self.h)

    def memory(self):
        """{live, cached, device_free, device_total} in bytes: the built-in allocator's live and
        cached (free, not yet returned to HIP) bytes and the device's free / total memory"""
        v = [ctypes.c_int64() for _ in range(4)]
        check(lib().cbh_ctx_memory(self.h, *[ctypes.byref(x) for x in v]), self.h)
        return dict(zip(("live", "cached", "device_free", "device_total"), (x.value for x in v)))

    def take_retries(self):
        """sub-tiles the task kernels retried with half the row range since the last call (resets)"""
        n = ctypes.c_int64()
        check(lib().cbh_ctx_take_retries(self.h, ctypes.byref(n)), self.h)
        return n.value

    def enable_timing(self, on=True):
        check(lib().cbh_ctx_enable_timing(self.h, int(on)), self.h)

    def kernel_times(self):
        t = _lib.cbh_kernel_times()
        check(lib().cbh_last_kernel_times(self.h, ctypes.byref(t)), self.h)
        return {"symbolic_ms": t.symbolic_ms, "numeric_ms": t.numeric_ms, "total_ms": t.total_ms,
                "numeric_launches": t.numeric_launches}

    def kernel_stats(self):
        """{kind: {ms, launches, alg_bytes}} accumulated while timing is enabled"""
        out = {}
        for k, name in enumerate(_lib.K_NAMES):
            st = _lib.cbh_kernel_stat()
            check(lib().cbh_kernel_stats(self.h, k, ctypes.byref(st)), self.h)
            out[name] = {"ms": st.ms, "launches": st.launches, "alg_bytes": st.alg_bytes}
        return out

    def reset_kernel_stats(self):
        check(lib().cbh_kernel_stats_reset(self.h), self.h)

    def set_phase_budget(self, nbytes):
        check(lib().cbh_ctx_set_phase_budget(self.h, int(nbytes)), self.h)

    def close(self):
        if self.h:
            lib().cbh_ctx_destroy(self.h)
            self.h = None
            self._live.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SpDCCols:
    """A device-resident local sparse block (wraps a cbh_mat handle)."""

    def __init__(self, ctx: Context, handle, keepalive=None, borrowed=False):
        # borrowed: a non-owning view the library hands out (the per-phase consumer of
        # cbh_spgemm_phased); free() only forgets it
        self.ctx, self.h, self._keep, self._borrowed = ctx, handle, keepalive, borrowed
        m, n, nnz, nzc, dt = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int()
        check(lib().cbh_mat_info(handle, ctypes.byref(m), ctypes.byref(n), ctypes.byref(nnz), ctypes.byref(nzc),
                                 ctypes.byref(dt)))
        self.m, self.n, self.nnz, self.nzc, self.dtype_code = m.value, n.value, nnz.value, nzc.value, dt.value

    # reference-style accessors
    def getnrow(self):
        return self.m

    def getncol(self):
        return self.n

    def getnnz(self):
        return self.nnz

    def getnzc(self):
        return self.nzc

    def isZero(self):
        return self.nnz == 0

    @property
    def np_dtype(self):
        return np.dtype(NP_OF_CODE[self.dtype_code])

    @staticmethod
    def from_host(ctx: Context, d: HostDcsc, dtype=None):
        num = d.num if dtype is None else d.num.astype(dtype)
        num = np.ascontiguousarray(num.astype(np.uint8) if num.dtype == np.bool_ else num)
        s = _lib.cbh_dcsc(d.m, d.n, d.nnz, d.nzc, d.cp.ctypes.data, d.jc.ctypes.data, d.ir.ctypes.data,
                          num.ctypes.data)
        h = ctypes.c_void_p()
        check(lib().cbh_mat_upload(ctx.h, ctypes.byref(s), DTYPE_CODE[num.dtype], ctypes.byref(h)), ctx.h)
        return SpDCCols(ctx, h)

    @staticmethod
    def from_tensors(ctx: Context, m, n, cp, jc, ir, num):
        """zero-copy wrap of torch device tensors (e.g. a received SUMMA broadcast)"""
        torch = _torch()
        code = {torch.float64: 0, torch.int64: 1, torch.uint8: 2, torch.bool: 2, torch.float32: 3,
                torch.int32: 4}[num.dtype]
        assert cp.dtype == torch.int64 and jc.dtype == torch.int64 and ir.dtype == torch.int32
        s = _lib.cbh_dcsc(m, n, ir.numel(), jc.numel(), cp.data_ptr(), jc.data_ptr(), ir.data_ptr(), num.data_ptr())
        h = ctypes.c_void_p()
        check(lib().cbh_mat_wrap_device(ctx.h, ctypes.byref(s), code, ctypes.byref(h)), ctx.h)
        return SpDCCols(ctx, h, keepalive=(cp, jc, ir, num))

    @staticmethod
    def from_tuples(ctx: Context, m, n, rows, cols, vals, removeloops=False):
        """SpDCCols(SpTuples) from device COO tensors (rows int32, cols int64, vals) in any order,
        duplicates combined (sum; OR for bool) -- SpTuples.cpp:70-118 + SpDCCols.cpp:109-183 on
        the device (cbh_tuples_to_dcsc)."""
        torch = _torch()
        code = {torch.float64: 0, torch.int64: 1, torch.uint8: 2, torch.bool: 2, torch.float32: 3,
                torch.int32: 4}[vals.dtype]
        rows = rows.to(torch.int32).contiguous()
        cols = cols.to(torch.int64).contiguous()
        vals = (vals.to(torch.uint8) if vals.dtype == torch.bool else vals).contiguous()
        h = ctypes.c_void_p()
        check(lib().cbh_tuples_to_dcsc(ctx.h, int(m), int(n), rows.numel(), ctypes.c_void_p(rows.data_ptr()),
                                       ctypes.c_void_p(cols.data_ptr()), ctypes.c_void_p(vals.data_ptr()), code,
                                       _lib.CBH_TUPLES_DROP_LOOPS if removeloops else 0, ctypes.byref(h)), ctx.h)
        return SpDCCols(ctx, h)

    def to_tuples(self):
        """SpTuples(const SpDCCols&): (rows int32, cols int64, vals) device tensors, column-sorted"""
        torch = _torch()
        dev = self.ctx.tdevice or torch.device("cuda", self.ctx.device)
        rows = torch.empty(self.nnz, dtype=torch.int32, device=dev)
        cols = torch.empty(self.nnz, dtype=torch.int64, device=dev)
        vals = torch.empty(self.nnz, dtype=torch_dtype(self.dtype_code), device=dev)
        torch.cuda.synchronize(dev)
        check(lib().cbh_dcsc_to_tuples(self.ctx.h, self.h, ctypes.c_void_p(rows.data_ptr()),
                                       ctypes.c_void_p(cols.data_ptr()), ctypes.c_void_p(vals.data_ptr())), self.ctx.h)
        return rows, cols, vals

    def tensors(self):
        """(cp, jc, ir, num) as torch tensors viewing device memory (no copy)."""
        if self._keep is not None:
            return self._keep
        torch = _torch()
        ptrs = [ctypes.c_void_p() for _ in range(4)]
        check(lib().cbh_mat_device_arrays(self.h, *[ctypes.byref(p) for p in ptrs]))
        sizes = [(self.nzc + 1) * 8, self.nzc * 8, self.nnz * 4, self.nnz * self.np_dtype.itemsize]
        dts = [torch.int64, torch.int64, torch.int32, torch_dtype(self.dtype_code)]
        out = []
        for p, nb, dt, cnt in zip(ptrs, sizes, dts, [self.nzc + 1, self.nzc, self.nnz, self.nnz]):
            out.append(self.ctx.tensor_at(p.value, nb).view(dt)[:cnt])
        return tuple(out)

    def to_host(self) -> HostDcsc:
        cp = np.empty(self.nzc + 1, np.int64)
        jc = np.empty(self.nzc, np.int64)
        ir = np.empty(self.nnz, np.int32)
        num = np.empty(self.nnz, NP_OF_CODE[self.dtype_code])
        check(lib().cbh_mat_copy_out(self.ctx.h, self.h, cp.ctypes.data, jc.ctypes.data, ir.ctypes.data,
                                     num.ctypes.data, 0), self.ctx.h)
        return HostDcsc(self.m, self.n, jc, cp, ir, num)

    def checksum(self):
        """(value sum, order-sensitive digest) computed on the device (cbh_mat_checksum; the same
        definition as tests/helpers.digest and the phased product's CBH_PHASE_CHECKSUM)"""
        s, d = ctypes.c_double(), ctypes.c_uint64()
        check(lib().cbh_mat_checksum(self.ctx.h, self.h, ctypes.byref(s), ctypes.byref(d)), self.ctx.h)
        return s.value, d.value

    def clone(self):
        """deep copy on the device (SpDCCols copy constructor, SpDCCols.cpp:214-226)"""
        h = ctypes.c_void_p()
        check(lib().cbh_mat_clone(self.ctx.h, self.h, ctypes.byref(h)), self.ctx.h)
        return SpDCCols(self.ctx, h)

    def free(self):
        if self.h is not None and self.ctx.h and not self._borrowed:
            lib().cbh_mat_free(self.ctx.h, self.h)
        self.h = None
        self._keep = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
