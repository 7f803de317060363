"""Test-side helpers: CBM1 file I/O, the order-sensitive digest, the ctypes binding of the
CPU oracle (oracle/liboracle.so) and deterministic value transforms used by the golden
fixtures. Test infrastructure only -- the product package never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")

VT_F64, VT_I64, VT_U8 = 0, 1, 2
NP_OF_VT = {VT_F64: np.float64, VT_I64: np.int64, VT_U8: np.uint8}


class Dcsc:
    """Host DCSC block: the arrays of combblas::Dcsc (dcsc.h:124-130) plus dimensions."""

    def __init__(self, m, n, jc, cp, ir, num):
        self.m, self.n = int(m), int(n)
        self.jc = np.ascontiguousarray(jc, dtype=np.int64)
        self.cp = np.ascontiguousarray(cp, dtype=np.int64)
        self.ir = np.ascontiguousarray(ir, dtype=np.int32)
        self.num = np.ascontiguousarray(num)
        if self.cp.size == 0:
            self.cp = np.zeros(1, np.int64)

    @property
    def nnz(self):
        return int(self.ir.size)

    @property
    def nzc(self):
        return int(self.jc.size)

    def astype(self, dt):
        return Dcsc(self.m, self.n, self.jc, self.cp, self.ir, self.num.astype(dt))

    def cols(self):
        """column id of every entry"""
        return np.repeat(self.jc, np.diff(self.cp))

    def to_dense(self):
        d = np.zeros((self.m, self.n), dtype=self.num.dtype)
        d[self.ir, self.cols()] = self.num
        return d

    def to_coo_sorted(self):
        """(col,row)-sorted arrays, independent of within-column order."""
        c = self.cols()
        o = np.lexsort((self.ir, c))
        return c[o], self.ir[o], self.num[o]

    @staticmethod
    def from_coo(m, n, rows, cols, vals):
        rows = np.asarray(rows, np.int64)
        cols = np.asarray(cols, np.int64)
        vals = np.asarray(vals)
        o = np.lexsort((rows, cols))
        rows, cols, vals = rows[o], cols[o], vals[o]
        jc, first = np.unique(cols, return_index=True)
        cp = np.append(first, rows.size).astype(np.int64)
        return Dcsc(m, n, jc, cp, rows.astype(np.int32), vals)

    def col_slice(self, c0, c1):
        """columns [c0,c1) keeping the global column space (a ColSplit piece)"""
        sel = (self.jc >= c0) & (self.jc < c1)
        idx = np.nonzero(sel)[0]
        if idx.size == 0:
            return Dcsc(self.m, self.n, [], [0], [], self.num[:0])
        s, e = self.cp[idx[0]], self.cp[idx[-1] + 1]
        return Dcsc(self.m, self.n, self.jc[idx], self.cp[idx[0]: idx[-1] + 2] - s, self.ir[s:e], self.num[s:e])

    def row_slice(self, r0, r1):
        """rows [r0,r1) keeping the global row space"""
        c = self.cols()
        keep = (self.ir >= r0) & (self.ir < r1)
        return Dcsc.from_coo(self.m, self.n, self.ir[keep], c[keep], self.num[keep])


def read_cbm(path) -> Dcsc:
    b = open(path, "rb").read()
    assert b[:4] == b"CBM1", path
    (vt,) = struct.unpack_from("<I", b, 4)
    m, n, nnz, nzc = struct.unpack_from("<4q", b, 8)
    o = 40
    jc = np.frombuffer(b, np.int64, nzc, o); o += 8 * nzc
    cp = np.frombuffer(b, np.int64, nzc + 1, o); o += 8 * (nzc + 1)
    ir = np.frombuffer(b, np.int32, nnz, o); o += 4 * nnz
    num = np.frombuffer(b, NP_OF_VT[vt], nnz, o)
    return Dcsc(m, n, jc.copy(), cp.copy(), ir.copy(), num.copy())


def write_cbm(path, d: Dcsc):
    dt = d.num.dtype
    vt = VT_F64 if dt == np.float64 else (VT_U8 if dt in (np.uint8, np.bool_) else VT_I64)
    num = d.num.astype(NP_OF_VT[vt])
    with open(path, "wb") as f:
        f.write(b"CBM1")
        f.write(struct.pack("<I4q", vt, d.m, d.n, d.nnz, d.nzc))
        f.write(d.jc.tobytes()); f.write(d.cp.tobytes()); f.write(d.ir.tobytes()); f.write(num.tobytes())


def save_npz(path, **mats):
    arrs = {}
    for k, d in mats.items():
        arrs[k + "_dims"] = np.array([d.m, d.n], np.int64)
        arrs[k + "_jc"], arrs[k + "_cp"], arrs[k + "_ir"], arrs[k + "_num"] = d.jc, d.cp, d.ir, d.num
    np.savez_compressed(path, **arrs)


def load_npz(path):
    z = np.load(path, allow_pickle=False)
    out = {}
    for k in {n[: -len("_dims")] for n in z.files if n.endswith("_dims")}:
        m, n = z[k + "_dims"]
        out[k] = Dcsc(m, n, z[k + "_jc"], z[k + "_cp"], z[k + "_ir"], z[k + "_num"])
    return out


# ------------------------------------------------------------------ digest (same as device)
_M1, _M2 = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)


def _mix64(z):
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def value_bits(num):
    if num.dtype == np.float64:
        return num.view(np.uint64)
    if num.dtype == np.float32:
        return num.view(np.uint32).astype(np.uint64)
    if num.dtype == np.int32:
        return num.view(np.uint32).astype(np.uint64)
    if num.dtype in (np.uint8, np.bool_):
        return num.astype(np.uint64)
    return num.astype(np.int64).view(np.uint64)


def digest(d: Dcsc, base=0):
    """(value sum, sum_p mix64(p ^ mix64(col ^ mix64(row ^ mix64(bits))))) mod 2^64, in C order"""
    p = np.arange(base, base + d.nnz, dtype=np.uint64)
    cols = d.cols().astype(np.uint64)
    rows = d.ir.astype(np.uint32).astype(np.uint64)
    h = _mix64(p ^ _mix64(cols ^ _mix64(rows ^ _mix64(value_bits(d.num)))))
    with np.errstate(over="ignore"):
        dig = int(np.sum(h, dtype=np.uint64))
    return float(np.sum(d.num.astype(np.float64))), dig


# ------------------------------------------------------------------ deterministic value transforms
def signed_small_ints(d: Dcsc, mod=17):
    """value' = ((row*7 + col*13) % mod) - mod//2, as int64 (exercises max/min semirings)"""
    c = d.cols()
    v = ((d.ir.astype(np.int64) * 7 + c * 13) % mod) - mod // 2
    return Dcsc(d.m, d.n, d.jc, d.cp, d.ir, v.astype(np.int64))


def dyadic_signed(d: Dcsc):
    """value' = count * (-1)^(row+col) / 2^(row % 4): exact in f64 under any summation order"""
    c = d.cols()
    sign = np.where((d.ir.astype(np.int64) + c) % 2 == 0, 1.0, -1.0)
    return Dcsc(d.m, d.n, d.jc, d.cp, d.ir, d.num.astype(np.float64) * sign / (2.0 ** (d.ir % 4)))


def with_explicit_zeros(d: Dcsc, every=5):
    """every k-th entry set to 0 (kept as an explicit zero, as TC's GetLowerTriangular does)"""
    num = d.num.copy()
    num[::every] = 0
    return Dcsc(d.m, d.n, d.jc, d.cp, d.ir, num)


# ------------------------------------------------------------------ oracle binding
class _OrMat(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int64), ("n", ctypes.c_int64), ("nnz", ctypes.c_int64), ("nzc", ctypes.c_int64),
                ("cp", ctypes.c_void_p), ("jc", ctypes.c_void_p), ("ir", ctypes.c_void_p), ("num", ctypes.c_void_p),
                ("dtype", ctypes.c_int), ("owned", ctypes.c_int)]


_DT_CODE = {np.dtype(np.float64): 0, np.dtype(np.int64): 1, np.dtype(np.uint8): 2, np.dtype(np.bool_): 2,
            np.dtype(np.float32): 3, np.dtype(np.int32): 4}
_NP_OF_CODE = {0: np.float64, 1: np.int64, 2: np.uint8, 3: np.float32, 4: np.int32}
SR_CODE = {"plus_times": 0, "select_max": 1, "min_plus": 2, "or_and": 0}
KERNEL_CODE = {"hybrid": 0, "hash": 1, "hashu": 2, "heap": 3}


class Oracle:
    """ctypes binding of oracle/liboracle.so (built by `make -C oracle`)."""

    def __init__(self):
        path = os.path.join(REPO, "oracle", "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
        self.lib = ctypes.CDLL(path)
        P = ctypes.POINTER(_OrMat)
        self.lib.oracle_spgemm.restype = P
        self.lib.oracle_spgemm.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int]
        self.lib.oracle_merge.restype = P
        self.lib.oracle_merge.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(P)]
        self.lib.oracle_symbolic.argtypes = [P, P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        self.lib.oracle_free.argtypes = [P]

    @staticmethod
    def _in(d: Dcsc):
        num = d.num.astype(np.uint8) if d.num.dtype == np.bool_ else d.num
        keep = (d, num)
        s = _OrMat(d.m, d.n, d.nnz, d.nzc, d.cp.ctypes.data, d.jc.ctypes.data, d.ir.ctypes.data,
                   num.ctypes.data, _DT_CODE[num.dtype], 0)
        return s, keep

    @staticmethod
    def _out(p):
        r = p.contents
        dt = _NP_OF_CODE[r.dtype]
        take = lambda ptr, n, t: np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(np.ctypeslib.as_ctypes_type(t))), (max(n, 1),))[:n].copy()
        d = Dcsc(r.m, r.n, take(r.jc, r.nzc, np.int64), take(r.cp, r.nzc + 1, np.int64),
                 take(r.ir, r.nnz, np.int32), take(r.num, r.nnz, dt))
        return d

    def spgemm(self, A: Dcsc, B: Dcsc, semiring="plus_times", kernel="hybrid", threads=1) -> Dcsc:
        a, ka = self._in(A)
        b, kb = self._in(B)
        p = self.lib.oracle_spgemm(SR_CODE[semiring], a.dtype, KERNEL_CODE[kernel], ctypes.byref(a), ctypes.byref(b), threads)
        assert p, "oracle_spgemm failed"
        out = self._out(p)
        self.lib.oracle_free(p)
        return out

    def merge(self, lists, semiring="plus_times") -> Dcsc:
        ins = [self._in(d) for d in lists]
        arr = (ctypes.POINTER(_OrMat) * len(ins))(*[ctypes.pointer(s) for s, _ in ins])
        p = self.lib.oracle_merge(SR_CODE[semiring], ins[0][0].dtype, len(ins), arr)
        assert p, "oracle_merge failed"
        out = self._out(p)
        self.lib.oracle_free(p)
        return out

    def symbolic(self, A: Dcsc, B: Dcsc, threads=1):
        a, ka = self._in(A)
        b, kb = self._in(B)
        f, z = ctypes.c_int64(), ctypes.c_int64()
        cf = np.zeros(B.nzc, np.int64)
        cz = np.zeros(B.nzc, np.int64)
        rc = self.lib.oracle_symbolic(ctypes.byref(a), ctypes.byref(b), ctypes.byref(f), ctypes.byref(z),
                                      cf.ctypes.data, cz.ctypes.data, threads)
        assert rc == 0
        return f.value, z.value, cf, cz


def assert_dcsc_equal(got: Dcsc, exp: Dcsc, rtol=0.0, sorted_rows=True, msg=""):
    """Structure exactly equal (Dcsc::operator==, dcsc.cpp:473-506); values bit-exact unless rtol."""
    assert (got.m, got.n) == (exp.m, exp.n), f"{msg} dims {got.m}x{got.n} vs {exp.m}x{exp.n}"
    assert got.nnz == exp.nnz, f"{msg} nnz {got.nnz} vs {exp.nnz}"
    np.testing.assert_array_equal(got.jc, exp.jc, err_msg=f"{msg} jc")
    np.testing.assert_array_equal(got.cp, exp.cp, err_msg=f"{msg} cp")
    if sorted_rows:
        g_ir, g_num, e_ir, e_num = got.ir, got.num, exp.ir, exp.num
    else:
        _, g_ir, g_num = got.to_coo_sorted()
        _, e_ir, e_num = exp.to_coo_sorted()
    np.testing.assert_array_equal(g_ir, e_ir, err_msg=f"{msg} ir")
    if rtol == 0.0:
        np.testing.assert_array_equal(value_bits(g_num.astype(e_num.dtype)), value_bits(e_num), err_msg=f"{msg} values")
    else:
        np.testing.assert_allclose(g_num, e_num, rtol=rtol, atol=0, err_msg=f"{msg} values")


SR_OF_TAG = {"pt_f64": "plus_times", "pt_i64": "plus_times", "max_i64": "select_max", "min_i64": "min_plus",
             "bool": "or_and"}


def values_for(tag, A: Dcsc) -> Dcsc:
    """input values per semiring tag, exactly as tests/golden/make_golden.py feeds the reference"""
    if tag == "pt_f64":
        return dyadic_signed(A)
    if tag == "pt_i64":
        return A.astype(np.int64)
    if tag in ("max_i64", "min_i64"):
        return signed_small_ints(A)
    if tag == "bool":
        return A.astype(np.uint8)
    raise ValueError(tag)


def random_dcsc(rng, m, n, density, dtype=np.float64, empty_cols=0.0):
    """uniform random sparse block (optional fraction of forced-empty columns)"""
    nnz = int(m * n * density)
    rows = rng.integers(0, m, nnz)
    cols = rng.integers(0, n, nnz)
    if empty_cols > 0:
        dead = rng.random(n) < empty_cols
        keep = ~dead[cols]
        rows, cols = rows[keep], cols[keep]
    key = np.unique(cols.astype(np.int64) * m + rows)
    rows, cols = key % m, key // m
    if dtype == np.float64:
        vals = rng.integers(-8, 9, rows.size) / 4.0
    elif dtype == np.uint8:
        vals = (rng.random(rows.size) < 0.8).astype(np.uint8)
    else:
        vals = rng.integers(-5, 6, rows.size).astype(dtype)
    return Dcsc.from_coo(m, n, rows, cols, np.asarray(vals, dtype))


# ------------------------------------------------------------------ closed forms
def product_value_sum(A: Dcsc, B: Dcsc = None):
    """sum of all values of A*B under PlusTimes = sum_k colsum_k(A) * rowsum_k(B) (exact in int64
    for multiplicity-valued R-MAT; a size-independent property of the whole product)."""
    B = A if B is None else B
    colsum = np.zeros(A.n, np.int64)
    colsum[A.jc] = np.add.reduceat(A.num.astype(np.int64), A.cp[:-1]) if A.nnz else 0
    rowsum = np.bincount(B.ir, weights=None, minlength=B.m).astype(np.int64) if B.num.dtype == bool else \
        np.bincount(B.ir, weights=B.num.astype(np.float64), minlength=B.m).astype(np.int64)
    return int(np.dot(colsum, rowsum))
