"""Multi-process harness for the distributed drivers (test infrastructure only).

`OracleBackend` supplies the local-block operations of combblas_amd.backend.HipBackend from the
CPU oracle, on host torch tensors, so that the grid logic of parfriends.py (stage broadcasts,
phase planning, 3D reduce-scatter, merges) runs under `gloo` in CPU processes. The product path
never uses it: HipBackend has no CPU fallback.

`run_world(fn, world, *args)` spawns `world` processes with a gloo process group on 127.0.0.1
and returns what rank 0's fn returned.
"""
from __future__ import annotations

import datetime
import os
import socket
import sys
import tempfile
import time
import traceback

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import helpers as H  # noqa: E402

ORACLE_SR = {"PlusTimesSRing": "plus_times", "SelectMaxSRing": "select_max", "MinPlusSRing": "min_plus",
             "OrAndSRing": "or_and"}
T_OF_NP = {np.dtype(np.float64): torch.float64, np.dtype(np.int64): torch.int64, np.dtype(np.uint8): torch.uint8,
           np.dtype(np.int32): torch.int32, np.dtype(np.float32): torch.float32}


class OBlock:
    def __init__(self, m, n, cp, jc, ir, num):
        self.m, self.n = int(m), int(n)
        self.cp, self.jc, self.ir, self.num = cp, jc, ir, num

    def dcsc(self):
        return H.Dcsc(self.m, self.n, self.jc.numpy(), self.cp.numpy(), self.ir.numpy(), self.num.numpy())


class OracleBackend:
    device = torch.device("cpu")

    def __init__(self):
        self.o = H.Oracle()

    @staticmethod
    def _from_dcsc(d):
        num = np.ascontiguousarray(d.num.astype(np.uint8) if d.num.dtype == np.bool_ else d.num)
        return OBlock(d.m, d.n, torch.from_numpy(np.ascontiguousarray(d.cp, np.int64)),
                      torch.from_numpy(np.ascontiguousarray(d.jc, np.int64)),
                      torch.from_numpy(np.ascontiguousarray(d.ir, np.int32)), torch.from_numpy(num))

    def from_host(self, h):
        return self._from_dcsc(h)

    @staticmethod
    def wrap(m, n, cp, jc, ir, num):
        return OBlock(m, n, cp.contiguous(), jc.contiguous(), ir.contiguous(), num.contiguous())

    @staticmethod
    def dims(b):
        return b.m, b.n, int(b.ir.numel()), int(b.jc.numel())

    @staticmethod
    def arrays(b):
        return b.cp, b.jc, b.ir, b.num

    @staticmethod
    def value_dtype(b):
        return b.num.dtype

    @staticmethod
    def to_host(b):
        import combblas_amd as cb
        return cb.HostDcsc(b.m, b.n, b.jc.numpy(), b.cp.numpy(), b.ir.numpy(), b.num.numpy())

    @staticmethod
    def free(b):
        pass

    def multiply(self, SR, A, B):
        if A.ir.numel() == 0 or B.ir.numel() == 0:
            return OBlock(A.m, B.n, torch.zeros(1, dtype=torch.int64), torch.zeros(0, dtype=torch.int64),
                          torch.zeros(0, dtype=torch.int32), torch.zeros(0, dtype=A.num.dtype))
        return self._from_dcsc(self.o.spgemm(A.dcsc(), B.dcsc(), ORACLE_SR[SR.name], "hybrid"))

    def merge(self, SR, blocks, m, n):
        return self._from_dcsc(self.o.merge([b.dcsc() for b in blocks], ORACLE_SR[SR.name]))

    def plan(self, A, B):
        be = self

        class _Plan:  # the phase-loop protocol of HipBackend.plan, on the oracle
            def col_nnz(self):
                return be.col_nnz(A, B)

            def multiply(self, SR, c0, c1):
                from combblas_amd.parfriends import _colslice

                return be.multiply(SR, A, _colslice(be, B, c0, c1))

            def close(self):
                pass

        return _Plan()

    def col_nnz(self, A, B):
        if A.ir.numel() == 0 or B.ir.numel() == 0:
            return torch.zeros(B.jc.numel(), dtype=torch.int64)
        return torch.from_numpy(self.o.symbolic(A.dcsc(), B.dcsc())[3])

    def synchronize(self):
        pass

    # ---- callers around the hot path (numpy restatements, oracle/apps_oracle.py)
    def ewise_mult(self, A, B):
        import apps_oracle as AO
        return self._from_dcsc(AO.ewise_mult(A.dcsc(), B.dcsc()))

    def masked(self, SR, A, B, M, pattern=False):
        import apps_oracle as AO
        C = self.multiply(SR, A, B).dcsc()
        ones = H.Dcsc(M.m, M.n, M.jc.numpy(), M.cp.numpy(), M.ir.numpy(), np.ones(M.ir.numel(), C.num.dtype))
        return self._from_dcsc(AO.ewise_mult(C, ones if pattern else M.dcsc()))

    @staticmethod
    def col_stats(A, hard):
        import apps_oracle as AO
        return tuple(torch.from_numpy(x) for x in AO.column_stats(A.dcsc(), hard))

    @staticmethod
    def kselect_hist(A, aidx, nact, prefix, shift):
        d = A.dcsc()
        hist = np.zeros((nact, 256), np.int32)
        ai = aidx.numpy()[d.cols()]
        sel = ai >= 0
        b = d.num[sel].astype(np.float64).view(np.uint64)
        key = np.where(b >> np.uint64(63), ~b, b | np.uint64(1 << 63))
        himask = np.uint64(0) if shift >= 56 else np.uint64((0xFFFFFFFFFFFFFFFF << (shift + 8)) & 0xFFFFFFFFFFFFFFFF)
        pre = prefix.numpy().view(np.uint64)[ai[sel]]
        match = (key & himask) == pre
        dig = ((key >> np.uint64(shift)) & np.uint64(255)).astype(np.int64)
        np.add.at(hist, (ai[sel][match], dig[match]), 1)
        return torch.from_numpy(hist.ravel())

    @staticmethod
    def kselect_pick(nact, hist, prefix, rank, shift):
        h = hist.numpy().reshape(nact, 256)
        pv, rv = prefix.numpy().view(np.uint64), rank.numpy()
        for a in range(nact):
            r = int(rv[a])
            if r < 0:
                continue
            b = 255
            while b > 0 and r >= h[a, b]:
                r -= int(h[a, b])
                b -= 1
            pv[a] |= np.uint64(b) << np.uint64(shift)
            rv[a] = r

    @staticmethod
    def kselect_value(nact, prefix):
        k = prefix.numpy().view(np.uint64)
        b = np.where(k >> np.uint64(63), k & np.uint64(0x7FFFFFFFFFFFFFFF), ~k)
        return torch.from_numpy(b.view(np.float64).copy())

    def prune_columns(self, A, thresh):
        import apps_oracle as AO
        return self._from_dcsc(AO.prune_column(A.dcsc(), thresh.numpy()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _trace(rank, msg):
    """CBH_TRACE_DIR: each rank appends its progress (flushed) to rank<r>.log there"""
    d = os.environ.get("CBH_TRACE_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"rank{rank}.log"), "a") as f:
            f.write(f"{time.time():.3f} {msg}\n")


def _worker(rank, world, port, fn, args, outdir, coll_timeout=200):
    import pickle

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    # gloo's default device resolves the host name, a DNS query that can block for the resolver's
    # timeouts on a box without name service; on the loopback interface it needs no lookup
    if "GLOO_SOCKET_IFNAME" not in os.environ and os.path.exists("/sys/class/net/lo"):
        os.environ["GLOO_SOCKET_IFNAME"] = "lo"
    _trace(rank, "spawned")
    res = None
    try:
        # a collective times out (and the rank reports where) before the world's deadline, instead
        # of waiting gloo's default 30 minutes
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=coll_timeout))
        _trace(rank, "process group")
        res = ("ok", fn(rank, world, *args))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:  # noqa: BLE001
        res = ("err", traceback.format_exc())
    with open(os.path.join(outdir, f"r{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)


def run_world(fn, world, *args, timeout=240):
    """Runs fn(rank, world, *args) on `world` gloo processes; returns rank 0's result."""
    import pickle

    import torch.multiprocessing as mp

    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        coll_timeout = max(30, timeout - 40)
        procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, d, coll_timeout)) for r in range(world)]
        for p in procs:
            p.start()
        deadline = time.monotonic() + timeout  # one budget for the whole world, not per rank
        for p in procs:
            p.join(max(0.0, deadline - time.monotonic()))
        alive = [r for r, p in enumerate(procs) if p.is_alive()]
        if alive:  # kill EVERY straggler: a live rank left behind blocks the interpreter's exit
            for r in alive:
                procs[r].kill()
            for r in alive:
                procs[r].join(10)
            errs = []
            for r in range(world):
                path = os.path.join(d, f"r{r}.pkl")
                if os.path.exists(path):
                    with open(path, "rb") as f:
                        st, v = pickle.load(f)
                    if st != "ok":
                        errs.append(f"rank {r}: {v}")
            raise TimeoutError(f"distributed test timed out; ranks still running: {alive}" +
                               ("".join("\n" + e for e in errs)))
        results = []
        for r in range(world):
            path = os.path.join(d, f"r{r}.pkl")
            if not os.path.exists(path):
                raise RuntimeError(f"rank {r} died (exit {procs[r].exitcode})")
            with open(path, "rb") as f:
                results.append(pickle.load(f))
        for r, (st, v) in enumerate(results):
            if st != "ok":
                raise AssertionError(f"rank {r} failed:\n{v}")
        return results[0][1]
