#!/usr/bin/env python3
"""Regenerates tests/golden/fullsize.json: known answers for the configs at their FULL sizes, which
tests/test_fullsize_gpu.py checks on the GPU box (the driver's -m gpu run must cover
them, not only the bench scripts).

  C3  Galerkin R^T (A R) on the 27-point Poisson operator of a 256^3 grid with trilinear
      prolongation onto 128^3 (combblas_amd.galerkin, GalerkinNew.cpp:100-106): nnz(AR), nnz(R^T A R),
      the value sum and the order-sensitive digest (helpers.digest) of R^T A R from the CPU oracle
      (oracle/spgemm_oracle.cpp, pinned to the reference at the fixture sizes). Every value is
      dyadic, so the device result must match bit for bit under any summation order.

CPU only (8 threads here: about a minute and 25 GB).
    python tests/golden/make_golden_fullsize.py
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import helpers as H  # noqa: E402

from combblas_amd.galerkin import poisson27_csc, prolongation_csc, transpose  # noqa: E402

NX = 256


def main():
    t0 = time.time()
    A, R = poisson27_csc(NX), prolongation_csc(NX)
    S = transpose(R)
    hA, hR, hS = (H.Dcsc(M.m, M.n, M.jc, M.cp, M.ir, M.num) for M in (A, R, S))
    del A, R, S
    O = H.Oracle()
    threads = len(os.sched_getaffinity(0))
    AT = O.spgemm(hA, hR, "plus_times", "hybrid", threads=threads)
    del hA
    SAT = O.spgemm(hS, AT, "plus_times", "hybrid", threads=threads)
    vsum, dig = H.digest(SAT)
    out = {"source": "tests/golden/make_golden_fullsize.py (CPU oracle, pinned to the reference at fixture sizes)",
           "galerkin": {"nx": NX, "nnzAT": int(AT.nnz), "nnzSAT": int(SAT.nnz), "sumSAT": float(vsum),
                        "digestSAT": str(dig)}}
    with open(os.path.join(HERE, "fullsize.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out), f"{time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
