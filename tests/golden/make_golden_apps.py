#!/usr/bin/env python3
"""Regenerates tests/golden/apps.npz + apps.json FROM THE REFERENCE ITSELF: the callers around the
SpGEMM hot path that BASELINE.json's configs C3-C5 exercise.

  TC (C4)        ref_harness tc <scale>: Applications/TC.cpp's flow on one rank -> L (with the
                 explicit zeros of GetLowerTriangular), C = (L*L) .* L, triangle count
  MCL (C5)       the expanded matrix A2 = Mult_AnXBn_Synch(A, A) of a column-stochastic
                 planted-partition graph (combblas_amd.mclgen), then MCLPruneRecoverySelect
                 (ParFriends.h:185-353) for two parameter sets chosen so that the recovery,
                 selection and post-selection recovery branches all fire
  Galerkin (C3)  GalerkinNew.cpp:100-106: AT = A*T, SAT = S*AT with S = T' on the 27-point
                 Poisson operator and trilinear prolongation (combblas_amd.galerkin), 8^3 grid

Needs oracle/_ref/ref_harness (make -C oracle ref); the GPU box only reads the committed files.
    python tests/golden/make_golden_apps.py
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import helpers as H  # noqa: E402

REF = os.path.join(H.REPO, "oracle", "_ref", "ref_harness")
TMP = tempfile.mkdtemp(prefix="cbapps_")

MCL_N, MCL_DEG, MCL_SEED = 1024, 24, 7
MCL_PARAMS = [(0.008, 15, 40, 0.8), (0.005, 25, 40, 0.9)]
GALERKIN_NX = 8


def run(*args):
    out = subprocess.run([REF, *map(str, args)], cwd=TMP, check=True, capture_output=True, text=True).stdout
    lines = [l for l in out.splitlines() if l.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def p(name):
    return os.path.join(TMP, name)


def d_of(h):
    return H.Dcsc(h.m, h.n, h.jc, h.cp, h.ir, h.num)


def synch(sr, A, B, tag):
    H.write_cbm(p(tag + "_A.cbm"), A)
    H.write_cbm(p(tag + "_B.cbm"), B)
    run("synch", sr, p(tag + "_A.cbm"), p(tag + "_B.cbm"), p(tag + "_C.cbm"))
    return H.read_cbm(p(tag + "_C.cbm"))


def main():
    from combblas_amd.galerkin import poisson27, prolongation, transpose
    from combblas_amd.mclgen import planted_partition

    full, meta = {}, {"source": "oracle/_ref/ref_harness built from the reference sources", "tc": {}, "mcl": {}}
    for s in (8, 10):
        r = run("tc", s, p(f"L{s}.cbm"), p(f"C{s}.cbm"))
        full[f"tc{s}_L"] = H.read_cbm(p(f"L{s}.cbm"))
        full[f"tc{s}_C"] = H.read_cbm(p(f"C{s}.cbm"))
        meta["tc"][str(s)] = r
    A = d_of(planted_partition(MCL_N, MCL_DEG, MCL_SEED))
    A2 = synch("pt_f64", A, A, "mcl")
    full["mcl_A"], full["mcl_A2"] = A, A2
    H.write_cbm(p("mcl_A2.cbm"), A2)
    for i, (hard, sel, rec, pct) in enumerate(MCL_PARAMS):
        run("mcl", p("mcl_A2.cbm"), p(f"mcl_out{i}.cbm"), repr(hard), sel, rec, repr(pct))
        full[f"mcl_out{i}"] = H.read_cbm(p(f"mcl_out{i}.cbm"))
        meta["mcl"][str(i)] = {"hard": hard, "select": sel, "recover": rec, "pct": pct, "nnz": full[f"mcl_out{i}"].nnz}
    meta["mcl"]["input"] = {"n": MCL_N, "avg_deg": MCL_DEG, "seed": MCL_SEED}
    Ag, T = d_of(poisson27(GALERKIN_NX)), d_of(prolongation(GALERKIN_NX))
    S = d_of(transpose(prolongation(GALERKIN_NX)))
    AT = synch("pt_f64", Ag, T, "gAT")
    SAT = synch("pt_f64", S, AT, "gSAT")
    full.update(gal_A=Ag, gal_T=T, gal_S=S, gal_AT=AT, gal_SAT=SAT)
    meta["galerkin"] = {"nx": GALERKIN_NX, "nnzAT": AT.nnz, "nnzSAT": SAT.nnz}
    H.save_npz(os.path.join(HERE, "apps.npz"), **full)
    with open(os.path.join(HERE, "apps.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
