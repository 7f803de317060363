#!/usr/bin/env python3
"""Regenerates the golden fixtures in tests/golden/ FROM THE REFERENCE ITSELF.

Runs oracle/_ref/ref_harness (the reference's LocalHybridSpGEMM / LocalSpGEMMHash / LocalSpGEMM /
MultiwayMerge and its Graph500 generator, compiled from /root/reference by `make -C oracle ref`)
on small deterministic inputs and stores inputs + outputs (small cases) or digests (larger
cases). Needs the reference checkout; the GPU box only reads the committed fixtures.

    python tests/golden/make_golden.py            # writes tests/golden/*.npz + golden.json
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import helpers as H  # noqa: E402

REF = os.path.join(H.REPO, "oracle", "_ref", "ref_harness")
REFDIR = os.environ.get("COMBBLAS_REF", "/root/reference")
TMP = tempfile.mkdtemp(prefix="cbgold_")


def run(*args):
    subprocess.check_call([REF, *map(str, args)], cwd=TMP, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


def gen(scale, ef=16):
    p = os.path.join(TMP, f"g{scale}.cbm")
    if not os.path.exists(p):
        run("gen", scale, ef, p)
    return H.read_cbm(p)


def ref_mult(sr, kernel, A, B, tag):
    pa, pb, pc = (os.path.join(TMP, f"{tag}_{x}.cbm") for x in "ABC")
    H.write_cbm(pa, A)
    H.write_cbm(pb, B)
    run("mult", sr, kernel, pa, pb, pc)
    return H.read_cbm(pc)


def ref_merge(sr, lists, tag):
    ins = []
    for i, d in enumerate(lists):
        p = os.path.join(TMP, f"{tag}_in{i}.cbm")
        H.write_cbm(p, d)
        ins.append(p)
    out = os.path.join(TMP, f"{tag}_out.cbm")
    run("merge", sr, out, *ins)
    return H.read_cbm(out)


values_for = H.values_for


def read_triples(path, one_based=True, header_lines=1):
    rows, cols, vals = [], [], []
    with open(path) as f:
        lines = [l for l in f if not l.startswith("%")]
    m, n = map(int, lines[0].split()[:2])
    for l in lines[header_lines:]:
        t = l.split()
        if len(t) < 2:
            continue
        rows.append(int(t[0]) - one_based)
        cols.append(int(t[1]) - one_based)
        vals.append(float(t[2]) if len(t) > 2 else 1.0)
    return H.Dcsc.from_coo(m, n, rows, cols, np.array(vals, np.float64))


def main():
    meta = {"generator": {}, "digests": {}, "source": "oracle/_ref/ref_harness built from " + REFDIR}
    full = {}
    # ---- generator pins (reference packed Graph500 generator, ef 16, removeloops=false)
    for s in (8, 10, 12, 14):
        A = gen(s)
        vs, dg = H.digest(A)
        meta["generator"][str(s)] = {"nnz": A.nnz, "nzc": A.nzc, "sum": vs, "digest": str(dg)}
    # ---- full outputs, small R-MAT A^2 for every semiring (LocalHybridSpGEMM)
    for s in (6, 8):
        base = gen(s)
        for sr in ("pt_f64", "pt_i64", "max_i64", "min_i64", "bool"):
            A = values_for(sr, base)
            C = ref_mult(sr, "hybrid", A, A, f"r{s}{sr}")
            full[f"rmat{s}_{sr}_A"] = A
            full[f"rmat{s}_{sr}_C"] = C
    # ---- kernel variants (same numeric contract; hashu = unsorted rows)
    A = values_for("pt_i64", gen(8))
    for k in ("hash", "hashu", "heap"):
        full[f"rmat8_pt_i64_{k}_C"] = ref_mult("pt_i64", k, A, A, f"k{k}")
    # ---- explicit zeros flow through (TC.cpp's zeroed lower triangle)
    Az = H.with_explicit_zeros(values_for("pt_i64", gen(8)))
    full["zeros8_A"] = Az
    full["zeros8_C"] = ref_mult("pt_i64", "hybrid", Az, Az, "zeros")
    # ---- rectangular: A (256x256) * B (256x40)
    A = values_for("pt_f64", gen(8))
    Bc = A.col_slice(0, 40)
    B = H.Dcsc(A.m, 40, Bc.jc, Bc.cp, Bc.ir, Bc.num)
    full["rect8_A"], full["rect8_B"] = A, B
    full["rect8_C"] = ref_mult("pt_f64", "hybrid", A, B, "rect")
    # ---- reference data files (largeseq, ReleaseTests, 3DSpGEMM/matlab)
    L1 = read_triples(os.path.join(REFDIR, "largeseq", "input1_0"))
    L2 = read_triples(os.path.join(REFDIR, "largeseq", "input2_0"))
    full["largeseq_A"], full["largeseq_B"] = L1, L2
    full["largeseq_C"] = ref_mult("pt_f64", "hybrid", L1, L2, "largeseq")
    for name, path in (("sevenvertex", "ReleaseTests/sevenvertex.mtx"), ("small_nonsym", "ReleaseTests/small_nonsym.mtx"),
                       ("bcsstk01", "3DSpGEMM/matlab/bcsstk01.mtx")):
        M = read_triples(os.path.join(REFDIR, path))
        full[f"{name}_A"] = M
        full[f"{name}_C"] = ref_mult("pt_f64", "hybrid", M, M, name)
    # ---- MultiwayMerge of SUMMA-like partials: A*B = sum_k A(:,Kk) * B(Kk,:)
    for sr in ("pt_i64", "pt_f64", "max_i64"):
        A = values_for(sr, gen(8))
        n = A.n
        for parts in (2, 3):
            cuts = [n * i // parts for i in range(parts + 1)]
            P = [ref_mult(sr, "hybrid", A.col_slice(cuts[i], cuts[i + 1]), A.row_slice(cuts[i], cuts[i + 1]),
                          f"mp{sr}{parts}{i}") for i in range(parts)]
            M = ref_merge(sr, P, f"mg{sr}{parts}")
            for i, p in enumerate(P):
                full[f"merge{parts}_{sr}_P{i}"] = p
            full[f"merge{parts}_{sr}_M"] = M
    H.save_npz(os.path.join(HERE, "fixtures.npz"), **full)
    # ---- digests of larger products (reference LocalHybridSpGEMM on the reference generator)
    for s in (10, 12):
        base = gen(s)
        for sr in ("pt_f64", "pt_i64", "max_i64", "min_i64", "bool"):
            A = values_for(sr, base)
            C = ref_mult(sr, "hybrid", A, A, f"d{s}{sr}")
            vs, dg = H.digest(C)
            meta["digests"][f"rmat{s}_{sr}"] = {"nnz": C.nnz, "nzc": C.nzc, "sum": vs, "digest": str(dg)}
    for s in (14, 16):
        A = values_for("pt_i64", gen(s))
        C = ref_mult("pt_i64", "hybrid", A, A, f"d{s}")
        vs, dg = H.digest(C)
        meta["digests"][f"rmat{s}_pt_i64"] = {"nnz": C.nnz, "nzc": C.nzc, "sum": vs, "digest": str(dg)}
        del C
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "fixtures.npz"), os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
