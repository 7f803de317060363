#!/usr/bin/env python3
"""Regenerates tests/golden/tc.json FROM THE REFERENCE ITSELF: Applications/TC.cpp's flow
(ref_harness tc <scale>: R-MAT, RemoveLoops, A += A', values 1, L = GetLowerTriangular with the
upper entries kept as explicit zeros, C = Mult_AnXBn_Synch(L, L).EWiseMult(L, false)) at the
scales the reference finishes on this container (12, 14, 16; scale 18's unmasked L*L exhausts
its 64 GB). Per scale: triangles, nnz(L), and nnz / nonzero columns / value sum / order-sensitive
digest (tests/helpers.digest) of C. The GPU tests compare both masked forms (expand and dot)
against these; tests/golden/apps.npz keeps the whole L and C at scales 8 and 10.

Needs oracle/_ref/ref_harness (make -C oracle ref); the GPU box only reads the committed file.
    python tests/golden/make_golden_tc.py
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import helpers as H  # noqa: E402

REF = os.path.join(H.REPO, "oracle", "_ref", "ref_harness")


def main():
    out = {"source": "oracle/_ref/ref_harness tc <scale> (built from the reference sources)", "scales": {}}
    with tempfile.TemporaryDirectory() as d:
        for s in (12, 14, 16):
            L, C = os.path.join(d, f"L{s}.cbm"), os.path.join(d, f"C{s}.cbm")
            res = subprocess.run([REF, "tc", str(s), L, C], cwd=d, check=True, capture_output=True, text=True).stdout
            meta = json.loads([l for l in res.splitlines() if l.startswith("{")][-1])
            c = H.read_cbm(C)
            vs, dg = H.digest(c)
            meta.update(nzcC=int(c.nzc), sumC=float(vs), digestC=str(dg))
            assert meta["nnzC"] == c.nnz and int(c.num.sum()) == meta["triangles"]
            out["scales"][str(s)] = meta
            print(s, meta, flush=True)
    with open(os.path.join(HERE, "tc.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
