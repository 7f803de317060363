#!/usr/bin/env python3
"""Pins the WHOLE scale-22 R-MAT A^2 (BASELINE config C2) to the reference itself.

Runs `oracle/_ref/ref_harness digest 22 16 65536 <sr>` -- the reference's own LocalHybridSpGEMM
(mtSpGEMM.h:212-460, compiled from /root/reference by `make -C oracle ref`) over all 64 column
blocks of B = A, entries visited in C order with a running global index -- for PlusTimes<int64>
and PlusTimes<double>, and writes tests/golden/scale22.json:
  total: nnz, value sum, order-sensitive digest of the whole C (tests/helpers.py digest())
  blocks: the same per 65,536-column block (gbase = global index of the block's first entry)
The GPU tests compare cbh_spgemm_phased(..., CBH_PHASE_CHECKSUM) against these numbers; the GPU
box never runs the reference. Takes ~15 min per semiring on 8 cores, ~12 GB of host memory.

    python tests/golden/make_golden_s22.py [scale] [block]
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref", "ref_harness")


def run(scale, block, sr):
    env = dict(os.environ, LD_LIBRARY_PATH="/usr/lib/x86_64-linux-gnu:/opt/conda/lib")
    out = subprocess.run([REF, "digest", str(scale), "16", str(block), sr], env=env, cwd="/tmp", check=True,
                         capture_output=True, text=True).stdout
    blocks, total = [], None
    for line in out.splitlines():
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if d.get("total"):
            total = {"nnz": d["nnz"], "sum": d["sum"], "digest": d["digest"]}
        else:
            blocks.append({k: d[k] for k in ("block", "gbase", "nnz", "sum", "digest")})
    assert total is not None, out[-2000:]
    return {"total": total, "blocks": blocks}


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    block = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    path = os.path.join(HERE, f"scale{scale}.json")
    meta = json.load(open(path)) if os.path.exists(path) else {}
    meta.update({"scale": scale, "edgefactor": 16, "block": block,
                 "source": "oracle/_ref/ref_harness digest (reference LocalHybridSpGEMM, mtSpGEMM.h:212-460)"})
    for sr in ("pt_i64", "pt_f64"):
        meta[sr] = run(scale, block, sr)
        with open(path, "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        print(sr, meta[sr]["total"], flush=True)


if __name__ == "__main__":
    main()
