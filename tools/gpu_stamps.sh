#!/bin/bash
# Per-phase cycle shares of the task kernels (diagnostic build), per work sub-bin.
set -e -o pipefail
TAG=${1:-stamps}
SD=${2:-20}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
CBH_LIB=stamps CBH_DIAG=1 timeout -k 10 300 python -u tools/phase_timing.py "$SD" 1 > "$OUT/stamps.log" 2>&1 || { tail -30 "$OUT/stamps.log"; exit 1; }
grep -E "cbh (diag|stamps)" "$OUT/stamps.log" | head -60
