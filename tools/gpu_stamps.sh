#!/bin/bash
# per-sub-bin kernel phase cycle shares of a diagnostic build (CBH_STAMPS)
#   gpurun -- bash tools/gpu_stamps2.sh TAG VARIANT SCALE
set -e -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
CBH_LIB=$2 CBH_DIAG=1 timeout -k 10 300 python -u tools/phase_timing.py ${3:-22} 2 > "$OUT/stamps.log" 2>&1 || { tail -30 "$OUT/stamps.log"; exit 1; }
grep -E "cbh diag|cbh stamps|call" "$OUT/stamps.log" | tail -60
