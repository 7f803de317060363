#!/bin/bash
# Environment sweep of the scale-SCALE phased product (tools/phase_timing.py, 2 calls each; the
# second call's time counts).   gpurun -- bash tools/gpu_envab.sh TAG SCALE "ENV=A" "ENV=B" ...
set -o pipefail
TAG=$1; SCALE=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for E in "BASE=1" "$@"; do
  i=$((i+1))
  echo "== $E"
  env $E PT_VERBOSE=1 timeout -k 10 240 python -u tools/phase_timing.py "$SCALE" 2 > "$OUT/v$i.log" 2>&1 || { tail -20 "$OUT/v$i.log"; exit 1; }
  grep -E "^call|^\{'sym" "$OUT/v$i.log" | tail -3 | cut -c1-300
done
