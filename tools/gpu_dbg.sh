#!/bin/bash
# debug: phased product at increasing scales with per-launch diag, each step time-limited
set -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
shift
for s in "$@"; do
  echo "== scale $s" | tee -a "$OUT/dbg.log"
  CBH_DIAG=1 timeout -k 5 60 python -u tools/phase_timing.py $s 1 >> "$OUT/dbg.log" 2>&1
  rc=$?
  echo "rc=$rc" | tee -a "$OUT/dbg.log"
  [ $rc -ne 0 ] && break
done
grep -E "==|rc=|call|numeric dense" "$OUT/dbg.log" | tail -60
