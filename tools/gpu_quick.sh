#!/bin/bash
# Quick GPU iteration: parity tests, bench without CPU baseline, sub-bin timing.
#   gpurun -- bash tools/gpu_quick.sh TAG [SCALE_DIAG]
set -e -o pipefail
TAG=${1:-quick}
SD=${2:-20}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
CBH_DIAG=1 timeout -k 10 300 python -u tools/phase_timing.py "$SD" 2 > "$OUT/diag.log" 2>&1 || { tail -30 "$OUT/diag.log"; exit 1; }
grep "cbh diag" "$OUT/diag.log" | tail -40
