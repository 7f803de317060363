#!/bin/bash
# Quick GPU iteration: the whole -m gpu suite (or the tests named in $TESTS), then the default
# bench line without the CPU baseline, optionally the per-sub-bin timing (DIAG=scale).
#   gpurun -- bash tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
[ -n "$NOBENCH" ] && exit 0
echo "== $(date +%T) bench"
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ -n "$DIAG" ]; then
  echo "== $(date +%T) diag"
  CBH_DIAG=1 timeout -k 10 300 python -u tools/phase_timing.py "$DIAG" 2 > "$OUT/diag.log" 2>&1 || { tail -30 "$OUT/diag.log"; exit 1; }
  grep "cbh diag" "$OUT/diag.log" | tail -40
fi
