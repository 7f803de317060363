#!/bin/bash
# Session-2 check: full GPU tests, TC dot-form timing over scales, quick bench (no CPU baseline).
#   gpurun -- bash tools/gpu_s2.sh TAG "16 18 20 22 24"
set -o pipefail
TAG=${1:-s2}
SCALES=${2:-"16 18 20 22"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
echo "== $(date +%T) pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
echo "== $(date +%T) bench (quick)"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "== $(date +%T) TC timing"
timeout -k 10 400 python -u tools/tc_timing.py $SCALES > "$OUT/timing.log" 2>&1 || { tail -20 "$OUT/timing.log"; exit 1; }
cat "$OUT/timing.log"
echo "== $(date +%T) done"
