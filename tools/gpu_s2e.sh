#!/bin/bash
# dot-form merge branch: apps tests, TC host check at 22, C4 line at 24.
set -o pipefail
TAG=${1:-s2e}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
echo "== $(date +%T) pytest apps"
timeout -k 10 400 python -u -m pytest tests/test_apps_gpu.py -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_apps.log" 2>&1 \
  || { tail -40 "$OUT/pytest_apps.log"; exit 1; }
tail -2 "$OUT/pytest_apps.log"
echo "== $(date +%T) TC debug 22"
timeout -k 10 300 python -u tools/tc_debug.py 22 > "$OUT/tcdebug.log" 2>&1 || { tail -20 "$OUT/tcdebug.log"; exit 1; }
cat "$OUT/tcdebug.log"
echo "== $(date +%T) bench_tc 24"
timeout -k 10 600 python -u bench_tc.py --scale 24 --steps 2 --warmup 1 > "$OUT/bench_tc.json" 2> "$OUT/bench_tc.err" \
  || { tail -20 "$OUT/bench_tc.err"; exit 1; }
cat "$OUT/bench_tc.json"
echo "== $(date +%T) done"
