#!/bin/bash
# dot-form prefetching merge: apps tests, TC 22 host check, C4 at 24 with a kernel trace.
set -o pipefail
TAG=${1:-s2g}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
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
cd /tmp || exit 1
echo "== $(date +%T) rocprof bench_tc"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$R/bench_tc.py" --scale 24 --steps 1 --warmup 0 --check-cols 10 --no-cpu-baseline > "$OUT/prof_tc.json" 2> "$OUT/prof_tc.err" \
  || { tail -20 "$OUT/prof_tc.err"; exit 1; }
head -6 "$OUT/prof/run_kernel_stats.csv" | cut -c1-200
echo "== $(date +%T) done"
