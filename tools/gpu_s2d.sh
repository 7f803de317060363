#!/bin/bash
# C4 bench line (TC at scale 24) and its rocprof kernel trace.
set -o pipefail
TAG=${1:-s2d}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
echo "== $(date +%T) bench_tc 24"
timeout -k 10 600 python -u bench_tc.py --scale 24 --steps 2 --warmup 1 > "$OUT/bench_tc.json" 2> "$OUT/bench_tc.err" \
  || { tail -20 "$OUT/bench_tc.err"; exit 1; }
cat "$OUT/bench_tc.json"
tail -3 "$OUT/bench_tc.err"
cd /tmp || exit 1
echo "== $(date +%T) rocprof bench_tc"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$R/bench_tc.py" --scale 24 --steps 1 --warmup 0 --check-cols 10 --no-cpu-baseline > "$OUT/prof_tc.json" 2> "$OUT/prof_tc.err" \
  || { tail -20 "$OUT/prof_tc.err"; exit 1; }
head -12 "$OUT/prof/run_kernel_stats.csv" | cut -c1-200
echo "== $(date +%T) done"
