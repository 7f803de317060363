#!/bin/bash
# C4 line on the shipped build and the rocprof kernel stats of the C3 line.
#   gpurun --timeout 900 -- bash tools/gpu_s3d.sh TAG
set -o pipefail
TAG=${1:-s3d}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
echo "== $(date +%T) C4 line"
timeout -k 10 600 python -u bench_tc.py --scale 24 --steps 2 --warmup 1 > "$OUT/bench_tc.json" 2> "$OUT/bench_tc.err" \
  || { tail -20 "$OUT/bench_tc.err"; exit 1; }
cat "$OUT/bench_tc.json"
echo "== $(date +%T) rocprof C3"
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profgal" -o run -- \
  python3 "$R/bench_galerkin.py" --no-oracle > "$OUT/prof_gal.json" 2> "$OUT/prof_gal.err" || { tail -20 "$OUT/prof_gal.err"; exit 1; }
head -8 "$OUT/profgal/run_kernel_stats.csv" | cut -c1-160
echo "== $(date +%T) done"
