#!/bin/bash
# One-launch Kselect + kept-stats prune check: the whole GPU suite, then the C5 line.
#   gpurun --timeout 900 -- bash tools/gpu_s3c.sh TAG
set -o pipefail
TAG=${1:-s3c}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
step() { echo "== $(date +%T) $*"; }
step "pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
step "C5 line"
timeout -k 10 600 python -u bench_mcl.py > "$OUT/bench_mcl.json" 2> "$OUT/bench_mcl.err" \
  || { tail -20 "$OUT/bench_mcl.err"; exit 1; }
cat "$OUT/bench_mcl.json"
step "rocprof C5"
cd /tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profmcl" -o run -- \
  python3 "$R/bench_mcl.py" --steps 2 --check-cols 20 > "$OUT/prof_mcl.json" 2> "$OUT/prof_mcl.err" \
  || { tail -20 "$OUT/prof_mcl.err"; exit 1; }
head -12 "$OUT/profmcl/run_kernel_stats.csv" | cut -c1-160
step done
