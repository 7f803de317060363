#!/bin/bash
# Round-2 confirmation call for the row-order-default build: the whole GPU suite, smoke, the
# default bench line, its rocprof kernel stats, and the C5 (MCL expansion + prune) line.
#   gpurun --timeout 1500 -- bash tools/gpu_final_s3.sh TAG
set -o pipefail
TAG=${1:-fs3}
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
step smoke
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
step "bench default"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
step "rocprof kernel stats"
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
  || { tail -20 "$OUT/prof.err"; exit 1; }
head -5 "$OUT/prof/run_kernel_stats.csv" | cut -c1-160
cd "$R" || exit 1
step "C5 line"
timeout -k 10 600 python -u bench_mcl.py > "$OUT/bench_mcl.json" 2> "$OUT/bench_mcl.err" \
  || { tail -20 "$OUT/bench_mcl.err"; exit 1; }
cat "$OUT/bench_mcl.json"
step done
