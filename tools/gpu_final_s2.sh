#!/bin/bash
# Round-2 session-2 measurement call: T=8192 A/B, the whole GPU suite, smoke, the default bench
# line (CPU baseline + merge sample), its rocprof kernel stats, per-bin PMC passes, the C4 line.
#   gpurun --timeout 1500 -- bash tools/gpu_final_s2.sh TAG
set -o pipefail
TAG=${1:-fs2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
step() { echo "== $(date +%T) $*"; }
step "t8k spgemm tests"
CBH_LIB=t8k timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 180 --timeout-method thread > "$OUT/pytest_t8k.log" 2>&1 \
  || { tail -30 "$OUT/pytest_t8k.log"; exit 1; }
tail -1 "$OUT/pytest_t8k.log"
for v in t8k base; do
  step "bench $v"
  if [ "$v" = base ]; then L=""; else L=$v; fi
  CBH_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/bench_ab_$v.json" 2> "$OUT/bench_ab_$v.err" \
    || { tail -20 "$OUT/bench_ab_$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_ab_$v.json')); print(d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['check']['ok'])"
done
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
step "per-bin PMC"
timeout -k 10 900 bash tools/gpu_bins.sh "$TAG/binsrun" 22 > "$OUT/bins.log" 2>&1 || { tail -20 "$OUT/bins.log"; exit 1; }
tail -3 "$OUT/bins.log"
step "C4 line"
timeout -k 10 600 python -u bench_tc.py --scale 24 --steps 2 --warmup 1 > "$OUT/bench_tc.json" 2> "$OUT/bench_tc.err" \
  || { tail -20 "$OUT/bench_tc.err"; exit 1; }
cat "$OUT/bench_tc.json"
step done
