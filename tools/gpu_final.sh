#!/bin/bash
# End-of-round measurement of the shipped build: the whole GPU suite, smoke, per-bin PMC passes
# (-> profiles/pmc_*.json for roofline.traffic), the default bench line, its rocprof kernel stats,
# and the C5 and C3 lines. TESTS_ONLY=1: the suite and smoke only.
#   gpurun --timeout 1200 -- bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-fs3}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
step() { echo "== $(date +%T) $*"; }
# PART=2 runs only the application lines (C5, C3, C4), so the two halves fit one call each
if [ "${PART:-1}" = 2 ]; then
  for app in mcl mcl_cpp galerkin tc c1; do
    step "bench_$app"
    args=""
    [ "$app" = mcl_cpp ] && args="--driver cpp"
    timeout -k 10 700 python -u bench_${app%_cpp}.py $args > "$OUT/bench_$app.json" 2> "$OUT/bench_$app.err" || { tail -20 "$OUT/bench_$app.err"; exit 1; }
    tail -c 600 "$OUT/bench_$app.json"; echo
  done
  step done
  exit 0
fi
# SKIP_TESTS=1 starts at the PMC passes (the suite and smoke in a call of their own)
if [ -z "$SKIP_TESTS" ]; then
step "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
step smoke
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
[ -n "$TESTS_ONLY" ] && { step done; exit 0; }
fi
step "per-bin PMC"
timeout -k 10 900 bash tools/gpu_bins.sh "$TAG/binsrun" 22 > "$OUT/bins.log" 2>&1 || { tail -20 "$OUT/bins.log"; exit 1; }
for k in "1024, 512, 8, 163776, 0>:num_dense" "1024, 512, 8, 163776, 1>:sym_bmp" "2048, 512, 512, 4, 1, false>:num_large" "PlusTimesD<long>, 8192, 512, 512, 16, 0, false>:sym_large"; do
  python3 tools/pmc_traffic.py "$OUT/binsrun/bins" "${k%:*}" "profiles/pmc_${k##*:}.json" "tools/gpu_final.sh $TAG (shipped build)" > /dev/null || exit 1
done
mkdir -p "$OUT/pmcjson" && cp profiles/pmc_*.json "$OUT/pmcjson/"
step "bench default"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
step "rocprof kernel stats"
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
  || { tail -20 "$OUT/prof.err"; exit 1; }
head -6 "$OUT/prof/run_kernel_stats.csv" | cut -c1-160
cd "$R" || exit 1
[ -n "$NOAPPS" ] && { step done; exit 0; }
step "C5 line"
timeout -k 10 600 python -u bench_mcl.py > "$OUT/bench_mcl.json" 2> "$OUT/bench_mcl.err" || { tail -20 "$OUT/bench_mcl.err"; exit 1; }
cat "$OUT/bench_mcl.json"
step "C3 line"
timeout -k 10 600 python -u bench_galerkin.py > "$OUT/bench_galerkin.json" 2> "$OUT/bench_galerkin.err" || { tail -20 "$OUT/bench_galerkin.err"; exit 1; }
cat "$OUT/bench_galerkin.json"
step done
