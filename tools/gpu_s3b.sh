#!/bin/bash
# Measurement of the 3072-value dense build: per-bin PMC passes, the default bench line (with the
# new PMC traffic), its rocprof kernel stats, and the rocprof kernel stats of the C5 line.
#   gpurun --timeout 1200 -- bash tools/gpu_s3b.sh TAG
set -o pipefail
TAG=${1:-s3b}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
step() { echo "== $(date +%T) $*"; }
step "per-bin PMC"
timeout -k 10 900 bash tools/gpu_bins.sh "$TAG/binsrun" 22 > "$OUT/bins.log" 2>&1 || { tail -20 "$OUT/bins.log"; exit 1; }
tail -3 "$OUT/bins.log"
for k in "4096, 512, 512, 8, 2, false>:num_dense" "4096, 512, 512, 8, 1, false>:num_large" "PlusTimesD<long>, 8192, 512, 512, 8, 0, false>:sym_large"; do
  python3 tools/pmc_traffic.py "$OUT/binsrun/bins" "${k%:*}" "profiles/pmc_${k##*:}.json" "tools/gpu_s3b.sh $TAG (round 2 session 3)" > /dev/null || exit 1
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
head -5 "$OUT/prof/run_kernel_stats.csv" | cut -c1-160
step "rocprof C5"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profmcl" -o run -- \
  python3 "$R/bench_mcl.py" --steps 2 --check-cols 20 > "$OUT/prof_mcl.json" 2> "$OUT/prof_mcl.err" \
  || { tail -20 "$OUT/prof_mcl.err"; exit 1; }
head -16 "$OUT/profmcl/run_kernel_stats.csv" | cut -c1-200
step done
