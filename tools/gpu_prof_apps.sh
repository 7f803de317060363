#!/bin/bash
# rocprofv3 kernel statistics of the application lines (C3 Galerkin, C5 MCL) on the shipped build.
#   gpurun -- bash tools/gpu_prof_apps.sh TAG [galerkin mcl]
set -o pipefail
TAG=${1:-profapps}
shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for app in ${@:-galerkin mcl}; do
  echo "== $(date +%T) rocprof bench_$app"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$app" -o run -- \
    python3 "$R/bench_$app.py" --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/$app.json" 2> "$OUT/$app.err" \
    || { tail -20 "$OUT/$app.err"; exit 1; }
  head -12 "$OUT/$app/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-150
done
