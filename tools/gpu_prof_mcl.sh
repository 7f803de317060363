#!/bin/bash
# rocprofv3 kernel statistics of the C5 line through both host paths (python mirror, C++ overload).
#   gpurun --timeout 900 -- bash tools/gpu_prof_mcl.sh TAG
set -o pipefail
TAG=${1:-profmcl}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
for drv in ${DRVS:-cpp python}; do
  echo "== $(date +%T) rocprof bench_mcl --driver $drv"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$drv" -o run -- \
    python3 "$R/bench_mcl.py" --driver $drv --steps 2 --warmup 1 --no-cpu-baseline --check-cols 10 > "$OUT/$drv.json" 2> "$OUT/$drv.err" \
    || { tail -20 "$OUT/$drv.err"; exit 1; }
  head -16 "$OUT/$drv/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-150
done
