#!/bin/bash
# Application lines (C3/C4/C5) on the shipped build; each step time-limited, stops at the first failure.
#   gpurun --timeout 1200 -- bash tools/gpu_apps.sh TAG [mcl galerkin tc]
set -o pipefail
TAG=${1:-apps}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for app in "${@:-mcl galerkin tc}"; do
  for a in $app; do
    echo "== $(date +%T) bench_$a ${BENCH_ARGS}"
    timeout -k 10 ${APP_TIMEOUT:-500} python -u bench_$a.py ${BENCH_ARGS} > "$OUT/bench_$a.json" 2> "$OUT/bench_$a.err" \
      || { tail -30 "$OUT/bench_$a.err"; exit 1; }
    cat "$OUT/bench_$a.json"
  done
done
