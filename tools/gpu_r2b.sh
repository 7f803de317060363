#!/bin/bash
# Round-2 GPU iteration with an environment A/B: parity, bench (product), bench (env A/B), diag.
#   gpurun -- bash tools/gpu_r2b.sh TAG "ENV=VAL ..." [PYTEST_K]
set -e -o pipefail
TAG=${1:-r2}
ABENV=${2:-}
K=${3:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ -n "$ABENV" ]; then
  env $ABENV timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify > "$OUT/bench_ab.json" 2> "$OUT/bench_ab.err" || { tail -20 "$OUT/bench_ab.err"; exit 1; }
  cat "$OUT/bench_ab.json"
fi
CBH_DIAG=1 timeout -k 10 300 python -u tools/phase_timing.py 22 2 > "$OUT/diag.log" 2>&1 || { tail -30 "$OUT/diag.log"; exit 1; }
grep -E "cbh diag|call" "$OUT/diag.log" | tail -40
