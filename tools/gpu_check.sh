#!/bin/bash
# Parity + bench after a kernel change: all -m gpu tests (or a -k selection), then the bench
# line (no CPU baseline) and the per-kind kernel times.   gpurun -- bash tools/gpu_check.sh TAG [PYTEST_K]
set -o pipefail
TAG=${1:-chk}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
echo "== $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread "${KARG[@]}" > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
echo "== $(date +%T) bench"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['roofline']['frac'], d['check']['ok'])"
