#!/bin/bash
# Iteration loop on the GPU box: parity tests, bench (no CPU baseline), stamped sub-bin shares.
#   gpurun -- bash tools/gpu_iter.sh TAG [DIAG_SCALE] [extra env for bench, e.g. CBH_TASK_FLOPS=32768]
set -e -o pipefail
TAG=${1:-iter}
SD=${2:-20}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('VALUE',d['value'],'ms',d['ms_per_step'],d['config']['kernel_ms'],d['check'])"
CBH_LIB=stamps CBH_DIAG=1 timeout -k 10 300 python -u tools/phase_timing.py "$SD" 1 > "$OUT/stamps.log" 2>&1 || { tail -30 "$OUT/stamps.log"; exit 1; }
grep -E "cbh (diag|stamps)" "$OUT/stamps.log" | head -60
