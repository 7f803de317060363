#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, kernel-trace profile.
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh [tag] [steps]
# Every GPU step has its own time limit; the first failure ends the script.
set -e -o pipefail
TAG=${1:-r01}
STEPS=${2:-3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
echo "== smoke"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "== bench"
timeout -k 10 400 python -u bench.py --steps "$STEPS" --warmup 1 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "== rocprofv3 kernel trace"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-verify > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err" \
  || { tail -20 "$GRAFT_REPO_ROOT/$OUT/prof.err"; exit 1; }
cd "$GRAFT_REPO_ROOT"
find "$OUT/prof" -name '*stats*'
echo done
