#!/bin/bash
# TC dot-form check: apps GPU tests, then timing over scales, then a kernel trace at the largest.
#   gpurun -- bash tools/gpu_tc.sh TAG "16 18 20 22 24"
set -o pipefail
TAG=${1:-tc}
SCALES=${2:-"16 18 20 22"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
echo "== pytest apps"
timeout -k 10 400 python -u -m pytest tests/test_apps_gpu.py -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_apps.log" 2>&1 \
  || { tail -40 "$OUT/pytest_apps.log"; exit 1; }
tail -2 "$OUT/pytest_apps.log"
echo "== timing"
timeout -k 10 500 python -u tools/tc_timing.py $SCALES > "$OUT/timing.log" 2>&1 || { tail -20 "$OUT/timing.log"; exit 1; }
cat "$OUT/timing.log"
echo done
