#!/bin/bash
# One GPU call of a working session: the -m gpu suite on the product build (TESTS= narrows it,
# NOTESTS=1 skips it), then a bench A/B over the given settings (tools/gpu_ab.sh; "" = product).
#   gpurun --timeout 1200 -- bash tools/gpu_session.sh TAG "" "CBH_LIB=variant" ...
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
  echo "== $(date +%T) pytest"
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
[ $# -gt 0 ] || exit 0
echo "== $(date +%T) A/B"
bash tools/gpu_ab.sh "$TAG" "$@"
