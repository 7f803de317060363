#!/bin/bash
# dot-form variants: apps tests + TC 22 check on the product build, then C4 timing per variant.
set -o pipefail
TAG=${1:-s2h}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
echo "== $(date +%T) pytest apps"
timeout -k 10 400 python -u -m pytest tests/test_apps_gpu.py -x -v --timeout 180 --timeout-method thread > "$OUT/pytest_apps.log" 2>&1 \
  || { tail -40 "$OUT/pytest_apps.log"; exit 1; }
tail -2 "$OUT/pytest_apps.log"
echo "== $(date +%T) TC debug 22"
timeout -k 10 300 python -u tools/tc_debug.py 22 > "$OUT/tcdebug.log" 2>&1 || { tail -20 "$OUT/tcdebug.log"; exit 1; }
cat "$OUT/tcdebug.log"
for v in base i0 a3 m16 m4; do
  echo "== $(date +%T) bench_tc $v"
  if [ "$v" = base ]; then L=""; else L=$v; fi
  CBH_LIB=$L timeout -k 10 300 python -u bench_tc.py --scale 24 --steps 1 --warmup 1 --check-cols 20 --no-cpu-baseline > "$OUT/tc_$v.json" 2> "$OUT/tc_$v.err" \
    || { tail -20 "$OUT/tc_$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/tc_$v.json')); print(d['ms_per_step'], d['check']['digest'], d['check']['ok'])"
done
echo "== $(date +%T) done"
