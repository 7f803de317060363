#!/bin/bash
# LDS-staged merge rounds of the dot form (apps tests, TC 22 host check, C4 at 24), then the
# fill / dense-ratio A/B of the A^2 product.
set -o pipefail
TAG=${1:-s2f}
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
echo "== $(date +%T) bench_tc 24"
timeout -k 10 600 python -u bench_tc.py --scale 24 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_tc.json" 2> "$OUT/bench_tc.err" \
  || { tail -20 "$OUT/bench_tc.err"; exit 1; }
cat "$OUT/bench_tc.json"
for v in base f3 f5 dr4; do
  echo "== $(date +%T) bench $v"
  if [ "$v" = base ]; then L=""; else L=$v; fi
  CBH_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" \
    || { tail -20 "$OUT/bench_$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['roofline']['kernel'][-12:], d['roofline']['frac'], d['check']['ok'])"
done
echo "== $(date +%T) done"
