#!/bin/bash
# row-order A/B (CBH_ROWORDER=1: tasks of a bin launch in row-block order) and the C3 line.
set -o pipefail
TAG=${1:-s2l}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
for v in 0 1; do
  echo "== $(date +%T) bench CBH_ROWORDER=$v"
  CBH_ROWORDER=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/bench_ro$v.json" 2> "$OUT/bench_ro$v.err" \
    || { tail -20 "$OUT/bench_ro$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_ro$v.json')); print(d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['check']['ok'])"
done
echo "== $(date +%T) C3 line"
timeout -k 10 900 python -u bench_galerkin.py --nx 256 --steps 3 --warmup 1 > "$OUT/bench_galerkin.json" 2> "$OUT/bench_galerkin.err" \
  || { tail -20 "$OUT/bench_galerkin.err"; exit 1; }
cat "$OUT/bench_galerkin.json"
tail -3 "$OUT/bench_galerkin.err"
echo "== $(date +%T) done"
