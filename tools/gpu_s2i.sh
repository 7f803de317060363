#!/bin/bash
# owner-search sweep variant (os1): spgemm/scale-22 GPU tests on it, then bench A/B.
set -o pipefail
TAG=${1:-s2i}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
echo "== $(date +%T) pytest spgemm on os1"
CBH_LIB=os1 timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py tests/test_convert_gpu.py -x -q --timeout 180 --timeout-method thread > "$OUT/pytest_os1.log" 2>&1 \
  || { tail -40 "$OUT/pytest_os1.log"; exit 1; }
tail -2 "$OUT/pytest_os1.log"
for v in base os1; do
  echo "== $(date +%T) bench $v"
  if [ "$v" = base ]; then L=""; else L=$v; fi
  CBH_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" \
    || { tail -20 "$OUT/bench_$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['roofline']['kernel'][-12:], d['roofline']['frac'], d['check']['ok'])"
done
echo "== $(date +%T) done"
