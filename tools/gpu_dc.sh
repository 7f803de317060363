#!/bin/bash
# direct-from-table hash commit A/B: spgemm GPU tests on the variant, then verified bench lines.
#   gpurun --timeout 900 -- bash tools/gpu_dc.sh TAG VARIANT
set -o pipefail
TAG=$1; V=$2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
echo "== $(date +%T) pytest spgemm on $V"
CBH_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py tests/test_scale22_gpu.py tests/test_f64_rounding_gpu.py tests/test_apps_gpu.py tests/test_convert_gpu.py -x -q --timeout 180 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in base $V base $V; do
  if [ "$v" = base ]; then L=""; else L=$v; fi
  echo "== $(date +%T) bench $v"
  CBH_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" \
    || { tail -20 "$OUT/bench_$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['roofline']['frac'], d['check']['ok'])"
done
echo "== $(date +%T) done"
