#!/bin/bash
# mid-size hash kernel A/B: spgemm GPU tests on the product build, then verified bench lines of the
# product (CBH_MIDCAP 1024) and the variants given (m256 = no mid bin, as before).
#   gpurun --timeout 900 -- bash tools/gpu_mid.sh TAG VARIANT [VARIANT ...]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
echo "== $(date +%T) pytest spgemm"
timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py tests/test_scale22_gpu.py tests/test_f64_rounding_gpu.py -x -q --timeout 180 --timeout-method thread > "$OUT/pytest.log" 2>&1 \
  || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for v in base "$@"; do
  if [ "$v" = base ]; then L=""; else L=$v; fi
  echo "== $(date +%T) bench $v"
  CBH_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" \
    || { tail -20 "$OUT/bench_$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print(d['value'], d['ms_per_step'], d['config']['kernel_ms'], d['roofline']['frac'], d['check']['ok'])"
done
echo "== $(date +%T) done"
