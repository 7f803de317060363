#!/bin/bash
# TC (C4) parity tests on the product build, then bench_tc.py A/B over the given settings.
#   gpurun --timeout 900 -- bash tools/gpu_tc_ab.sh TAG "" "CBH_LIB=variant"
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== $(date +%T) TC tests"
timeout -k 10 600 python -u -m pytest tests/test_apps_gpu.py tests/test_fullsize_gpu.py -m gpu -x -q -k "tc or dot or mask or c4 or triangle" \
  --timeout 180 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 400 python -u bench_tc.py --no-cpu-baseline > "$OUT/tc$i.json" 2> "$OUT/tc$i.err" || { tail -20 "$OUT/tc$i.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], d['check'])" "$OUT/tc$i.json" "[$cfg]"
done
