#!/bin/bash
# MCL prune parity tests + the C5 line through both host paths (after a change to the prune kernels).
#   gpurun --timeout 900 -- bash tools/gpu_mcl_check.sh TAG
set -o pipefail
TAG=${1:-mclchk}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== $(date +%T) pytest (apps, fallbacks, apps_dist)"
timeout -k 10 500 python -u -m pytest tests/test_apps_gpu.py tests/test_fallbacks_gpu.py tests/test_apps_dist_gpu.py -m gpu -x -q \
  --timeout 180 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for drv in cpp python; do
  echo "== $(date +%T) bench_mcl --driver $drv"
  timeout -k 10 400 python -u bench_mcl.py --driver $drv --no-cpu-baseline > "$OUT/mcl_$drv.json" 2> "$OUT/mcl_$drv.err" \
    || { tail -20 "$OUT/mcl_$drv.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['check'])" "$OUT/mcl_$drv.json"
done
