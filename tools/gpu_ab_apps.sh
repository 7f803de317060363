#!/bin/bash
# A/B of runtime switches / library variants on an application line (C3 galerkin, C5 mcl):
# one run per argument (space-separated VAR=value settings), 2 timed steps, no CPU baseline.
#   gpurun -- bash tools/gpu_ab_apps.sh TAG mcl "CBH_LIB=" "CBH_LIB=mid8"
set -o pipefail
TAG=$1
APP=$2
shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 ${APP_TIMEOUT:-400} python -u bench_$APP.py --steps 2 --warmup 1 --no-cpu-baseline \
    > "$OUT/$APP$i.json" 2> "$OUT/$APP$i.err" || { echo "[$cfg] failed"; tail -20 "$OUT/$APP$i.err"; exit 1; }
  python3 - "$OUT/$APP$i.json" "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"[{sys.argv[2]}] {d['value']} {d['unit']}, {d['ms_per_step']} ms, ok {d['check'].get('ok')}", flush=True)
PY
done
