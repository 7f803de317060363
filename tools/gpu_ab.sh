#!/bin/bash
# A/B of runtime switches on the default bench line: one bench run (3 timed steps, no CPU baseline,
# no merge sample) per argument, each argument a space-separated list of VAR=value settings.
#   gpurun -- bash tools/gpu_ab.sh TAG "" "CBH_LIB=h2048"   (product vs a build variant, combblas_amd/build.py --variant)
set -o pipefail
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/ab$i.json" 2> "$OUT/ab$i.err" \
    || { echo "[$cfg] failed"; tail -20 "$OUT/ab$i.err"; exit 1; }
  python3 - "$OUT/ab$i.json" "$cfg" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = d["config"]["kernel_ms"]
print(f"[{sys.argv[2]}] {d['value']} GFLOP/s, {d['ms_per_step']} ms, phases {d['config']['phases']}, ok {d['check']['ok']}, "
      + ", ".join(f"{n} {v:.1f}" for n, v in k.items() if v > 0.5))
PY
done
