#!/bin/bash
# A/B of runtime settings on the GPU box: optional parity tests under the first setting, then the
# scale-SCALE product under each setting ("-" = defaults), kernel_ms per setting.
#   gpurun -- bash tools/gpu_ab.sh TAG SCALE TESTS(0|1) 'CBH_NUMCFG=1' '-' ...
set -e -o pipefail
TAG=${1:-ab}
SC=${2:-22}
TESTS=${3:-0}
shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for E in "$@"; do
  i=$((i+1))
  [ "$E" = "-" ] && E=""
  if [ "$TESTS" = 1 ] && [ $i = 1 ]; then
    env $E timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/pytest_$i.log" 2>&1 \
      || { tail -40 "$OUT/pytest_$i.log"; exit 1; }
    echo "tests under '$E': $(tail -1 "$OUT/pytest_$i.log")"
  fi
  echo "== setting $i: '${E:-defaults}'"
  env $E timeout -k 10 240 python -u tools/phase_timing.py "$SC" 3 > "$OUT/ab_$i.log" 2>&1 || { tail -20 "$OUT/ab_$i.log"; exit 1; }
  grep -E "^call 2" "$OUT/ab_$i.log"
  python -c "import ast,sys;d=ast.literal_eval(open('$OUT/ab_$i.log').read().strip().splitlines()[-1]);print({k:round(v['ms'],1) for k,v in d.items() if v['ms']})"
done
