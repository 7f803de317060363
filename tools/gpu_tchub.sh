#!/bin/bash
# TC dot form: hub groups vs the binary-search branch (CBH_DOT_HUB_MIN=0), parity tests first.
#   gpurun -- bash tools/gpu_tchub.sh TAG [extra bench_tc args]
set -o pipefail
TAG=${1:-tchub}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_apps_gpu.py "tests/test_fullsize_gpu.py::test_c4_tc_scale22_dot_vs_expand" \
  "tests/test_fullsize_gpu.py::test_c4_tc_scale24_dot" tests/test_regress_gpu.py -k "dot or tc" -x -q --timeout 180 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in ${VARIANTS:-"CBH_DOT_HUB_MIN=0" "CBH_DOT_HUB_MIN=16" "CBH_DOT_HUB_MIN=64"}; do
  env ${v//,/ } CBH_DIAG=1 timeout -k 10 300 python -u bench_tc.py --no-cpu-baseline --steps 2 "$@" > $OUT/tc_$v.json 2> $OUT/tc_$v.err \
    || { tail -20 $OUT/tc_$v.err; exit 1; }
  echo "[$v] $(python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['check']['ok'], d['check']['digest'])" $OUT/tc_$v.json)"
  grep "dot hub" $OUT/tc_$v.err | tail -1
done
if [ -n "$PROF" ]; then
  R=$PWD
  for v in ${PROFV:-0 16}; do
    (cd /tmp && CBH_DOT_HUB_MIN=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof$v" -o run -- \
      python3 "$R/bench_tc.py" --no-cpu-baseline --steps 1 --warmup 0 "$@" > "$R/$OUT/prof$v.log" 2>&1) || { tail -20 $OUT/prof$v.log; exit 1; }
    head -8 $OUT/prof$v/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
  done
fi
