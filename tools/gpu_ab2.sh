#!/bin/bash
# bench A/B of library variants (no tests): product vs each CBH_LIB variant given
#   gpurun -- bash tools/gpu_ab2.sh TAG VARIANT [VARIANT ...]
set -e -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify > "$OUT/bench_base.json" 2> "$OUT/bench_base.err" || { tail -20 "$OUT/bench_base.err"; exit 1; }
cat "$OUT/bench_base.json"
for v in "$@"; do
  CBH_LIB=$v timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || { tail -20 "$OUT/bench_$v.err"; exit 1; }
  cat "$OUT/bench_$v.json"
done
