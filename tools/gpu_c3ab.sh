#!/bin/bash
# C3 A/B of library variants (verified against the oracle digest and the closed-form sum)
#   gpurun --timeout 600 -- bash tools/gpu_c3ab.sh TAG VARIANT [VARIANT ...]
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT" || exit 1
for v in base "$@"; do
  if [ "$v" = base ]; then L=""; else L=$v; fi
  echo "== $(date +%T) C3 $v"
  CBH_LIB=$L timeout -k 10 300 python -u bench_galerkin.py > "$OUT/gal_$v.json" 2> "$OUT/gal_$v.err" || { tail -20 "$OUT/gal_$v.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/gal_$v.json')); print(d['value'], d['ms_per_step'], d['check']['ok'])"
done
echo "== $(date +%T) done"
