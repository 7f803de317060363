#!/bin/bash
# TC dot-form debug at scale 20/22, quick bench, per-phase stamps of the current build.
set -o pipefail
TAG=${1:-s2b}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
echo "== $(date +%T) bench (quick)"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
echo "== $(date +%T) stamps"
CBH_LIB=stamps CBH_DIAG=1 timeout -k 10 300 python -u tools/phase_timing.py 22 2 > "$OUT/stamps.log" 2>&1 || { tail -30 "$OUT/stamps.log"; exit 1; }
grep -E "cbh diag|cbh stamps|call" "$OUT/stamps.log" | tail -60
echo "== $(date +%T) TC debug"
timeout -k 10 400 python -u tools/tc_debug.py 20 22 > "$OUT/tcdebug.log" 2>&1 || { tail -20 "$OUT/tcdebug.log"; exit 1; }
cat "$OUT/tcdebug.log"
echo "== $(date +%T) done"
