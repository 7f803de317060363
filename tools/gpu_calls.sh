#!/bin/bash
# phased product NCALLS times at one scale (first-call vs steady state), optional diag/variant env
#   gpurun -- bash tools/gpu_calls.sh TAG SCALE NCALLS [ENV=VAL ...]
set -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
S=$2; N=$3; shift 3
env "$@" timeout -k 5 240 python -u tools/phase_timing.py $S $N > "$OUT/calls.log" 2>&1
rc=$?
grep -E "call|cbh diag|stamps" "$OUT/calls.log" | tail -80
echo "rc=$rc"
