#!/bin/bash
# Kernel-phase ablations (diagnostic builds, wrong results, times only): the product library and
# each libcombblas_hip_<variant>.so run the same scale-SCALE product; kernel_ms per variant.
#   gpurun -- bash tools/gpu_ablate.sh TAG SCALE variant [variant ...]
set -e -o pipefail
TAG=${1:-abl}
SC=${2:-22}
shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for V in "" "$@"; do
  echo "== variant '${V:-product}'"
  CBH_LIB=$V timeout -k 10 240 python -u tools/phase_timing.py "$SC" 3 > "$OUT/abl_${V:-product}.log" 2>&1 \
    || { tail -20 "$OUT/abl_${V:-product}.log"; exit 1; }
  grep -E "^call|num_large|sym_large" "$OUT/abl_${V:-product}.log" | tail -2
done
