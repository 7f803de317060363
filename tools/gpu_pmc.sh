#!/bin/bash
# HBM traffic of the dominant task kernels: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
# over one scale-SCALE product.  gpurun -- bash tools/gpu_pmc.sh TAG SCALE
# Then: python tools/pmc_traffic.py gpurun_out/TAG 'task_kernel<cbh::PlusTimesD<double>, 4096' profiles/pmc_num_large.json
set -e -o pipefail
TAG=${1:-pmc}
SCALE=${2:-22}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for PMC in "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "== pmc pass $i: $PMC"
  timeout -s KILL 240 rocprofv3 --pmc $PMC --kernel-include-regex 'task_kernel' --output-format csv -d "$OUT/pmc$i" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/phase_timing.py" "$SCALE" 1 > "$OUT/pmc$i.log" 2>&1 || { tail -20 "$OUT/pmc$i.log"; exit 1; }
done
echo done
