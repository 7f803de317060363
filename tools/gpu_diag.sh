#!/bin/bash
# Diagnostics on the GPU box: per-sub-bin kernel times (CBH_DIAG=1) and PMC passes on the
# dominant numeric kernel.  gpurun -- bash tools/gpu_diag.sh TAG SCALE
set -e -o pipefail
TAG=${1:-diag}
SCALE=${2:-20}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for PMC in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_FLAT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  echo "== pmc pass $i: $PMC"
  timeout -s KILL 240 rocprofv3 --pmc $PMC --kernel-include-regex 'task_kernel' --output-format csv -d "$OUT/pmc$i" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/phase_timing.py" "$SCALE" 1 > "$OUT/pmc$i.log" 2>&1 || { tail -20 "$OUT/pmc$i.log"; exit 1; }
done
echo done
