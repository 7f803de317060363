#!/bin/bash
# Per-bin PMC passes (one scale-SCALE product + the merge sample) and, with STAMPS=1, the stamps
# build's per-phase cycle shares of the same product.   gpurun -- bash tools/gpu_bins.sh TAG [SCALE]
set -o pipefail
TAG=${1:-bins}
SCALE=${2:-22}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT/bins"
export TMPDIR=/tmp
cd /tmp || exit 1
step() { echo "== $(date +%T) $*"; }
step phase timing
timeout -k 10 300 python3 -u "$R/tools/phase_timing.py" "$SCALE" 2 > "$OUT/ks.log" 2>&1 || { tail -20 "$OUT/ks.log"; exit 1; }
tail -3 "$OUT/ks.log"
i=0
for PMC in "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  step "pmc pass $i: $PMC"
  timeout -s KILL 300 rocprofv3 --pmc $PMC --kernel-include-regex 'task_kernel|dense_kernel' --output-format csv -d "$OUT/bins/pmc$i" -o run -- \
    python3 "$R/tools/phase_timing.py" "$SCALE" 1 > "$OUT/bins/pmc$i.log" 2>&1 || { tail -20 "$OUT/bins/pmc$i.log"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc $PMC --kernel-include-regex 'task_kernel.*true|merge2_kernel' --output-format csv -d "$OUT/bins/pmcm$i" -o run -- \
    python3 "$R/tools/merge_sample.py" "$SCALE" 0.0625 1 > "$OUT/bins/pmcm$i.log" 2>&1 || { tail -20 "$OUT/bins/pmcm$i.log"; exit 1; }
done
python3 "$R/tools/pmc_bins.py" "$OUT/bins" "$OUT/ks.log" "$R/profiles/pmc_calib.json" "$OUT/pmc_bins.json"
if [ "${STAMPS:-0}" = 1 ]; then
  step stamps
  cd "$R" || exit 1
  CBH_LIB=stamps CBH_DIAG=1 timeout -k 10 300 python -u tools/phase_timing.py "$SCALE" 2 > "$OUT/stamps.log" 2>&1 || { tail -30 "$OUT/stamps.log"; exit 1; }
  grep -E "cbh stamps|call" "$OUT/stamps.log" | tail -40
fi
step done
