#!/bin/bash
# Round-2 measurement call: allocator tests, the default bench line (with the CPU baseline),
# rocprofv3 kernel stats of the bench, FETCH_SIZE calibration, per-bin PMC passes over one
# scale-22 product and over the merge sample.
#   gpurun -- bash tools/gpu_r2p.sh TAG
set -o pipefail
TAG=${1:-r2p}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R" || exit 1
step() { echo "== $(date +%T) $*"; }
step pytest allocator
timeout -k 10 400 python -u -m pytest tests/test_allocator_gpu.py tests/test_dist_gpu.py tests/test_spgemm_gpu.py -k "allocator or plan or dist or Trim or trim or poison or side_stream" -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_alloc.log" 2>&1 \
  || { tail -40 "$OUT/pytest_alloc.log"; exit 1; }
tail -2 "$OUT/pytest_alloc.log"
step bench default
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
cd /tmp || exit 1
step rocprof kernel stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-merge > "$OUT/prof_bench.json" 2> "$OUT/prof.log" \
  || { tail -20 "$OUT/prof.log"; exit 1; }
cat "$OUT/prof_bench.json"
step calibration
mkdir -p "$OUT/calib"
timeout -k 10 120 "$R/tools/bin/pmc_calib" > "$OUT/calib/calib.log" 2>&1 || { cat "$OUT/calib/calib.log"; exit 1; }
cat "$OUT/calib/calib.log"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$OUT/calib/pmc1" -o run -- \
  "$R/tools/bin/pmc_calib" > "$OUT/calib/pmc1.log" 2>&1 || { tail -20 "$OUT/calib/pmc1.log"; exit 1; }
python3 "$R/tools/pmc_calib.py" "$OUT/calib" "$OUT/pmc_calib.json" || exit 1
step phase timing
timeout -k 10 300 python3 -u "$R/tools/phase_timing.py" 22 2 > "$OUT/ks.log" 2>&1 || { tail -20 "$OUT/ks.log"; exit 1; }
tail -3 "$OUT/ks.log"
mkdir -p "$OUT/bins"
i=0
for PMC in "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  step "pmc pass $i: $PMC"
  timeout -s KILL 300 rocprofv3 --pmc $PMC --kernel-include-regex 'task_kernel' --output-format csv -d "$OUT/bins/pmc$i" -o run -- \
    python3 "$R/tools/phase_timing.py" 22 1 > "$OUT/bins/pmc$i.log" 2>&1 || { tail -20 "$OUT/bins/pmc$i.log"; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc $PMC --kernel-include-regex 'task_kernel.*true' --output-format csv -d "$OUT/bins/pmcm$i" -o run -- \
    python3 "$R/tools/merge_sample.py" 22 0.0625 1 > "$OUT/bins/pmcm$i.log" 2>&1 || { tail -20 "$OUT/bins/pmcm$i.log"; exit 1; }
done
python3 "$R/tools/pmc_bins.py" "$OUT/bins" "$OUT/ks.log" "$OUT/pmc_calib.json" "$OUT/pmc_bins.json"
step done
