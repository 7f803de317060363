# session run r4o: DPP neighbours/totals (CBH_LIB=dpp2) and the dense/hash two-stream overlap
# (CBH_LIB=ovl): parity of each, then A/B against the DPP-scan default
set -o pipefail
OUT=gpurun_out/r4o; mkdir -p $OUT; export TMPDIR=/tmp
for v in dpp2 ovl; do
  echo "== $(date +%T) pytest (CBH_LIB=$v)"
  CBH_LIB=$v timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_regress_gpu.py tests/test_apps_gpu.py tests/test_scale22_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { tail -40 $OUT/pytest_$v.log; exit 1; }
  tail -1 $OUT/pytest_$v.log
done
echo "== $(date +%T) A/B"
bash tools/gpu_ab.sh r4o "" "CBH_LIB=dpp2" "CBH_LIB=ovl" "" "CBH_LIB=dpp2" "CBH_LIB=ovl" || exit 1
echo "== $(date +%T) done"
