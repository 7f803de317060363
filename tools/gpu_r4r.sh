# session run r4r: fewer barriers per sub-tile (CBH_LIB=fewbar): parity, A/B
set -o pipefail
OUT=gpurun_out/r4r; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) pytest (CBH_LIB=fewbar)"
CBH_LIB=fewbar timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_regress_gpu.py tests/test_apps_gpu.py tests/test_scale22_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_fewbar.log 2>&1 || { tail -40 $OUT/pytest_fewbar.log; exit 1; }
tail -1 $OUT/pytest_fewbar.log
echo "== $(date +%T) A/B"
bash tools/gpu_ab.sh r4r "" "CBH_LIB=fewbar" "" "CBH_LIB=fewbar" || exit 1
echo "== $(date +%T) done"
