# session run r4n: DPP wave scans (CBH_LIB=dscan): parity, then A/B
set -o pipefail
OUT=gpurun_out/r4n; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) pytest (CBH_LIB=dscan)"
CBH_LIB=dscan timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_regress_gpu.py tests/test_apps_gpu.py tests/test_scale22_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/pytest_dscan.log 2>&1 || { tail -40 $OUT/pytest_dscan.log; exit 1; }
tail -1 $OUT/pytest_dscan.log
echo "== $(date +%T) A/B"
bash tools/gpu_ab.sh r4n "" "CBH_LIB=dscan" "" "CBH_LIB=dscan" || exit 1
echo "== $(date +%T) done"
