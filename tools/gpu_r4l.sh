# session run r4l: run-aligned commit batches (CBH_LIB=ra): parity, then A/B
set -o pipefail
OUT=gpurun_out/r4l; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) pytest (CBH_LIB=ra)"
CBH_LIB=ra timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_regress_gpu.py tests/test_scale22_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/pytest_ra.log 2>&1 || { tail -40 $OUT/pytest_ra.log; exit 1; }
tail -1 $OUT/pytest_ra.log
echo "== $(date +%T) A/B"
bash tools/gpu_ab.sh r4l "" "CBH_LIB=ra" "" "CBH_LIB=ra" || exit 1
echo "== $(date +%T) done"
