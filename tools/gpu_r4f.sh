# session run r4f: the ordered-insertion hash variant's parity, then A/B of the queued variants
set -o pipefail
OUT=gpurun_out/r4f; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) pytest (CBH_LIB=ord)"
CBH_LIB=ord timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_regress_gpu.py tests/test_f64_rounding_gpu.py tests/test_scale22_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_ord.log 2>&1 || { tail -60 $OUT/pytest_ord.log; exit 1; }
tail -2 $OUT/pytest_ord.log
echo "== $(date +%T) A/B"
bash tools/gpu_ab.sh r4f "" "CBH_LIB=ord" "CBH_LIB=dpp" "CBH_LIB=e256" "CBH_LIB=d2k" "CBH_LIB=d2ku8" "CBH_LIB=tf64k" "CBH_LIB=tf256k" "CBH_LIB=dr4" "CBH_LIB=dr7" || exit 1
echo "== $(date +%T) stamps (ord)"
bash tools/gpu_stamps.sh r4f/st ordstamps 22
echo "== $(date +%T) done"
