# session run r4q: generation-tagged owner maps (CBH_LIB=owngen): parity, A/B; stamps of the default
set -o pipefail
OUT=gpurun_out/r4q; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) pytest (CBH_LIB=owngen)"
CBH_LIB=owngen timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_regress_gpu.py tests/test_apps_gpu.py tests/test_scale22_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_owngen.log 2>&1 || { tail -40 $OUT/pytest_owngen.log; exit 1; }
tail -1 $OUT/pytest_owngen.log
echo "== $(date +%T) A/B"
bash tools/gpu_ab.sh r4q "" "CBH_LIB=owngen" "" "CBH_LIB=owngen" || exit 1
echo "== $(date +%T) stamps"
bash tools/gpu_stamps.sh r4q/st stamps 22 | grep -v entry-visits | tail -45
echo "== $(date +%T) done"
