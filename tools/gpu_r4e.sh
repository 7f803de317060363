# session run r4e: drop-in / allocator / regression tests, C1, C5 (C++ and Python), A/B of task size and dense split
set -o pipefail
OUT=gpurun_out/r4e; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests/test_devpath_gpu.py tests/test_allocator_gpu.py tests/test_regress_gpu.py tests/test_dropin_gpu.py -m gpu -x -v -rP --timeout 180 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
echo "== $(date +%T) C1"
timeout -k 10 300 python -u bench_c1.py > $OUT/bench_c1.json 2> $OUT/bench_c1.err || { tail -20 $OUT/bench_c1.err; exit 1; }
cat $OUT/bench_c1.json
echo "== $(date +%T) C5 cpp"
timeout -k 10 600 python -u bench_mcl.py --driver cpp > $OUT/bench_mcl_cpp.json 2> $OUT/bench_mcl_cpp.err || { tail -30 $OUT/bench_mcl_cpp.err; cat $OUT/bench_mcl_cpp.json; exit 1; }
cat $OUT/bench_mcl_cpp.json
echo "== $(date +%T) C5 python"
timeout -k 10 600 python -u bench_mcl.py --no-cpu-baseline > $OUT/bench_mcl_py.json 2> $OUT/bench_mcl_py.err || { tail -30 $OUT/bench_mcl_py.err; exit 1; }
cat $OUT/bench_mcl_py.json
echo "== $(date +%T) A/B"
bash tools/gpu_ab.sh r4e "" "CBH_LIB=dpp" "CBH_LIB=tf64k" "CBH_LIB=tf256k" "CBH_LIB=dr4" "CBH_LIB=dr7" "CBH_LIB=e256" "CBH_LIB=e256u2" "CBH_LIB=d2k" "CBH_LIB=d2ku8"
echo "== $(date +%T) stamps"
bash tools/gpu_stamps.sh r4e/st stamps 22
echo "== $(date +%T) done"
