# session run r4g: A/B of the dense split ratio at 262144-flop tasks, C1, C5 (C++ and Python), stamps, tests
set -o pipefail
OUT=gpurun_out/r4g; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) A/B"
bash tools/gpu_ab.sh r4g "" "CBH_LIB=t256d6" "CBH_LIB=t256d7" "CBH_LIB=t256d8" "CBH_LIB=t256d10" || exit 1
echo "== $(date +%T) C1"
timeout -k 10 300 python -u bench_c1.py > $OUT/bench_c1.json 2> $OUT/bench_c1.err || { tail -20 $OUT/bench_c1.err; exit 1; }
cat $OUT/bench_c1.json
echo "== $(date +%T) C5 cpp"
timeout -k 10 600 python -u bench_mcl.py --driver cpp > $OUT/bench_mcl_cpp.json 2> $OUT/bench_mcl_cpp.err || { tail -30 $OUT/bench_mcl_cpp.err; cat $OUT/bench_mcl_cpp.json; exit 1; }
cat $OUT/bench_mcl_cpp.json
echo "== $(date +%T) stamps"
bash tools/gpu_stamps.sh r4g/st stamps 22 | tail -40
echo "== $(date +%T) pytest"
timeout -k 10 400 python -u -m pytest tests/test_devpath_gpu.py tests/test_allocator_gpu.py tests/test_regress_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
echo "== $(date +%T) done"
