set -o pipefail
OUT=gpurun_out/r4d; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 180 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
echo "== $(date +%T) bench"
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-merge > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "== $(date +%T) C5 cpp"
timeout -k 10 600 python -u bench_mcl.py --driver cpp > $OUT/bench_mcl_cpp.json 2> $OUT/bench_mcl_cpp.err || { tail -30 $OUT/bench_mcl_cpp.err; cat $OUT/bench_mcl_cpp.json; exit 1; }
cat $OUT/bench_mcl_cpp.json
echo "== $(date +%T) C5 python"
timeout -k 10 600 python -u bench_mcl.py --no-cpu-baseline > $OUT/bench_mcl_py.json 2> $OUT/bench_mcl_py.err || { tail -30 $OUT/bench_mcl_py.err; exit 1; }
cat $OUT/bench_mcl_py.json
echo "== $(date +%T) done"
