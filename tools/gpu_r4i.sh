# session run r4i: C1 drop-in, C5 through the C++ overload, then the application lines (C5, C3, C4)
set -o pipefail
OUT=gpurun_out/r4i; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) C1"
timeout -k 10 300 python -u bench_c1.py > $OUT/bench_c1.json 2> $OUT/bench_c1.err || { tail -20 $OUT/bench_c1.err; exit 1; }
cat $OUT/bench_c1.json
echo "== $(date +%T) C5 cpp"
timeout -k 10 600 python -u bench_mcl.py --driver cpp > $OUT/bench_mcl_cpp.json 2> $OUT/bench_mcl_cpp.err || { tail -30 $OUT/bench_mcl_cpp.err; cat $OUT/bench_mcl_cpp.json; exit 1; }
cat $OUT/bench_mcl_cpp.json
PART=2 bash tools/gpu_final.sh r4i
