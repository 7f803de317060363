# session run r4t: C5 through the C++ overload, with the device memory state on OOM
set -o pipefail
OUT=gpurun_out/r4t; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) C5 cpp"
timeout -k 10 600 python -u bench_mcl.py --driver cpp > $OUT/bench_mcl_cpp.json 2> $OUT/bench_mcl_cpp.err || { tail -12 $OUT/bench_mcl_cpp.err; exit 1; }
cat $OUT/bench_mcl_cpp.json
echo "== $(date +%T) done"
