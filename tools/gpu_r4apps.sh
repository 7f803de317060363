# session run r4apps: application lines on the final round-4 build (C1, C3, C4, C5 Python and C++)
set -o pipefail
OUT=gpurun_out/r4apps; mkdir -p $OUT; export TMPDIR=/tmp
for app in c1 galerkin tc mcl; do
  echo "== $(date +%T) bench_$app"
  timeout -k 10 600 python -u bench_$app.py > $OUT/bench_$app.json 2> $OUT/bench_$app.err || { tail -20 $OUT/bench_$app.err; exit 1; }
  cut -c1-300 $OUT/bench_$app.json
done
echo "== $(date +%T) bench_mcl cpp"
timeout -k 10 600 python -u bench_mcl.py --driver cpp > $OUT/bench_mcl_cpp.json 2> $OUT/bench_mcl_cpp.err || { tail -20 $OUT/bench_mcl_cpp.err; exit 1; }
cut -c1-300 $OUT/bench_mcl_cpp.json
echo "== $(date +%T) done"
