# session run r4cap: C5 through C++ with the block cache cap raised to 290 GB (default 0.85 x 309 GB)
set -o pipefail
OUT=gpurun_out/r4cap; mkdir -p $OUT; export TMPDIR=/tmp
for cap in 290 275; do
  echo "== $(date +%T) cap $cap"
  CBH_CACHE_CAP_GB=$cap COMBBLAS_HIP_MEMDIAG=1 timeout -k 10 600 python -u bench_mcl.py --driver cpp --no-cpu-baseline > $OUT/cpp_$cap.json 2> $OUT/cpp_$cap.err || { grep -v memdiag $OUT/cpp_$cap.err | tail -8; exit 1; }
  cut -c1-260 $OUT/cpp_$cap.json; grep "memdiag" $OUT/cpp_$cap.err | tail -24 | cut -c1-130
done
echo "== $(date +%T) done"
