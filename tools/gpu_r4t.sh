# session run r4t: C5 through the C++ overload with the memory milestones; re-tune A/B under DPP scans
set -o pipefail
OUT=gpurun_out/r4t; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) C5 cpp (memdiag)"
COMBBLAS_HIP_MEMDIAG=1 CBH_MEMDIAG=1 timeout -k 10 600 python -u bench_mcl.py --driver cpp > $OUT/bench_mcl_cpp.json 2> $OUT/bench_mcl_cpp.err
echo "rc=$?"; grep memdiag $OUT/bench_mcl_cpp.err | tail -40; tail -4 $OUT/bench_mcl_cpp.err; cat $OUT/bench_mcl_cpp.json
echo "== $(date +%T) A/B"
true
echo "== $(date +%T) done"
