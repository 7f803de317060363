# session run r4rel: cache cap 0.9 of the device and partial release before RCCL setup: allocator,
# fallbacks and device-path tests, then C5 through C++ with the defaults
set -o pipefail
OUT=gpurun_out/r4rel; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) pytest"
timeout -k 10 700 python -u -m pytest tests/test_allocator_gpu.py tests/test_fallbacks_gpu.py tests/test_devpath3d_gpu.py tests/test_devpath_gpu.py tests/test_dropin_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
echo "== $(date +%T) C5 cpp"
COMBBLAS_HIP_MEMDIAG=1 timeout -k 10 600 python -u bench_mcl.py --driver cpp > $OUT/bench_mcl_cpp.json 2> $OUT/bench_mcl_cpp.err || { grep -v memdiag $OUT/bench_mcl_cpp.err | tail -8; exit 1; }
cut -c1-300 $OUT/bench_mcl_cpp.json; grep "memdiag\] \(MemEff\|stage plans\|phase loop\|step\)" $OUT/bench_mcl_cpp.err | cut -c1-140
echo "== $(date +%T) done"
