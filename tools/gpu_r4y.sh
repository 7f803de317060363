# session run r4y: splitting pool for blocks >= 16 MiB: allocator / device-path tests, then C5 through C++
set -o pipefail
OUT=gpurun_out/r4y; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) pytest"
timeout -k 10 700 python -u -m pytest tests/test_allocator_gpu.py tests/test_fallbacks_gpu.py tests/test_devpath3d_gpu.py tests/test_devpath_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
echo "== $(date +%T) C5 cpp (memdiag)"
COMBBLAS_HIP_MEMDIAG=1 timeout -k 10 600 python -u bench_mcl.py --driver cpp > $OUT/bench_mcl_cpp.json 2> $OUT/bench_mcl_cpp.err
echo "rc=$?"; grep memdiag $OUT/bench_mcl_cpp.err | tail -24; tail -4 $OUT/bench_mcl_cpp.err; cut -c1-600 $OUT/bench_mcl_cpp.json
echo "== $(date +%T) done"
