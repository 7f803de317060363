# session run r4z: the pool over one reserved virtual address range with physical chunks mapped on
# demand (hipMemCreate / hipMemMap): allocator / device-path tests, C2 (allocator-backed A, B,
# bitmaps, scratch) and C5 through C++
set -o pipefail
OUT=gpurun_out/r4z; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) pytest"
timeout -k 10 700 python -u -m pytest tests/test_allocator_gpu.py tests/test_fallbacks_gpu.py tests/test_devpath3d_gpu.py tests/test_devpath_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
echo "== $(date +%T) C2"
for v in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c2_$v.json 2> $OUT/c2_$v.err || { tail -20 $OUT/c2_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/c2_$v.json')); k=d['config']['kernel_ms']; print('$v', d['value'], d['ms_per_step'], d['check']['ok'], 'dense', k['num_dense'], 'hash', k['num_large'], 'sym', k['sym_large'])"
done
echo "== $(date +%T) C5 cpp (memdiag)"
COMBBLAS_HIP_MEMDIAG=1 CBH_MEMDIAG=1 timeout -k 10 600 python -u bench_mcl.py --driver cpp > $OUT/bench_mcl_cpp.json 2> $OUT/bench_mcl_cpp.err
echo "rc=$?"; grep memdiag $OUT/bench_mcl_cpp.err | tail -30; grep -v memdiag $OUT/bench_mcl_cpp.err | tail -4; cut -c1-700 $OUT/bench_mcl_cpp.json
echo "== $(date +%T) done"
