# session run r4y: splitting pool for blocks >= 16 MiB (allocator / device-path tests, C5 through
# C++); dense window ends snapped to absolute row blocks (A/B against the relative snap); dense
# windows in a 8192-slot table's LDS (one group per CU), U 8 / 16
set -o pipefail
OUT=gpurun_out/r4y; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) preflight"
timeout -k 10 180 python -c "import torch; print('torch sees', torch.cuda.device_count(), 'devices, available', torch.cuda.is_available())" || exit 1
echo "== $(date +%T) pytest"
timeout -k 10 700 python -u -m pytest tests/test_allocator_gpu.py tests/test_fallbacks_gpu.py tests/test_devpath3d_gpu.py tests/test_devpath_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
echo "== $(date +%T) A/B dense snap / dense window LDS"
for v in abs relsnap d8k d8k16 abs relsnap d8k d8k16; do
  if [ $v = abs ]; then unset CBH_LIB; else export CBH_LIB=$v; fi
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/ab_$v.json 2> $OUT/ab_$v.err || { tail -20 $OUT/ab_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/ab_$v.json')); k=d['config']['kernel_ms']; print('$v', d['value'], d['check']['ok'], 'dense', k['num_dense'], 'hash', k['num_large'], 'sym', k['sym_large'])"
done
unset CBH_LIB
echo "== $(date +%T) C5 cpp (memdiag)"
COMBBLAS_HIP_MEMDIAG=1 timeout -k 10 600 python -u bench_mcl.py --driver cpp > $OUT/bench_mcl_cpp.json 2> $OUT/bench_mcl_cpp.err
echo "rc=$?"; grep memdiag $OUT/bench_mcl_cpp.err | tail -24; tail -4 $OUT/bench_mcl_cpp.err; cut -c1-600 $OUT/bench_mcl_cpp.json
echo "== $(date +%T) done"
