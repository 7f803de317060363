#!/bin/bash
# round 6: multi-rank tests with the overlapped 3D schedule, a traced 1x1x2 rehearsal, and the
# per-sub-bin phase cycle shares of the stamps build at scale 22
set -o pipefail
OUT=gpurun_out/r6e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_devpath3d_gpu.py tests/test_bench_cpp_gpu.py tests/test_dropin3d_gpu.py -x -q --timeout 220 --timeout-method thread > $OUT/pytest_multirank.log 2>&1 || { tail -40 $OUT/pytest_multirank.log; exit 1; }
tail -1 $OUT/pytest_multirank.log
port=$((29500 + RANDOM % 1000))
COMBBLAS_HIP_TRACE=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
  --master-port $port bench.py --gpus 2 --steps 1 --warmup 0 --scale 16 --share-gpu --dist-backend gloo --driver cpp \
  --phases 3 > $OUT/trace_1x1x2.json 2> $OUT/trace_1x1x2.err || { tail -30 $OUT/trace_1x1x2.err; exit 1; }
grep "\[trace\] rank 0" $OUT/trace_1x1x2.err | head -40
CBH_LIB=stamps CBH_DIAG=1 timeout -k 10 300 python -u tools/phase_timing.py 22 2 > $OUT/stamps.log 2>&1 || { tail -30 $OUT/stamps.log; exit 1; }
grep -E "cbh stamps|call" $OUT/stamps.log | tail -40
