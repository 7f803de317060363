#!/bin/bash
# Distributed path on a one-GPU box: dist GPU tests (ranks share cuda:0, gloo staging), then
# bench rehearsals at N=4 (2D 2x2) and N=2 / N=8 (3D) with --share-gpu --dist-backend gloo.
#   gpurun -- bash tools/gpu_dist.sh TAG [SCALE]
set -e -o pipefail
TAG=${1:-dist}
SC=${2:-18}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_dist.log" 2>&1 \
  || { tail -60 "$OUT/pytest_dist.log"; exit 1; }
tail -3 "$OUT/pytest_dist.log"
for N in 4 2 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500+N)) \
    bench.py --gpus $N --steps 1 --warmup 1 --scale $SC --dist-backend gloo --share-gpu --no-cpu-baseline > "$OUT/bench$N.json" 2> "$OUT/bench$N.err" \
    || { tail -40 "$OUT/bench$N.err"; exit 1; }
  cat "$OUT/bench$N.json"
done
