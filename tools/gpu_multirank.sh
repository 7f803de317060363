#!/bin/bash
# Rehearsal of bench.py's N-GPU line on a one-GPU box: torch.distributed.run starts N bench.py
# ranks (gloo, no GPU use), rank 0 runs the C++ host path under mpirun (every MPI rank on cuda:0,
# exchanges staged through host MPI: COMBBLAS_HIP_COMM=mpi via --share-gpu).
#   gpurun --timeout 900 -- bash tools/gpu_multirank.sh TAG SCALE "2 4 8" [DRIVER]
set -o pipefail
TAG=${1:-mr}
SCALE=${2:-18}
NS=${3:-"2 4"}
DRIVER=${4:-cpp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
port=29600
for n in $NS; do
  echo "== $(date +%T) N=$n scale $SCALE driver $DRIVER"
  port=$((port + 1))
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus "$n" --steps 3 --warmup 1 --scale "$SCALE" --share-gpu --dist-backend gloo \
    --driver "$DRIVER" > "$OUT/n$n.json" 2> "$OUT/n$n.err" || { tail -30 "$OUT/n$n.err"; exit 1; }
  cat "$OUT/n$n.json"
done
echo "== $(date +%T) done"
