#!/bin/bash
# C1's host download: copy-engine wait vs host-side conversion, with and without THP advice
set -o pipefail
OUT=gpurun_out/${1:-r6i}
mkdir -p $OUT
export LD_LIBRARY_PATH=/usr/lib/x86_64-linux-gnu:/opt/conda/lib
export OMP_NUM_THREADS=16
cat /sys/kernel/mm/transparent_hugepage/enabled > $OUT/thp.txt 2>&1
for v in "" "COMBBLAS_HIP_NO_THP=1" ""; do
  env $v CBH_XFER_DIAG=1 timeout -k 10 300 oracle/_ref/dropin_harness bench 16 5 > $OUT/c1.out 2> $OUT/c1.err || { tail -20 $OUT/c1.err; exit 1; }
  echo "[$v] $(grep BENCHC1 $OUT/c1.out | cut -c1-400)"
  grep "cbh xfer" $OUT/c1.err | tail -3
done
cat $OUT/thp.txt
