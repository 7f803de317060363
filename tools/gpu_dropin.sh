#!/bin/bash
mkdir -p gpurun_out/dropin
LD_LIBRARY_PATH=/usr/lib/x86_64-linux-gnu:/opt/conda/lib OMP_NUM_THREADS=8 timeout -k 5 60 oracle/_ref/dropin_harness ${1:-8} > gpurun_out/dropin/out.log 2>&1
echo "rc=$?"
cat gpurun_out/dropin/out.log
