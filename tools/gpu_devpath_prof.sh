#!/bin/bash
# rocprof trace (kernels + memory copies) of the device-resident SUMMA harness at 1 rank, and a
# probe of RCCL with 2 ranks on one GPU
set -o pipefail
mkdir -p gpurun_out/devprof
export LD_LIBRARY_PATH=/usr/lib/x86_64-linux-gnu:/opt/conda/lib TMPDIR=/tmp
OMP_NUM_THREADS=8 timeout -k 5 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/devprof/trace -o run -- oracle/_ref/devpath_harness ${1:-16} 3 > gpurun_out/devprof/prof.log 2>&1; rc=$?
grep DEVPATH gpurun_out/devprof/prof.log; echo "prof rc=$rc"
find gpurun_out/devprof/trace -name "*stats*.csv" | head


exit 0
