#!/bin/bash
# device-resident SUMMA harness: 1 rank over RCCL, 4 ranks sharing the GPU (host-staged MPI)
set -o pipefail
mkdir -p gpurun_out/devpath
export LD_LIBRARY_PATH=/usr/lib/x86_64-linux-gnu:/opt/conda/lib
S=${1:-12}
OMP_NUM_THREADS=8 timeout -k 5 120 oracle/_ref/devpath_harness $S 3 > gpurun_out/devpath/np1.log 2>&1; rc=$?
cat gpurun_out/devpath/np1.log | grep -v "^graph" ; echo "np1 rc=$rc"
[ $rc -ne 0 ] && exit $rc
COMBBLAS_HIP_COMM=mpi OMP_NUM_THREADS=2 timeout -k 5 150 /opt/conda/bin/mpirun -np 4 oracle/_ref/devpath_harness $S 2 > gpurun_out/devpath/np4.log 2>&1; rc=$?
cat gpurun_out/devpath/np4.log | grep -v "^graph"; echo "np4 rc=$rc"
exit $rc
