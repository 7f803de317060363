# session run r4u: consuming concatenation near HBM capacity (probe)
set -o pipefail
OUT=gpurun_out/r4u; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/concat_mem_probe.py 148 5 18 > $OUT/probe.log 2>&1; echo rc=$?; cat $OUT/probe.log
