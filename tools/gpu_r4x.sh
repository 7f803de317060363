# session run r4x: C5 (Python driver) on round 3's generator (torch) for a like-for-like comparison
set -o pipefail
OUT=gpurun_out/r4x; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u bench_mcl.py --gen torch --no-cpu-baseline > $OUT/bench_mcl_torch.json 2> $OUT/bench_mcl_torch.err || { tail -20 $OUT/bench_mcl_torch.err; exit 1; }
cut -c1-900 $OUT/bench_mcl_torch.json
