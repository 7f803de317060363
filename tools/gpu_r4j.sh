# session run r4j: A/B of the hash table size, dense U and task size at the round-4 split; stamps
set -o pipefail
OUT=gpurun_out/r4j; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) A/B"
bash tools/gpu_ab.sh r4j "" "CBH_LIB=dp4" "CBH_LIB=h4k" "CBH_LIB=du4" "CBH_LIB=tf512k" "CBH_LIB=tf384k" || exit 1
echo "== $(date +%T) stamps"
bash tools/gpu_stamps.sh r4j/st stamps 22 | tail -60
echo "== $(date +%T) done"
