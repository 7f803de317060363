# session run r4s: re-tune under the DPP-scan build: dense split 6/4, 8/4; symbolic U 8; 393216-flop tasks
set -o pipefail
OUT=gpurun_out/r4s; mkdir -p $OUT; export TMPDIR=/tmp
echo "== $(date +%T) A/B"
bash tools/gpu_ab.sh r4s "" "CBH_LIB=d6" "CBH_LIB=d8" "CBH_LIB=su8" "CBH_LIB=t384" "" "CBH_LIB=d6" "CBH_LIB=d8" "CBH_LIB=su8" "CBH_LIB=t384" || exit 1
echo "== $(date +%T) done"
