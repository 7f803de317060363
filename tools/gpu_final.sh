set -e -o pipefail
bash tools/gpu_round.sh r01g 3
bash tools/gpu_pmc.sh pmc22g 22
