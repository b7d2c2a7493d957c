set -o pipefail
bash tools/gpu_quick.sh r04b || exit $?
bash tools/gpu_k1x.sh r04b_k1x 0 1 || exit $?
