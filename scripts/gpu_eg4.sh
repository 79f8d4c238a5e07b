set -o pipefail
bash scripts/gpu_eg3.sh && bash scripts/gpu_egprof.sh
