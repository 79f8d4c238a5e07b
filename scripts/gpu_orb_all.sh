set -o pipefail
bash scripts/gpu_orb.sh && bash scripts/gpu_orb_bench.sh
