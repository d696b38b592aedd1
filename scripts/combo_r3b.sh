set -e
bash scripts/gpu_round_check.sh
bash scripts/algo_survey2.sh
