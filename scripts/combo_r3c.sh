set -e
bash scripts/gpu_round_check.sh
bash scripts/prof_slow_algos.sh
