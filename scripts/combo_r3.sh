set -e
bash scripts/gpu_round_check.sh
bash scripts/cat_pair_ab.sh
