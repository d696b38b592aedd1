set -e
bash scripts/gpu_round_check.sh
export TMPDIR=/tmp
ALGO=rulefit timeout -k 10 300 python -u scripts/prof_rulefit.py > gpurun_out/prof_rulefit_cd.log 2>&1
grep train_s gpurun_out/prof_rulefit_cd.log
