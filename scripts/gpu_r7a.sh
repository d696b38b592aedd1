set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7a
timeout -k 10 300 python -u scripts/prof_rulefit.py > gpurun_out/r7a/rulefit_prof.txt 2>&1 || { echo "rulefit prof failed"; tail -20 gpurun_out/r7a/rulefit_prof.txt; exit 1; }
head -3 gpurun_out/r7a/rulefit_prof.txt
