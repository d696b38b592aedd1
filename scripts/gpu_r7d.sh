set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7d
timeout -k 10 900 python -u scripts/munging_survey.py > gpurun_out/r7d/munging_survey.log 2>&1 || { echo "munging survey failed"; tail -20 gpurun_out/r7d/munging_survey.log; exit 1; }
grep "{" gpurun_out/r7d/munging_survey.log | cut -c1-150
