set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6z
timeout -k 10 500 python -u scripts/algo_survey.py > gpurun_out/r6z/algo_survey.log 2>&1 || { echo "survey1 failed"; tail -20 gpurun_out/r6z/algo_survey.log; exit 1; }
grep "{" gpurun_out/r6z/algo_survey.log | cut -c1-160
timeout -k 10 600 python -u scripts/algo_survey2.py > gpurun_out/r6z/algo_survey2.log 2>&1 || { echo "survey2 failed"; tail -20 gpurun_out/r6z/algo_survey2.log; exit 1; }
grep "{" gpurun_out/r6z/algo_survey2.log | cut -c1-160
