set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/automl_r6d
ROWS=10000000 COLS=200 BUDGET=840 NSCORE=100000 OUT=gpurun_out/automl_r6d \
  timeout -k 10 1120 python -u scripts/automl_baseline.py > gpurun_out/automl_r6d/run.log 2>&1
echo "automl rc=$?"
tail -5 gpurun_out/automl_r6d/run.log
