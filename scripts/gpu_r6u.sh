set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6u
true
true
timeout -k 10 170 python -u scripts/logit_hist_mb.py > gpurun_out/r6u/mb.txt 2>&1 || { echo "mb failed"; tail -20 gpurun_out/r6u/mb.txt; exit 1; }
cat gpurun_out/r6u/mb.txt
timeout -k 10 400 python -u scripts/gbm_automl_prof.py > gpurun_out/r6u/gbm_automl_prof.txt 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r6u/gbm_automl_prof.txt; exit 1; }
head -2 gpurun_out/r6u/gbm_automl_prof.txt
