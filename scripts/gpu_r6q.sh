set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6q
timeout -k 10 400 python -u scripts/gbm_automl_prof.py > gpurun_out/r6q/gbm_automl_prof.txt 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r6q/gbm_automl_prof.txt; exit 1; }
head -5 gpurun_out/r6q/gbm_automl_prof.txt
bash scripts/gpu_r6p.sh
