set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7q
timeout -k 10 400 python -u scripts/dl_automl_prof.py > gpurun_out/r7q/dl_automl_prof.txt 2>&1 || { echo "dl prof failed"; tail -20 gpurun_out/r7q/dl_automl_prof.txt; exit 1; }
head -2 gpurun_out/r7q/dl_automl_prof.txt
